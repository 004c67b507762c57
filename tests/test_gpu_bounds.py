"""The Z-slab paths on the bounds-checked library (make BOUNDS=1 -> libsdfgen_hip_bounds.so,
geom.hpp SDF_CHK): every global index the sweep kernels form is checked against the buffer it
addresses, and the first violation is reported as an error instead of faulting the GPU.

Regression guard for the round-2 fault of commit ab6d4a7: the branch-free request atomics sent a
no-target slot's `atomicAdd(..., 0)` to the requesting cell's counter, which for an inbound-ring
entry belongs to the upstream slab -- an out-of-range address on the slab's own buffer.  The GPU
suite ran no slab test at an address that faulted; on this build any grid reports it
(site 24, sweep_sparse.hpp).  Runs the 2-slab in-process path and the one-process-per-slab IPC
path (bench.py under torch.distributed.run) at C2 size, each checked against the reference digest.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_LIB = os.path.join(ROOT, "sdfgenfast_amd", "libsdfgen_hip_bounds.so")


def setup_module(_):
    assert os.path.exists(BOUNDS_LIB), f"{BOUNDS_LIB} missing: __graft_entry__.build() makes it (make BOUNDS=1)"


def _env(**kw):
    return dict(os.environ, SDFGEN_LIB_OVERRIDE=BOUNDS_LIB, HSA_ENABLE_IPC_MODE_LEGACY="0", **kw)


def test_bounds_library_is_the_checked_build():
    """The override really loads the bounds build (a different build identity)."""
    code = ("import sys; sys.path.insert(0, %r); from sdfgenfast_amd import _lib; "
            "print(_lib.LIB_PATH, _lib.build_id())" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    path, bid = out.stdout.split()
    assert path == BOUNDS_LIB
    plain = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sdfgenfast_amd"), "build-id"],
                           capture_output=True, text=True).stdout.strip()
    assert bid != plain


@pytest.mark.parametrize("what", [("2", "40", "36", "44"), ("2", "c2_sphere70k_128", "2")])
def test_bounds_two_slabs_in_process(what):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "slab_inprocess_check.py"), *what],
                       env=_env(GPU_MAX_HW_QUEUES="8", SDFGEN_TILE_GRID="96"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "libsdfgen_hip_bounds.so" in r.stdout


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bounds_two_ranks_ipc_zslab():
    """One process per slab, inboxes / halo planes / inbound rings mapped over HIP IPC: the path
    of the ab6d4a7 fault (inbound-ring entries turned into recheck requests)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--workload", "c2_sphere70k_128", "--mode", "zslab",
           "--no-side", "--no-latency", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=_env(SDFGEN_TILE_GRID="64"), capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert "zslab_error" not in res, res.get("zslab_error")
    assert res["config"]["parallelism"] == "zslab2", res
    assert res["parity"] == "bit-exact vs reference (sha256 of phi)", res
