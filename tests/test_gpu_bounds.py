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


@pytest.mark.parametrize("mode", ["hybrid", "sparse", "sparse-2buf", "sparse-brick"])
def test_bounds_one_gpu_sweep_paths(mode):
    """The one-GPU sweep paths on the bounds build: the tile first pass and every second-pass repair
    variant (in place, two buffers, brick-owned), all 16 sweeps sparse where named -- every index the
    kernels form is checked, and the result must still match the oracle bit for bit."""
    env = {"hybrid": {}, "sparse": {"SDFGEN_SPARSE_FROM": "0"},
           "sparse-2buf": {"SDFGEN_SPARSE_FROM": "0", "SDFGEN_SPARSE_INPLACE": "0"},
           "sparse-brick": {"SDFGEN_SPARSE_FROM": "0", "SDFGEN_SPARSE_BRICK": "1"}}[mode]
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import numpy as np\n"
        "from oracle import oracle as O\n"
        "from sdfgenfast_amd import _lib, meshgen\n"
        "v, t = meshgen.bumpy_sphere(90, 31); dims = (57, 33, 70)\n"
        "o, dx = meshgen.grid_mode2b(v, *dims, 2)\n"
        "want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))\n"
        "got = _lib.make_level_set3(v, t, o, dx, *dims, 1)\n"
        "print('OK' if np.array_equal(got.view(np.uint32), want.view(np.uint32)) else 'MISMATCH', _lib.LIB_PATH)\n"
    ) % (ROOT, os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], env=_env(**env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.stdout.split()[0] == "OK" and r.stdout.split()[1] == BOUNDS_LIB, r.stdout


def test_bounds_band_sign_prep_kernels():
    """k_prep_soup, k_band_lds, k_band_big, the ray-parity counts, k_sign and k_sign_kfast on the bounds
    build (SDF_CHK sites 40-50): the golden and edge fixtures' stage 1 against oracle.band and their whole
    calls in both layouts against the reference's output, plus coarse soups through the big-triangle list.
    A wrong pair -> triangle search (the round-5 half-wave ballot build) now fails as a named site here,
    not as a GPU fault that surfaces later as a failed allocation."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "band_bounds_check.py")], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert last[0] == "OK" and last[1] == BOUNDS_LIB, r.stdout[-3000:]
