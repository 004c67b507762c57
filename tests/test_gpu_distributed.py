"""sdfgenfast_amd.distributed on the GPU: 2 ranks (torch.distributed, gloo control plane) on
the box's one GPU, inboxes mapped over HIP IPC; and bench.py's multi-rank mode."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as tmp

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import meshgen

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dims, result_path):
    os.environ["SDFGEN_TILE_GRID"] = "64"   # both ranks share one GPU here: keep both resident
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from sdfgenfast_amd import distributed as D
    try:
        v, t = meshgen.bumpy_sphere(90, 31)
        o, dx = meshgen.grid_mode2b(v, *dims, 2)
        for _ in range(2):   # second call reuses the mapped sessions
            phi, kb, ke = D.make_level_set3(v, t, o, dx, *dims, 1, backend="gpu", device=0, gather_to=0)
        if rank == 0:
            np.save(result_path, np.asfortranarray(phi))
        dist.barrier()
        D.release()
        if rank == 0:
            # a one-GPU call after release() in a process that held IPC imports of the peer's blocks (ADVICE
            # r05: release keeps those mappings and the block pool, so no later allocation lands on them)
            from sdfgenfast_amd import _lib
            _lib.release()
            np.save(result_path + ".after.npy",
                    np.asfortranarray(_lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dims", [(40, 36, 44), (30, 50, 21)])
def test_distributed_gpu_two_ranks_match_oracle(tmp_path, dims):
    path = str(tmp_path / "phi.npy")
    tmp.spawn(_worker, args=(2, _free_port(), dims, path), nprocs=2, join=True)
    v, t = meshgen.bumpy_sphere(90, 31)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, *dims, 1))
    got = np.load(path)
    assert bits_equal(got, want), diff_report(got, want, dx)
    after = np.load(path + ".after.npy")
    assert bits_equal(after, want), "one-GPU call after release: " + diff_report(after, want, dx)


def _bench_two_ranks(*extra):
    env = dict(os.environ, SDFGEN_TILE_GRID="64", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--workload", "c2_sphere70k_128", *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    import json
    return json.loads(line)


def test_bench_two_ranks_zslab_parity():
    """bench.py --mode zslab under torch.distributed.run, 2 ranks on one GPU: bit-exact headline."""
    res = _bench_two_ranks("--mode", "zslab", "--no-side")
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "zslab2" and res["scaling"] == "strong", res
    assert res["parity"] == "bit-exact vs reference (sha256 of phi)", res
    assert "zslab_c4" not in res and "zslab_error" not in res
    assert res["efficiency"] > 0 and res["sweep_impl"] == 2


def test_bench_two_ranks_default_line():
    """Default N > 1 line: Z-slab headline with its efficiency, the second grid's Z-slab run and
    the replicas run as side objects; every one bit-exact."""
    res = _bench_two_ranks("--c4-workload", "c2_sphere70k_128")
    assert res["config"]["parallelism"] == "zslab2" and res["scaling"] == "strong", res
    assert res["parity"] == "bit-exact vs reference (sha256 of phi)", res
    zs = res["zslab_c4"]
    assert "error" not in zs, zs
    assert zs["parallelism"] == "zslab2" and zs["parity"] == "bit-exact vs reference (sha256 of phi)", zs
    assert zs["efficiency"] > 0
    rep = res["replicas"]
    assert rep["parallelism"] == "replicas2" and rep["parity"] == "bit-exact vs reference (sha256 of phi)", rep
