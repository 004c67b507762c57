"""Multi-process Z-slab path on CPU (gloo, world sizes 2 and 3): sdfgenfast_amd.distributed.

The same slab split, plane hand-off order and gather as the GPU ranks use; the planes
travel with send/recv over gloo.  Bit-exact against the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as tmp

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import meshgen


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dims, result_path):
    import torch.distributed as dist
    from sdfgenfast_amd import distributed as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        v, t = meshgen.bumpy_sphere(40, 17)
        o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)
        phi, kb, ke = D.make_level_set3(v, t, o, dx, *dims, 1, backend="cpu", gather_to=0)
        assert (kb, ke) == ((0, dims[2]) if rank == 0 else D.slab_range(dims[2], world, rank))
        phi2, kb2, ke2 = D.make_level_set3(v, t, o, dx, *dims, 1, backend="cpu", gather_to=None)
        assert (kb2, ke2) == D.slab_range(dims[2], world, rank) and phi2.shape == (dims[0], dims[1], ke2 - kb2)
        if rank == 0:
            np.save(result_path, np.asfortranarray(phi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dims", [(2, (20, 18, 22)), (3, (17, 21, 15)), (2, (9, 12, 4))])
def test_cpu_slabs_over_gloo_match_oracle(tmp_path, world, dims):
    path = str(tmp_path / "phi.npy")
    tmp.spawn(_worker, args=(world, _free_port(), dims, path), nprocs=world, join=True)
    v, t = meshgen.bumpy_sphere(40, 17)
    o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, *dims, 1))
    got = np.load(path)
    assert got.shape == tuple(dims)
    assert bits_equal(got, want), diff_report(got, want, dx)


def _subgroup_worker(rank, world, port, dims, result_path):
    """3 processes; ranks 1 and 2 form a gloo subgroup and split the grid between them
    (group-local ranks 0 and 1); rank 0 takes no part."""
    import torch.distributed as dist
    from sdfgenfast_amd import distributed as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sub = dist.new_group(ranks=[1, 2], backend="gloo")   # collective over the whole world
        if rank in (1, 2):
            v, t = meshgen.bumpy_sphere(40, 17)
            o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)
            phi, kb, ke = D.make_level_set3(v, t, o, dx, *dims, 1, backend="cpu", group=sub, gather_to=1)
            if rank == 2:   # group rank 1 holds the gathered grid
                assert (kb, ke) == (0, dims[2])
                np.save(result_path, np.asfortranarray(phi))
            else:
                assert (kb, ke) == D.slab_range(dims[2], 2, 0)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_cpu_slabs_on_a_subgroup(tmp_path):
    """A 2-of-3-rank subgroup: group-local ranks, neighbours and gather target map to the
    right global ranks."""
    dims = (16, 14, 18)
    path = str(tmp_path / "phi.npy")
    tmp.spawn(_subgroup_worker, args=(3, _free_port(), dims, path), nprocs=3, join=True)
    v, t = meshgen.bumpy_sphere(40, 17)
    o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, *dims, 1))
    got = np.load(path)
    assert bits_equal(got, want), diff_report(got, want, dx)


def test_cpu_slab_session_single_process_chain():
    """Drive all slabs of a grid from one process, handing the planes on by hand."""
    from sdfgenfast_amd import _lib
    dims = (15, 13, 11)
    v, t = meshgen.bumpy_sphere(30, 13)
    o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)
    n = 3
    slabs = [_lib.CpuSlab(n, s, *dims) for s in range(n)]
    for sl in slabs:
        sl.band(v, t, o, dx, 1)
    for s in range(16):
        order = range(n) if slabs[0].upstream_is_below(s) else range(n - 1, -1, -1)
        plane = None
        for r in order:
            last = r == (n - 1 if slabs[0].upstream_is_below(s) else 0)
            plane = slabs[r].sweep(s, plane, not last)
    got = np.concatenate([sl.sign().ravel(order="F") for sl in slabs]).reshape(dims, order="F")
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, *dims, 1))
    assert bits_equal(got, want), diff_report(got, want, dx)
    with pytest.raises(ValueError):
        slabs[1].sweep(0, None, True)   # a middle slab needs its upstream plane


def test_slab_range_partition():
    from sdfgenfast_amd.distributed import slab_range
    for nk, w in [(256, 8), (29, 3), (10, 4), (512, 7)]:
        rs = [slab_range(nk, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == nk
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        assert all(e - b >= nk // w for b, e in rs)
