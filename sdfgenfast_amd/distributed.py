"""Z-slab decomposition over torch.distributed: one process per GPU (or per CPU rank).

north_star: "the voxel grid shards naturally along Z into per-GPU slabs across the 8
MI355X of one node".  Rank r of W owns the k planes [r*nk/W, (r+1)*nk/W).

* backend="gpu": each rank drives one GPU through an sdfgen_hip_slab session.  The
  ranks exchange the IPC handles of their inboxes once (all_gather over the process
  group), map their neighbours' inboxes, and from then on the sweeps' boundary planes
  move GPU-to-GPU inside the running kernels (one-sided stores over xGMI) -- no
  collective sits on the data path.  Launch with torch.distributed.run, one rank per GPU.
* backend="cpu": the CPU slab sessions; each sweep's boundary plane is sent to the next
  slab with point-to-point send/recv on the process group (works with gloo).  This is
  the path the multi-process CPU tests exercise.

Either way the assembled result is bit-identical to the single-device run and to the
reference's single-threaded CPU path.  The reference has no multi-device layer (SURVEY
§1: README.md:220 lists multi-GPU support as future work), so this module has no
reference counterpart; its per-rank output is exactly the reference's phi restricted to
the rank's planes.
"""
from __future__ import annotations

import numpy as np

from . import _lib

__all__ = ["slab_range", "make_level_set3", "control_group", "release"]

_sessions: dict = {}


def slab_range(nk: int, world: int, rank: int) -> tuple[int, int]:
    """k planes [k_begin, k_end) owned by `rank` (the sessions' own split)."""
    return rank * nk // world, (rank + 1) * nk // world


def _dist():
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        raise RuntimeError("sdfgenfast_amd.distributed needs an initialised torch.distributed process group")
    return dist


def _group_ranks(dist, group):
    """Global ranks of `group` in group-rank order (the default group: 0..world-1)."""
    if group is None or group == dist.group.WORLD:
        return list(range(dist.get_world_size()))
    return list(dist.get_process_group_ranks(group))


def control_group(group=None):
    """The gloo group that carries this module's host-side objects (IPC handles, barriers,
    the gather) for `group`: `group` itself when it is gloo.  For a non-gloo group (e.g. the
    nccl default group) a gloo group over exactly the same ranks is created by
    torch.distributed.new_group, which is collective over the DEFAULT group: every process
    of the default group must take part.  That holds automatically for the default group
    (every rank calls make_level_set3); for a non-gloo SUBGROUP call this function on every
    rank of the default group, members or not, before the first make_level_set3 on it."""
    dist = _dist()
    if dist.get_backend(group) == "gloo":
        return group
    ranks = _group_ranks(dist, group)
    key = ("gloo", tuple(ranks))
    if key not in _sessions:
        _sessions[key] = dist.new_group(ranks=ranks, backend="gloo")
    return _sessions[key]


def _control_group(dist, group):
    if dist.get_backend(group) == "gloo":
        return group
    ranks = _group_ranks(dist, group)
    key = ("gloo", tuple(ranks))
    if key not in _sessions and len(ranks) != dist.get_world_size():
        raise ValueError("make_level_set3 on a non-gloo subgroup needs its gloo control group: call "
                         "sdfgenfast_amd.distributed.control_group(group) on EVERY rank of the default group first")
    return control_group(group)


def _gpu_session(dist, group, device: int, dims, world: int, rank: int):
    key = ("gpu", device, dims, world, rank, id(group))
    sess = _sessions.get(key)
    if sess is None:
        sess = _lib.Slab(device, world, rank, *dims)
        ctl = _control_group(dist, group)
        handles = [None] * world
        dist.all_gather_object(handles, sess.export(), group=ctl)
        sess.connect_ipc(handles[rank - 1] if rank > 0 else None, handles[rank + 1] if rank < world - 1 else None)
        dist.barrier(group=ctl)   # every inbox is mapped and zeroed before anyone writes
        _sessions[key] = sess
    return sess


def _cpu_slab(dist, group, v, t, origin, dx, dims, exact_band, world, rank):
    import torch
    ni, nj, _ = dims
    sess = _lib.CpuSlab(world, rank, *dims)
    sess.band(v, t, origin, dx, exact_band)
    ranks = _group_ranks(dist, group)
    for s in range(16):
        below = sess.upstream_is_below(s)
        up = rank - 1 if below else rank + 1
        down = rank + 1 if below else rank - 1
        plane_in = None
        if 0 <= up < world:
            buf = torch.empty(ni * nj, dtype=torch.int64)
            dist.recv(buf, src=ranks[up], group=group)
            plane_in = buf.numpy().view(np.uint64)
        out = sess.sweep(s, plane_in, 0 <= down < world)
        if out is not None:
            dist.send(torch.from_numpy(out.view(np.int64)), dst=ranks[down], group=group)
    phi = sess.sign(_lib.LAYOUT_ARRAY3)
    sess.close()
    return phi


def make_level_set3(vertices, triangles, origin, dx: float, ni: int, nj: int, nk: int, exact_band: int = 1, *,
                    backend: str = "gpu", device: int | None = None, group=None, gather_to: int | None = 0):
    """Collective: every rank of `group` calls it with the same mesh and grid.

    Returns (phi, k_begin, k_end).  phi is this rank's slab, phi[i, j, k - k_begin]
    (ni x nj x (k_end - k_begin), float32); on rank `gather_to` (None: no gather) it is
    the whole (ni, nj, nk) grid instead, with k_begin, k_end = 0, nk.
    """
    dist = _dist()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dims = (int(ni), int(nj), int(nk))
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(triangles, dtype=np.uint32).reshape(-1, 3)
    if backend == "gpu":
        dev = rank % max(_lib.device_count(), 1) if device is None else int(device)
        sess = _gpu_session(dist, group, dev, dims, world, rank)
        phi, _ = sess.run(v, t, origin, dx, exact_band, _lib.LAYOUT_ARRAY3)
    elif backend == "cpu":
        phi = _cpu_slab(dist, group, v, t, origin, dx, dims, exact_band, world, rank)
    else:
        raise ValueError(f"backend must be 'gpu' or 'cpu', got {backend!r}")
    kb, ke = slab_range(nk, world, rank)
    if gather_to is None:
        return phi, kb, ke
    ctl = _control_group(dist, group)
    ranks = _group_ranks(dist, group)
    parts = [None] * world if rank == gather_to else None
    dist.gather_object(np.asfortranarray(phi), parts, dst=ranks[gather_to], group=ctl)
    if rank != gather_to:
        return phi, kb, ke
    full = np.concatenate([np.asfortranarray(p).ravel(order="F") for p in parts])
    return full.reshape(dims, order="F"), 0, nk


def release() -> None:
    """Destroy this process's cached slab sessions (unmaps the neighbours' inboxes)."""
    for k in list(_sessions):
        if k[0] == "gpu":
            _sessions.pop(k).close()
