"""Z-slab decomposition (sdfgen_hip_slab_*) -- bit-exact against the oracle.

Slabs of one grid run concurrently on ONE GPU here (the box has one), either in one
process (connect_local, one HIP stream per slab) or one process per slab with the
inboxes mapped through HIP IPC (the 8-GPU layout, minus xGMI).  Every slab's tile
kernel is capped (SDFGEN_TILE_GRID) so that all slabs' workgroups are resident at
once -- on separate GPUs nothing is shared and no cap is needed.
"""
import multiprocessing as mp
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import meshgen

pytestmark = pytest.mark.gpu


def _mesh(nu=90, nv=31, dims=(40, 36, 44)):
    v, t = meshgen.bumpy_sphere(nu, nv)
    o, dx = meshgen.grid_mode2b(v, *(max(d, 8) for d in dims), 2)   # small grids: a crop of an 8^3 layout
    return v, t, o, dx, dims


@pytest.fixture(autouse=True)
def _cap_grid(monkeypatch):
    monkeypatch.setenv("SDFGEN_TILE_GRID", "96")


# In one process every slab needs its own hardware queue (a consumer kernel spinning in
# a queue shared with its producer would wait forever); GPU_MAX_HW_QUEUES is 4 on the box,
# so in-process tests use 2 slabs and the 3-4 slab layouts run one process per slab.
@pytest.mark.parametrize("nslabs,dims", [(2, (40, 36, 44)), (2, (33, 41, 29)), (2, (9, 9, 4)), (2, (17, 5, 60))])
def test_slabs_one_process_match_oracle(nslabs, dims):
    from sdfgenfast_amd import _hiprt, _lib
    v, t, o, dx, dims = _mesh(dims=dims)
    ni, nj, nk = dims
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, ni, nj, nk, 1))
    slabs = [_lib.Slab(0, nslabs, s, ni, nj, nk) for s in range(nslabs)]
    for s, sl in enumerate(slabs):
        sl.connect_local(slabs[s - 1] if s > 0 else None, slabs[s + 1] if s < nslabs - 1 else None)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    outs = [_hiprt.DeviceBuffer(ni * nj * (sl.k_end - sl.k_begin) * 4) for sl in slabs]
    for sl_ in slabs:   # every slab set up before any slab's kernels run
        sl_.prepare(t.shape[0])
    for sl, d in zip(slabs, outs):
        sl.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_ARRAY3, d.ptr)
    profs = [sl.finish(v.shape[0]) for sl in slabs]
    got = np.concatenate([d.download(np.float32, ni * nj * (sl.k_end - sl.k_begin)) for sl, d in zip(slabs, outs)])
    got = got.reshape((ni, nj, nk), order="F")
    assert [sl.k_begin for sl in slabs][0] == 0 and slabs[-1].k_end == nk
    impl = 1 if os.environ.get("SDFGEN_SLAB_SPARSE") == "0" else 2   # diagnostics may turn parts off
    multi = 0 if os.environ.get("SDFGEN_TILE_MULTI") == "0" else 8
    assert all(p["sweep_impl"] == impl and p["slabs"] == nslabs and p["tile_multi"] == multi for p in profs)
    assert bits_equal(got, want), diff_report(got, want, dx)


def test_slab_kfast_layout_and_host_run():
    from sdfgenfast_amd import _lib
    v, t, o, dx, dims = _mesh()
    ni, nj, nk = dims
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, ni, nj, nk, 1))
    slabs = [_lib.Slab(0, 2, s, ni, nj, nk) for s in range(2)]
    slabs[0].connect_local(None, slabs[1])
    slabs[1].connect_local(slabs[0], None)
    # host-array entry runs one slab at a time: run slab 0's producer side by enqueueing
    # the device path for slab 1 first is not possible with run(); use enqueue for both
    from sdfgenfast_amd import _hiprt
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    outs = [_hiprt.DeviceBuffer(ni * nj * (sl.k_end - sl.k_begin) * 4) for sl in slabs]
    for sl_ in slabs:   # every slab set up before any slab's kernels run
        sl_.prepare(t.shape[0])
    for sl, d in zip(slabs, outs):
        sl.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_KFAST, d.ptr)
    for sl in slabs:
        sl.finish()
    parts = [d.download(np.float32, ni * nj * (sl.k_end - sl.k_begin)).reshape(ni, nj, sl.k_end - sl.k_begin)
             for sl, d in zip(slabs, outs)]
    got = np.concatenate(parts, axis=2)
    assert bits_equal(got, want), diff_report(got, want, dx)


def test_slab_validation():
    from sdfgenfast_amd import _lib
    with pytest.raises(ValueError):
        _lib.Slab(0, 3, 0, 10, 10, 5)      # fewer than 2 planes per slab
    with pytest.raises(ValueError):
        _lib.Slab(0, 2, 2, 10, 10, 10)     # slab index out of range
    s = _lib.Slab(0, 2, 0, 10, 10, 10)
    with pytest.raises(ValueError):
        s.connect_local(None, None)        # slab 0 of 2 needs its upper neighbour


def _ipc_worker(nslabs, slab, dims, q_out, q_in, barrier, res):
    os.environ["SDFGEN_TILE_GRID"] = "64"
    from sdfgenfast_amd import _lib
    v, t, o, dx, dims = _mesh(dims=dims)
    sl = _lib.Slab(0, nslabs, slab, *dims)
    q_out.put((slab, sl.export()))
    handles = q_in.get(timeout=120)
    sl.connect_ipc(handles.get(slab - 1), handles.get(slab + 1))
    barrier.wait(timeout=120)
    phi, prof = sl.run(v, t, o, dx, 1, _lib.LAYOUT_ARRAY3)
    res.put((slab, sl.k_begin, sl.k_end, np.asfortranarray(phi).tobytes(order="F"), prof["sweep_impl"]))
    barrier.wait(timeout=120)   # keep the inbox mapped until every peer has finished writing
    sl.close()


@pytest.mark.parametrize("nslabs,dims", [(3, (33, 41, 29)), (4, (24, 20, 17)), (3, (8, 70, 6))])
def test_slabs_middle_slabs_in_process(nslabs, dims):
    """Slabs with both an upstream and a downstream neighbour; one HW queue per slab stream."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", SDFGEN_TILE_GRID="64")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_inprocess_check.py"),
                        str(nslabs), *map(str, dims)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout + r.stderr[-3000:]


@pytest.mark.parametrize("name", ["c4_sphere1m_512", "c5_sphere4m_1024"])
def test_two_slabs_full_size_match_reference_digest(name):
    """north_star's Z-slab configurations at full size (C4 512^3; C5 1024^3 = 1.07G cells, past
    2^31: the slab offsets cell_mem - plane * k_begin and the 64-bit indices), two slabs on this
    box's one GPU in one process, against the reference's SHA-256 of phi."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", SDFGEN_TILE_GRID="192")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_inprocess_check.py"),
                        "2", name, "1"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("name,mode", [("c2_sphere70k_128", "slabs"), ("c2_sphere70k_128", "cabi"),
                                       ("c4_sphere1m_512", "slabs")])
def test_eight_slabs_in_process_match_reference_digest(name, mode):
    """north_star's 8-way Z split (C4 names 8 GPUs): eight slabs of one grid on this box's one GPU in
    one process -- every slab with both neighbours but the ends, seven slab boundaries per sweep --
    against the reference's SHA-256 of phi.  `slabs`: the slab C-ABI driven per slab (8 streams, one
    hardware queue each); `cabi`: sdfgen_hip_make_level_set3(ngpu=8), the library's own in-process
    multi-device path, with SDFGEN_DEBUG_SLABS_ONE_DEVICE.  The LIBRARY caps the persistent grids so
    that all eight slabs stay co-resident (no SDFGEN_TILE_GRID / SDFGEN_SPARSE_WORKERS here): it counts
    the slab sessions alive on the device and gives each half of the tile kernel's resident workgroups
    / 8 and a quarter of the repair kernel's / 8 (a slab's repair kernel ends only after its upstream
    neighbour's, so all eight must be resident at once: 8 x the default 256 one-wave repair workgroups
    at 171 VGPRs are exactly the chip's 2,048 wave slots for them -- a round-5 run without a cap ran into
    the repair watchdogs).  One hardware queue per slab stream (GPU_MAX_HW_QUEUES; the library refuses
    more sessions on a device than queues).  On 8 GPUs nothing is shared."""
    env = {k: v for k, v in os.environ.items() if k not in ("SDFGEN_TILE_GRID", "SDFGEN_SPARSE_WORKERS")}
    env["GPU_MAX_HW_QUEUES"] = "16"
    args = ["8", name, "2" if name.startswith("c2") else "1"] + (["--cabi"] if mode == "cabi" else [])
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_inprocess_check.py"), *args],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


# One process per slab, inboxes mapped with HIP IPC.  Two processes only: more processes
# sharing one GPU's hardware queues are not guaranteed to run their kernels concurrently.
@pytest.mark.parametrize("nslabs,dims", [(2, (40, 36, 44)), (2, (19, 23, 31))])
def test_slabs_ipc_one_process_per_slab_match_oracle(nslabs, dims):
    ctx = mp.get_context("spawn")
    q_out, res, barrier = ctx.Queue(), ctx.Queue(), ctx.Barrier(nslabs)
    q_ins = [ctx.Queue() for _ in range(nslabs)]
    procs = [ctx.Process(target=_ipc_worker, args=(nslabs, s, dims, q_out, q_ins[s], barrier, res))
             for s in range(nslabs)]
    for p in procs:
        p.start()
    try:
        handles = dict(q_out.get(timeout=100) for _ in range(nslabs))
        for q in q_ins:
            q.put(handles)
        parts = sorted(res.get(timeout=100) for _ in range(nslabs))
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    v, t, o, dx, (ni, nj, nk) = _mesh(dims=dims)
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, ni, nj, nk, 1))
    got = np.concatenate([np.frombuffer(b, np.float32) for _, _, _, b, _ in parts]).reshape((ni, nj, nk), order="F")
    assert [p[4] for p in parts] == [2] * nslabs
    assert bits_equal(got, want), diff_report(got, want, dx)


@pytest.mark.parametrize("layout", ["array3", "kfast"])
def test_c_abi_ngpu_zslab_path_matches_oracle(monkeypatch, layout):
    """sdfgen_hip_make_level_set3(ngpu=2): the in-process multi-device Z-slab path, with
    both slabs placed on this box's one GPU (SDFGEN_DEBUG_SLABS_ONE_DEVICE) -- host
    upload, enqueue-all-then-copy ordering and the strided k-fastest assembly."""
    from sdfgenfast_amd import _lib
    monkeypatch.setenv("SDFGEN_DEBUG_SLABS_ONE_DEVICE", "1")
    v, t, o, dx, dims = _mesh(dims=(33, 41, 29))
    want = O.make_level_set3(v, t, o, dx, *dims, 1)
    lay = _lib.LAYOUT_ARRAY3 if layout == "array3" else _lib.LAYOUT_KFAST
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, lay, ngpu=2)
    assert bits_equal(got, want), diff_report(got, want, dx)


def test_c_abi_ngpu_more_than_visible_is_enodev():
    from sdfgenfast_amd import _lib
    n = _lib.device_count()
    v, t, o, dx, dims = _mesh(dims=(20, 20, 20))
    with pytest.raises(RuntimeError, match="visible"):
        _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_KFAST, ngpu=n + 1)


def test_c_abi_ngpu_all_means_every_visible_device():
    """ngpu = SDFGEN_NGPU_ALL (0) = all visible devices; on a one-GPU box that
    is the single-device run, bit-exact like ngpu = SDFGEN_NGPU_CURRENT (1)."""
    from sdfgenfast_amd import _lib
    v, t, o, dx, dims = _mesh(dims=(24, 20, 28))
    want = O.make_level_set3(v, t, o, dx, *dims, 1)
    got_all = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_KFAST, ngpu=_lib.NGPU_ALL)
    got_cur = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_KFAST, ngpu=_lib.NGPU_CURRENT)
    assert bits_equal(got_all, want), diff_report(got_all, want, dx)
    assert bits_equal(got_cur, want), diff_report(got_cur, want, dx)
    if _lib.device_count() == 1:
        assert _lib.last_profile()["sweep_impl"] != 3  # one device: not the slab path


@pytest.mark.parametrize("ngpu", ["2"])   # (2 slabs: GPU_MAX_HW_QUEUES is 4 in this process, see above)
def test_generate_sdf_sdfgen_ngpu_knob(ngpu, monkeypatch):
    """SDFGEN_NGPU, the Python drop-in's GPU-count knob (generate_sdf keeps the reference signature,
    python/sdfgen_py.cpp:160-218): the grid splits into Z-slabs, here sessions on this box's one GPU
    (SDFGEN_DEBUG_SLABS_ONE_DEVICE) with the library's own grid caps (no SDFGEN_TILE_GRID), bit-exact
    against the oracle; a malformed value is a ValueError."""
    import sdfgenfast_amd as S
    from sdfgenfast_amd import _lib
    monkeypatch.delenv("SDFGEN_TILE_GRID", raising=False)
    monkeypatch.setenv("SDFGEN_DEBUG_SLABS_ONE_DEVICE", "1")
    monkeypatch.setenv("SDFGEN_NGPU", ngpu)
    v, t, o, dx, dims = _mesh(dims=(37, 41, 46))
    got = S.generate_sdf(v, t, o, dx, *dims, exact_band=1, backend="gpu")
    assert _lib.last_profile()["slabs"] == int(ngpu)
    want = np.asarray(O.make_level_set3(v, t, o, dx, *dims, 1))
    assert bits_equal(got, want), diff_report(got, want, dx)
    monkeypatch.setenv("SDFGEN_NGPU", "x2")
    with pytest.raises(ValueError):
        S.generate_sdf(v, t, o, dx, *dims, exact_band=1, backend="gpu")
