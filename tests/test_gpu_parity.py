"""Parity of the HIP/gfx950 path with the reference, through the C-ABI.

Run on an MI355X: python -m pytest tests -m gpu.  Each test calls
libsdfgen_hip.so (sdfgen_hip_* entry points); the oracle (oracle/) is only the
checker.  The bar is bit-exact float32 phi (hence |diff| <= 1e-5*dx trivially)
and a bit-exact signbit array; small cases compare whole arrays with the
reference fixtures / the oracle, full-size configs compare SHA-256 digests of
the reference's own output (tests/golden/hashes.json)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen

pytestmark = pytest.mark.gpu


def setup_module(_):
    assert _lib.device_count() > 0, "no HIP device visible: the -m gpu suite needs an MI355X"


def _hash_i_fastest(phi_ijk: np.ndarray) -> str:
    flat = np.asfortranarray(phi_ijk).ravel(order="F").astype("<f4")
    return hashlib.sha256(flat.tobytes()).hexdigest()


# ---------------------------------------------------------------- geometry
def _ptd_inputs(n, seed):
    rng = np.random.default_rng(seed)
    pts = rng.uniform(-2, 2, size=(n, 12)).astype(np.float32)
    pts[::97, 6:9] = pts[::97, 3:6]
    pts[::101, 0:3] = pts[::101, 3:6]
    pts[1::7] *= np.float32(1e-3)
    pts[4::9] *= np.float32(1e-19)           # denormal intermediates
    pts[2::11] = np.round(pts[2::11] * 4) / 4
    pts[3::13, 9:12] = pts[3::13, 3:6]
    pts[5::17] += np.float32(1000.0)
    return pts


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_device_ptd_bitwise_vs_oracle(variant):
    pts = _ptd_inputs(4_000_000, 7)
    got = _lib.debug_ptd(pts, variant=variant)
    want = O.ptd_batch(pts)
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), f"{(~same).sum()} of {len(pts)} point-triangle distances differ"


def test_device_pit2d_bitwise_vs_oracle():
    rng = np.random.default_rng(11)
    p = rng.uniform(-3, 3, size=(1_000_000, 8))
    p[::3] = np.round(p[::3])
    p[1::5, 2:4] = p[1::5, 4:6]
    p[2::7, 0:2] = p[2::7, 2:4]
    got = _lib.debug_pit2d(p)
    want = O.pit2d_batch(p)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


# ---------------------------------------------------------------- golden cases
@pytest.mark.parametrize("layout", [_lib.LAYOUT_KFAST, _lib.LAYOUT_ARRAY3])
def test_gpu_matches_reference_fixture(golden_case, layout):
    c = golden_case
    got = _lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, layout)
    got = np.ascontiguousarray(got)
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)
    assert np.array_equal(np.signbit(got), np.signbit(c.phi))


def test_gpu_generate_sdf_api(golden_case):
    import sdfgenfast_amd as S
    c = golden_case
    got = S.generate_sdf(c.vertices, c.triangles, tuple(c.origin), c.dx, *c.dims, exact_band=c.exact_band,
                         backend="gpu")
    assert got.shape == c.dims and got.dtype == np.float32 and got.flags.c_contiguous
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)


# ---------------------------------------------------------------- seeded random vs oracle
@pytest.mark.parametrize("seed", range(6))
def test_gpu_random_soup_vs_oracle(seed):
    rng = np.random.default_rng(1000 + seed)
    nv = int(rng.integers(10, 400))
    v = rng.normal(size=(nv, 3)).astype(np.float32)
    t = rng.integers(0, nv, size=(int(rng.integers(1, 300)), 3)).astype(np.uint32)
    dims = tuple(int(x) for x in rng.integers(2, 41, size=3))
    o, dx = meshgen.grid_mode2b(v, max(dims[0], 4), max(dims[1], 4), max(dims[2], 4), 1)
    band = int(rng.integers(0, 4))
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=band))
    got = _lib.make_level_set3(v, t, o, dx, *dims, band)
    assert bits_equal(got, want), diff_report(got, want, dx)


@pytest.mark.parametrize("nu,nv,dims", [(90, 31, (57, 33, 70)), (200, 61, (64, 64, 64)),
                                        (40, 21, (96, 20, 24)), (300, 101, (33, 80, 47))])
def test_gpu_sphere_vs_oracle(nu, nv, dims):
    v, t = meshgen.bumpy_sphere(nu, nv)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    assert bits_equal(got, want), diff_report(got, want, dx)


def test_gpu_repeatable():
    v, t = meshgen.bumpy_sphere(150, 51)
    o, dx = meshgen.grid_mode2b(v, 48, 48, 48, 2)
    a = _lib.make_level_set3(v, t, o, dx, 48, 48, 48, 1)
    b = _lib.make_level_set3(v, t, o, dx, 48, 48, 48, 1)
    assert bits_equal(a, b)


# ---------------------------------------------------------------- full-size configs
def _hashes():
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["c2_sphere70k_128", "c3_sphere1m_256", "c4_sphere1m_512", "c5_sphere4m_1024"])
def test_gpu_full_size_matches_reference_hash(name):
    """C5 (1024^3, 4M triangles, 4 GB of phi) only when its digest was recorded: the
    reference needs ~1.5 h single-threaded (tests/golden/make_golden.py --large c5)."""
    db = _hashes()
    if name not in db:
        pytest.skip(f"{name}: no reference digest recorded")
    rec = db[name]
    v, t, o, dx, dims = meshgen.workload(name)
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    assert int(np.count_nonzero(got < 0)) == rec["inside_lt0"]
    assert int(np.count_nonzero(np.signbit(got))) == rec["signbit_count"]
    sb = np.packbits(np.signbit(np.asfortranarray(got).ravel(order="F")))
    assert hashlib.sha256(sb.tobytes()).hexdigest() == rec["sha256_signbit"]
    assert _hash_i_fastest(got) == rec["sha256_phi"]


def test_gpu_brick_repair_full_size_matches_reference_hash(monkeypatch):
    """The brick-owned repair (SDFGEN_SPARSE_BRICK=1) at C3 size against the reference digest."""
    db = _hashes()
    name = "c3_sphere1m_256"
    if name not in db:
        pytest.skip(f"{name}: no reference digest recorded")
    monkeypatch.setenv("SDFGEN_SPARSE_BRICK", "1")
    v, t, o, dx, dims = meshgen.workload(name)
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    assert _lib.last_profile()["sparse_sweeps"] == 8
    assert _hash_i_fastest(got) == db[name]["sha256_phi"]


# ---------------------------------------------------------------- contracts
def test_gpu_bad_index_raises():
    v = np.eye(3, dtype=np.float32)
    t = np.array([[0, 1, 2], [0, 1, 999]], np.uint32)
    with pytest.raises(IndexError):
        _lib.make_level_set3(v, t, (0, 0, 0), 0.1, 8, 8, 8, 1)


def _hip_runtime():
    """The HIP runtime libsdfgen_hip.so itself links (same process-wide instance)."""
    import ctypes
    rt = ctypes.CDLL("libamdhip64.so.7")
    rt.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    rt.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    rt.hipFree.argtypes = [ctypes.c_void_p]
    return rt


def test_gpu_device_entry_with_device_buffers():
    """sdfgen_hip_make_level_set3_device on caller-owned HBM buffers (no torch: torch
    bundles its own HIP runtime)."""
    import ctypes
    rt = _hip_runtime()
    v, t = meshgen.bumpy_sphere(100, 41)
    o, dx = meshgen.grid_mode2b(v, 40, 36, 44, 2)
    n = 40 * 36 * 44
    bufs = []
    def dmalloc(nbytes):
        p = ctypes.c_void_p()
        assert rt.hipMalloc(ctypes.byref(p), nbytes) == 0
        bufs.append(p)
        return p.value
    try:
        dv, dt, dout = dmalloc(v.nbytes), dmalloc(t.nbytes), dmalloc(4 * n)
        assert rt.hipMemcpy(dv, v.ctypes.data, v.nbytes, 1) == 0
        assert rt.hipMemcpy(dt, t.ctypes.data, t.nbytes, 1) == 0
        _lib.make_level_set3_device(0, dt, t.shape[0], dv, v.shape[0], o, dx, 40, 36, 44, 1,
                                    _lib.LAYOUT_KFAST, dout)
        got = np.empty(n, np.float32)
        assert rt.hipMemcpy(got.ctypes.data, dout, 4 * n, 2) == 0
    finally:
        for p in bufs:
            rt.hipFree(p)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, 40, 36, 44, 1))
    assert bits_equal(got.reshape(40, 36, 44), want), diff_report(got.reshape(40, 36, 44), want, dx)
    prof = _lib.last_profile()
    assert prof["total_ms"] > 0 and prof["band_evals"] > 0


# ---------------------------------------------------------------- both sweep implementations
# plane: one launch per hyperplane; tile: the column wavefront for all 16 sweeps;
# hybrid (default): wavefront for the first pass, Jacobi + repair for the second;
# sparse: Jacobi + repair for all 16 (stresses the repair protocol: most labels change);
# *-brick: the same with the brick-owned repair (sweep_sparse.hpp k_sp_brick, not the default);
# *-2buf: the repair on two swapped buffers instead of in place (SpParams::sv, the default).
SWEEP_MODES = {"plane": ({"SDFGEN_SWEEP": "plane"}, 0), "tile": ({"SDFGEN_SPARSE_FROM": "16"}, 1),
               "hybrid": ({}, 2), "sparse": ({"SDFGEN_SPARSE_FROM": "0"}, 2),
               "sparse-2buf": ({"SDFGEN_SPARSE_FROM": "0", "SDFGEN_SPARSE_INPLACE": "0"}, 2),
               "hybrid-brick": ({"SDFGEN_SPARSE_BRICK": "1"}, 2),
               "sparse-brick": ({"SDFGEN_SPARSE_FROM": "0", "SDFGEN_SPARSE_BRICK": "1"}, 2)}


@pytest.fixture(params=list(SWEEP_MODES))
def sweep_impl(request, monkeypatch):
    for k in ("SDFGEN_SWEEP", "SDFGEN_SPARSE_FROM", "SDFGEN_SPARSE_BRICK", "SDFGEN_SPARSE_INPLACE"):
        monkeypatch.delenv(k, raising=False)
    env, _ = SWEEP_MODES[request.param]
    for k, val in env.items():
        monkeypatch.setenv(k, val)
    return request.param


@pytest.mark.parametrize("dims", [(2, 2, 2), (3, 2, 9), (9, 2, 3), (2, 17, 3), (10, 9, 17), (33, 8, 16), (5, 41, 9)])
def test_gpu_sweep_impls_small_and_ragged_grids(sweep_impl, dims):
    v, t = meshgen.bumpy_sphere(30, 13)
    o, dx = meshgen.grid_mode2b(v, max(dims[0], 5), max(dims[1], 5), max(dims[2], 5), 1)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    assert bits_equal(got, want), diff_report(got, want, dx)


# The second pass's k-streaming pair scan (sweep_sparse.hpp k_sp_jscan3) cuts each row into segments of
# 64 x 2 NP cells, groups 4 rows per workgroup and walks chunks of planes: rows of several segments with a
# partial last one (the lanes past the row end, the DPP hand-off across a segment edge in both i
# directions), row groups and plane chunks that do not divide the grid.
@pytest.mark.parametrize("dims", [(300, 9, 11), (513, 5, 7), (257, 6, 13)])
@pytest.mark.parametrize("mode", ["hybrid", "sparse"])
def test_gpu_second_pass_scan_row_segments(mode, dims, monkeypatch):
    for k in ("SDFGEN_SWEEP", "SDFGEN_SPARSE_FROM", "SDFGEN_SPARSE_BRICK", "SDFGEN_SPARSE_INPLACE"):
        monkeypatch.delenv(k, raising=False)
    for k, val in SWEEP_MODES[mode][0].items():
        monkeypatch.setenv(k, val)
    v, t = meshgen.bumpy_sphere(60, 23)
    o, dx = meshgen.grid_mode2b(v, *dims, 1)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    prof = _lib.last_profile()
    assert prof["sparse_sweeps"] == (16 if mode == "sparse" else 8)
    assert bits_equal(got, want), diff_report(got, want, dx)


@pytest.mark.parametrize("nu,nv,dims", [(90, 31, (57, 33, 70)), (40, 21, (17, 40, 35)), (200, 61, (64, 48, 40))])
def test_gpu_sweep_impls_agree_with_oracle(sweep_impl, nu, nv, dims):
    v, t = meshgen.bumpy_sphere(nu, nv)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    prof = _lib.last_profile()
    assert prof["sweep_impl"] == SWEEP_MODES[sweep_impl][1]
    if sweep_impl.startswith("sparse"):
        assert prof["sparse_sweeps"] == 16 and prof["sparse_rechecks"] > 0
    assert bits_equal(got, want), diff_report(got, want, dx)


# ---------------------------------------------------------------- host entry point
@pytest.mark.parametrize("layout", [_lib.LAYOUT_ARRAY3, _lib.LAYOUT_KFAST])
def test_gpu_host_entry_into_offset_and_pinned_arrays(layout):
    """sdfgen_hip_make_level_set3 into an output array 4 bytes off its allocation's alignment and
    into HIP-pinned host memory (hipHostMalloc, like a pinned torch tensor), from read-only inputs:
    the reference's bits."""
    import ctypes
    db = _hashes()
    name = "c2_sphere70k_128"
    if name not in db:
        pytest.skip(f"{name}: no reference digest recorded")
    v, t, o, dx, dims = meshgen.workload(name)
    v.setflags(write=False)
    t.setflags(write=False)
    n = dims[0] * dims[1] * dims[2]
    for off in (0, 1):
        out = np.empty(n + 1, np.float32)[off:off + n]
        got = _lib.make_level_set3(v, t, o, dx, *dims, 1, layout, out=out)
        assert _hash_i_fastest(got) == db[name]["sha256_phi"], f"offset {4 * off} B"
    rt = _hip_runtime()
    rt.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    rt.hipHostFree.argtypes = [ctypes.c_void_p]
    p = ctypes.c_void_p()
    assert rt.hipHostMalloc(ctypes.byref(p), 4 * n, 0) == 0
    try:
        out = np.ctypeslib.as_array((ctypes.c_float * n).from_address(p.value))
        got = _lib.make_level_set3(v, t, o, dx, *dims, 1, layout, out=out)
        assert _hash_i_fastest(got) == db[name]["sha256_phi"], "pinned output"
    finally:
        rt.hipHostFree(p)


def test_gpu_host_entry_fresh_outputs_c2_c4_c2():
    """The shipped host path (sdfgen_hip_make_level_set3: pageable hipMemcpy in and out, no registration
    of caller memory) into FRESH numpy arrays at C2 -> C4 -> C2 in one process, fresh inputs each time:
    the sequence in which round 3's host-mapped prototype faulted (the C4 output is above
    the ROCm runtime's own pinning threshold, the C2 ones below it).  Bit-exact against the reference."""
    db = _hashes()
    for name in ("c2_sphere70k_128", "c4_sphere1m_512", "c2_sphere70k_128"):
        v, t, o, dx, dims = meshgen.workload(name)
        got = _lib.make_level_set3(v.copy(), t.copy(), o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
        assert _hash_i_fastest(got) == db[name]["sha256_phi"], name
        del got, v, t
