"""The band phase (narrow band + ray parity, cpu_lib/makelevelset3.cpp:196-236) on the GPU, on its
own and inside whole calls: fine meshes (batched, LDS-merged), coarse meshes and wide bands (the
big-triangle list spread over the chip), and the inputs whose boxes go through C++ int(double)
out of range, NaN, +-Inf and the +band+1 wrap.

Stage-1 tests compare the device's pre-sweep state (sdfgen_hip_debug_band: phi, closest_tri and the
intersection counts) with oracle.band -- the restatement pinned to the reference -- array for array.
Whole calls compare with the reference's own output (edge_cases.npz, hashes.json digests)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import EDGE_CASES, GOLDEN, GOLDEN_CASES, bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen

pytestmark = pytest.mark.gpu

BIG_VOL, BIG_LAT = 4096, 1024   # sdfgen_hip.hip BAND_BIG_VOL / BAND_BIG_LAT


def setup_module(_):
    assert _lib.device_count() > 0, "no HIP device visible: the -m gpu suite needs an MI355X"


def _stage1_equal(got, want):
    phi, ct, cnt, _ = got
    wphi, wct, wcnt = want
    msgs = []
    if not np.array_equal(np.asarray(phi).view(np.uint32), np.asarray(wphi).view(np.uint32)):
        msgs.append(f"phi: {int((np.asarray(phi).view(np.uint32) != np.asarray(wphi).view(np.uint32)).sum())} cells")
    if not np.array_equal(ct, wct):
        msgs.append(f"closest_tri: {int((ct != wct).sum())} cells")
    if not np.array_equal(cnt.astype(np.int64), wcnt.astype(np.int64)):
        msgs.append(f"counts: {int((cnt.astype(np.int64) != wcnt).sum())} cells")
    return msgs


def _boxes(v, t, o, dx, dims, band):
    """Band-box volumes and ray-lattice sizes per triangle (numpy restatement of :206-225 for finite,
    in-range inputs) -- to assert which path a test exercises."""
    f = (v[t].astype(np.float64) - o.astype(np.float64)) / np.float64(dx)   # (T, 3 vertices, 3 axes)
    lo = np.trunc(f.min(axis=1)).astype(np.int64)
    hi = np.trunc(f.max(axis=1)).astype(np.int64)
    n = np.array(dims, np.int64)
    b0 = np.clip(lo - band, 0, n - 1)
    b1 = np.clip(hi + band + 1, 0, n - 1)
    vol = np.prod(np.maximum(b1 - b0 + 1, 0), axis=1)
    l0 = np.clip(np.ceil(f.min(axis=1)[:, 1:]).astype(np.int64), 0, n[1:] - 1)
    l1 = np.clip(np.floor(f.max(axis=1)[:, 1:]).astype(np.int64), 0, n[1:] - 1)
    lat = np.prod(np.maximum(l1 - l0 + 1, 0), axis=1)
    return vol, lat


# ---------------------------------------------------------------- stage 1 vs the oracle
@pytest.mark.parametrize("case", GOLDEN_CASES + EDGE_CASES, ids=[c.name for c in GOLDEN_CASES + EDGE_CASES])
def test_band_stage1_fixture_inputs(case):
    c = case
    with np.errstate(all="ignore"):
        want = O.band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
        got = _lib.debug_band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band)
    assert not _stage1_equal(got, want), _stage1_equal(got, want)


@pytest.mark.parametrize("seed", range(8))
def test_band_stage1_coarse_random(seed):
    """Random soups of large triangles with bands 0-6 on ragged grids: both work classes in one
    call (some triangles batched, some big), against oracle.band."""
    rng = np.random.default_rng(1000 + seed)
    nt = int(rng.integers(20, 300))
    v = rng.uniform(-1, 1, size=(nt * 2, 3)).astype(np.float32)
    t = rng.integers(0, len(v), size=(nt, 3)).astype(np.uint32)
    # a quarter of the triangles tiny (batched), the rest as they come (mostly big)
    small = rng.random(nt) < 0.25
    v2 = v.copy()
    for q in np.nonzero(small)[0]:
        c0 = v[t[q, 0]]
        for r in range(3):
            v2 = np.concatenate([v2, (c0 + rng.normal(0, 0.01, 3)).astype(np.float32)[None]])
        t[q] = [len(v2) - 3, len(v2) - 2, len(v2) - 1]
    v = v2.astype(np.float32)
    dims = tuple(int(x) for x in rng.integers(8, 64, size=3))
    o, dx = meshgen.grid_mode2b(v, *(max(d, 6) for d in dims), 1)
    band = int(rng.integers(0, 7))
    want = O.band(v, t, o, dx, *dims, exact_band=band)
    got = _lib.debug_band(v, t, o, dx, *dims, band)
    vol, lat = _boxes(v, t, o, dx, dims, band)
    n_big = int(((vol > BIG_VOL) | (lat > BIG_LAT)).sum())
    assert got[3] == n_big, (got[3], n_big)
    assert not _stage1_equal(got, want), _stage1_equal(got, want)


def test_band_stage1_batch_boxes_past_2_32():
    """One 64-triangle batch whose band boxes sum past 2^32 cells (16 tetrahedra inscribed in a
    410 x 412 x 414 grid: every face box spans the grid, 64 x ~70M = 4.5G (triangle, cell) pairs) --
    the count that wrapped in 32 bits before round 4.  Against the plane-split oracle (bit-identical
    to oracle.band, tests/test_oracle_golden.py)."""
    vt, tt = meshgen.tetrahedron()
    rng = np.random.default_rng(5)
    vs, ts = [], []
    for q in range(16):
        vs.append((vt * np.float32(1.0 - 0.0005 * q) + rng.uniform(-0.0004, 0.0004, size=(4, 3))).astype(np.float32))
        ts.append(tt + 4 * q)
    v, t = np.concatenate(vs), np.concatenate(ts).astype(np.uint32)
    dims = (410, 412, 414)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    vol, lat = _boxes(v, t, o, dx, dims, 1)
    assert len(t) == 64 and int(vol.sum()) > 2**32, int(vol.sum())
    got = _lib.debug_band(v, t, o, dx, *dims, 1)
    assert got[3] == 64
    want = O.band_mt(v, t, o, dx, *dims, exact_band=1)
    assert not _stage1_equal(got, want), _stage1_equal(got, want)


# ---------------------------------------------------------------- whole calls on the reference's edge fixtures
@pytest.mark.parametrize("layout", [_lib.LAYOUT_KFAST, _lib.LAYOUT_ARRAY3])
def test_gpu_edge_fixtures_c_abi(edge_case, layout):
    c = edge_case
    with np.errstate(all="ignore"):
        got = np.ascontiguousarray(_lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims,
                                                        c.exact_band, layout))
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)


def test_gpu_edge_fixtures_generate_sdf(edge_case):
    import sdfgenfast_amd as S
    c = edge_case
    with np.errstate(all="ignore"):
        got = S.generate_sdf(c.vertices, c.triangles, tuple(float(x) for x in c.origin), c.dx, *c.dims,
                             exact_band=c.exact_band, backend="gpu")
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)


@pytest.mark.parametrize("name", ["far_nan_band40", "sphere_with_bad_tris", "far_z+300", "pinf_z"])
def test_gpu_edge_fixtures_two_slabs(monkeypatch, name):
    """The Z-slab band (boxes clamped to the whole grid, then cut to the slab) on the same inputs."""
    monkeypatch.setenv("SDFGEN_DEBUG_SLABS_ONE_DEVICE", "1")
    monkeypatch.setenv("SDFGEN_TILE_GRID", "96")
    c = next(e for e in EDGE_CASES if e.name == name)
    with np.errstate(all="ignore"):
        got = np.ascontiguousarray(_lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims,
                                                        c.exact_band, _lib.LAYOUT_KFAST, ngpu=2))
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)


# ---------------------------------------------------------------- the reference's benchmark workload, a coarse 512^3 mesh
def _hashes():
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["x3y4z5_prop64", "x3y4z5_prop128", "x3y4z5_prop256", "tetra_512"])
def test_gpu_coarse_workloads_match_reference_digest(name):
    """tests/benchmark_performance.cpp:151, 181-185 (test_x3y4z5_bin.stl, 36 triangles, proportional
    grids 64x84x104 .. 256x340x424 with padding 2: the reference's published numbers, README.md:256-260)
    and a tetrahedron whose 4 faces each span a 512^3 grid -- against the reference's SHA-256 of phi
    (1 thread)."""
    rec = _hashes().get(name)
    if rec is None:
        pytest.skip(f"no reference digest for {name}")
    v, t, o, dx, dims = meshgen.workload(name)
    assert hashlib.sha256(v.tobytes() + t.tobytes()).hexdigest() == rec["mesh_sha256"]
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    flat = np.asfortranarray(got).ravel(order="F").astype("<f4")
    assert hashlib.sha256(flat.tobytes()).hexdigest() == rec["sha256_phi"]
    assert int(np.count_nonzero(flat < 0)) == rec["inside_lt0"]
    p = _lib.last_profile()
    assert p["band_evals"] > 0


def test_gpu_first_call_after_slab_sessions_fresh_process():
    """Round 4's freed-uncached-memory failure: stage-1 calls, in-process two-slab calls, then the
    first one-GPU call, in a fresh process (tests/slab_then_one_gpu_check.py)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_then_one_gpu_check.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
