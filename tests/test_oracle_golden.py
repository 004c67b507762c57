"""The oracle (oracle/sdf_oracle.c) is pinned bit-for-bit against the reference.

Fixtures in tests/golden/ come from the reference's own
cpu_lib/makelevelset3.cpp (tests/golden/make_golden.py).  When the reference
build oracle/_ref is present (development container) the restatement is also
checked against it on randomised inputs."""
import hashlib
import io
import os
import struct

import numpy as np
import pytest

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import meshgen


def test_oracle_matches_reference_fixtures(golden_case):
    c = golden_case
    phi = O.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
    assert bits_equal(np.ascontiguousarray(phi), c.phi), diff_report(phi, c.phi, c.dx)


def test_x3y4z5_sdf_file_hash():
    """`SDFGen test_x3y4z5_bin.stl 32 32 32 1 1` writes an .sdf whose
    SHA-256 is 426adb5c...; rebuild those bytes from the oracle's phi."""
    c = next(g for g in __import__("conftest").GOLDEN_CASES if g.name == "x3y4z5_stl_32")
    phi = np.ascontiguousarray(O.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, 32, 32, 32, 1))
    buf = io.BytesIO()
    buf.write(struct.pack("<3i", 32, 32, 32))
    o = np.asarray(c.origin, np.float32)
    dx = np.float32(c.dx)
    buf.write(o.tobytes())
    buf.write(np.array([o[q] + np.float32(32) * dx for q in range(3)], np.float32).tobytes())
    buf.write(phi.astype("<f4").tobytes())
    assert hashlib.sha256(buf.getvalue()).hexdigest() == \
        "426adb5ca3b0aa53834ec05384a6aedefb58f16a6581ae0b80b37c26b5147d9b"
    assert int((phi < 0).sum()) == 5698
    assert int(((phi == 0) & np.signbit(phi)).sum()) == 187


def test_oracle_stages_compose(golden_case):
    """band -> sweep -> sign through the staged entry points equals the whole call."""
    c = golden_case
    phi, ct, cnt = O.band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
    phi2, ct2 = O.sweep(c.vertices, c.triangles, c.origin, c.dx, phi, ct)
    par = np.cumsum(cnt, axis=0) % 2 == 1
    out = np.where(par, -phi2, phi2)
    assert bits_equal(np.ascontiguousarray(out), c.phi)
    # closest_tri is a valid label wherever phi moved off the initial value
    init = np.float32(sum(c.dims)) * np.float32(c.dx)
    assert ((ct2 >= 0) == (phi2 != init)).all()


@pytest.mark.skipif(not O.ref_available(), reason="reference build oracle/_ref not present")
def test_oracle_ptd_matches_reference_randomised():
    rng = np.random.default_rng(20251205)
    n = 400_000
    pts = rng.uniform(-2, 2, size=(n, 12)).astype(np.float32)
    pts[::97, 6:9] = pts[::97, 3:6]          # degenerate edge
    pts[::101, 0:3] = pts[::101, 3:6]        # query on a vertex
    pts[1::7] *= np.float32(1e-3)            # tiny
    pts[2::11] = np.round(pts[2::11] * 4) / 4  # lattice ties
    pts[3::13, 9:12] = pts[3::13, 3:6]       # repeated vertex (zero-area)
    a = O.ptd_batch(pts)
    b = O.ref_ptd_batch(pts)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{(~same).sum()} mismatches"


@pytest.mark.skipif(not O.ref_available(), reason="reference build oracle/_ref not present")
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_reference_random_meshes(seed):
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1, 1, size=(60, 3)).astype(np.float32)
    t = rng.integers(0, 60, size=(40, 3)).astype(np.uint32)
    dims = tuple(int(x) for x in rng.integers(3, 24, size=3))
    o, dx = meshgen.grid_mode2b(v, max(dims[0], 5), max(dims[1], 5), max(dims[2], 5), 1)
    band = int(rng.integers(0, 3))
    a = O.make_level_set3(v, t, o, dx, *dims, exact_band=band)
    b = O.ref_make_level_set3(v, t, o, dx, *dims, exact_band=band)
    assert bits_equal(np.ascontiguousarray(a), np.ascontiguousarray(b)), diff_report(a, b, dx)


def test_golden_hashes_cover_full_size_configs():
    """Every digest in hashes.json is of the input meshgen rebuilds today (mesh bytes, grid)."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "hashes.json")) as f:
        db = json.load(f)
    assert "c2_sphere70k_128" in db and "c3_sphere1m_256" in db
    for name, rec in db.items():
        if name == "c5_sphere4m_1024":   # 4M triangles: slow to rebuild here; the GPU test checks it
            continue
        v, t, o, dx, dims = meshgen.workload(name)
        assert hashlib.sha256(v.tobytes() + t.tobytes()).hexdigest() == rec["mesh_sha256"], name
        assert [float(a) for a in o] == rec["origin"] and float(dx) == rec["dx"], name
        assert list(dims) == rec["dims"], name


@pytest.mark.parametrize("threads", [2, 3, 7])
def test_oracle_band_mt_equals_band(golden_case, threads):
    """oracle_band_mt (planes split over host threads, every triangle in ascending t per thread)
    is bit-identical to oracle_band, the restatement of cpu_lib/makelevelset3.cpp:196-236."""
    c = golden_case
    a = O.band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
    b = O.band_mt(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band, threads=threads)
    for x, y in zip(a, b):
        assert np.array_equal(np.ascontiguousarray(x).view(np.uint32), np.ascontiguousarray(y).view(np.uint32))


def test_oracle_matches_reference_edge_fixtures(edge_case):
    """The restatement's int(double) (INT_MIN out of range / NaN, x86 cvttsd2si) and wrapping
    +-band arithmetic reproduce the reference on far, NaN and infinite vertices and extreme bands."""
    c = edge_case
    with np.errstate(all="ignore"):
        phi = O.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
    assert bits_equal(np.ascontiguousarray(phi), c.phi), diff_report(phi, c.phi, c.dx)


def test_edge_fixtures_discriminate():
    """The edge fixtures exercise what they are for: vertices past 2^31 cells, NaN, +-Inf and a band
    whose +band+1 wraps (the clamp then flips the box)."""
    from conftest import EDGE_CASES
    names = {c.name for c in EDGE_CASES}
    assert {"far_x+300", "far_y-300", "far_z+220", "nan_x", "pinf_z", "ninf_y", "cube_band_2147483647"} <= names
    far = next(c for c in EDGE_CASES if c.name == "far_z+300")
    f = (far.vertices[-1].astype(np.float64) - far.origin.astype(np.float64)) / np.float64(far.dx)
    assert abs(f[2]) > 2**31
    assert any(np.isnan(c.vertices).any() for c in EDGE_CASES)
    assert any(np.isinf(c.vertices).any() for c in EDGE_CASES)
