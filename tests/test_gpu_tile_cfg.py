"""The first-pass tile kernel configurations (sweep_tile.hpp StCfgLat / StCfgThr / StCfgQuad / StCfgDuo) against
the oracle and the reference digests.  The library picks one by the tiles a sweep offers (st_use_thr:
256^3 runs the 2-wave tiles, 512^3 and 1024^3 the 1-wave tiles); SDFGEN_TILE_CFG forces either, so
each is pinned on every grid shape here -- ragged, tiny, shifted, full size and Z-slabs."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen

pytestmark = pytest.mark.gpu
CFGS = [0, 1, 2, 3, 4, 5]


@pytest.fixture(params=CFGS, ids=["lat", "thr", "quad", "duo", "oct", "qfp"])
def cfg(request, monkeypatch):
    monkeypatch.setenv("SDFGEN_TILE_CFG", str(request.param))
    return request.param


def test_golden_cases(cfg, golden_case):
    c = golden_case
    got = _lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, _lib.LAYOUT_KFAST)
    assert bits_equal(got, c.phi), diff_report(got, c.phi, c.dx)


@pytest.mark.parametrize("nu,nv,dims", [(90, 31, (57, 33, 70)), (200, 61, (64, 64, 64)), (40, 21, (96, 20, 24)),
                                        (300, 101, (33, 80, 47)), (120, 41, (9, 130, 17))])
def test_spheres_vs_oracle(cfg, nu, nv, dims):
    v, t = meshgen.bumpy_sphere(nu, nv)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=1))
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    assert bits_equal(got, want), diff_report(got, want, dx)
    p = _lib.last_profile()
    assert p["tile_multi"] == 0 or p["tile_cfg"] == cfg


@pytest.mark.parametrize("seed", range(4))
def test_random_soups_vs_oracle(cfg, seed):
    rng = np.random.default_rng(2000 + seed)
    nv = int(rng.integers(10, 400))
    v = rng.normal(size=(nv, 3)).astype(np.float32)
    t = rng.integers(0, nv, size=(int(rng.integers(1, 300)), 3)).astype(np.uint32)
    dims = tuple(int(x) for x in rng.integers(2, 41, size=3))
    o, dx = meshgen.grid_mode2b(v, max(dims[0], 4), max(dims[1], 4), max(dims[2], 4), 1)
    band = int(rng.integers(0, 4))
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=band))
    got = _lib.make_level_set3(v, t, o, dx, *dims, band)
    assert bits_equal(got, want), diff_report(got, want, dx)


@pytest.mark.parametrize("name", ["c2_sphere70k_128", "c3_sphere1m_256", "c4_sphere1m_512"])
def test_full_size_digest(cfg, name):
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        rec = json.load(f)[name]
    v, t, o, dx, dims = meshgen.workload(name)
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    assert _lib.last_profile()["tile_cfg"] == cfg
    h = hashlib.sha256(np.asfortranarray(got).ravel(order="F").astype("<f4").tobytes()).hexdigest()
    assert h == rec["sha256_phi"]


def test_default_selection_by_grid(monkeypatch):
    """No override: the quad-lane tiles up to 2,000 tiles per sweep (256^3: 1,024; 320^3: 1,600),
    the 1-wave tiles above (384^3: 2,304; 512^3: 4,096) -- sweep_tile.hpp ST_QUAD_MAX_TILES."""
    monkeypatch.delenv("SDFGEN_TILE_CFG", raising=False)
    for name, want in (("c3_sphere1m_256", 2), ("sphere1m_320", 2), ("sphere1m_384", 1), ("c4_sphere1m_512", 1)):
        v, t, o, dx, dims = meshgen.workload(name)
        _lib.make_level_set3(v, t, o, dx, *dims, 1)
        assert _lib.last_profile()["tile_cfg"] == want, name


@pytest.mark.parametrize("what", [("2", "40", "36", "44"), ("2", "c2_sphere70k_128", "1")])
def test_two_slabs_in_process(cfg, what):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", SDFGEN_TILE_GRID="96", SDFGEN_TILE_CFG=str(cfg))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_inprocess_check.py"), *what],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_two_slabs_in_process_per_sweep_launches(cfg):
    """The Z-slab path with one launch per first-pass sweep (SDFGEN_TILE_MULTI=0: what it falls back
    to when the overlapped launch's halo buffers do not fit) -- round 4 found these launches adding
    their phase timers through an uninitialised pointer (an aperture-violation fault)."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", SDFGEN_TILE_GRID="96", SDFGEN_TILE_CFG=str(cfg), SDFGEN_TILE_MULTI="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "slab_inprocess_check.py"),
                        "2", "40", "36", "44"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
