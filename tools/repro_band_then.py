"""Diagnostics: which earlier calls make the next x3y4z5_prop64 call go wrong (round 4).
    python tools/repro_band_then.py VARIANT
VARIANT: dband_all | whole_all | dband_golden | dband_edge | dband_coarse | whole_coarse"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import EDGE_CASES, GOLDEN_CASES  # noqa: E402
from sdfgenfast_amd import _lib, meshgen  # noqa: E402

variant = sys.argv[1]


def coarse(seed):   # tests/test_gpu_band.py::test_band_stage1_coarse_random's inputs
    rng = np.random.default_rng(1000 + seed)
    nt = int(rng.integers(20, 300))
    v = rng.uniform(-1, 1, size=(nt * 2, 3)).astype(np.float32)
    t = rng.integers(0, len(v), size=(nt, 3)).astype(np.uint32)
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
    return v, t, o, dx, dims, int(rng.integers(0, 7))


if variant in ("dband_coarse", "whole_coarse"):
    for seed in range(8):
        v, t, o, dx, dims, band = coarse(seed)
        if variant == "dband_coarse":
            _lib.debug_band(v, t, o, dx, *dims, band)
        else:
            _lib.make_level_set3(v, t, o, dx, *dims, band, _lib.LAYOUT_KFAST)
cases = {"dband_all": GOLDEN_CASES + EDGE_CASES, "whole_all": GOLDEN_CASES + EDGE_CASES,
         "dband_golden": GOLDEN_CASES, "dband_edge": EDGE_CASES}.get(variant, [])
for c in cases:
    with np.errstate(all="ignore"):
        if variant.startswith("dband"):
            _lib.debug_band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band)
        else:
            _lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, _lib.LAYOUT_KFAST)
rec = json.load(open(os.path.join(ROOT, "tests", "golden", "hashes.json")))
for name in ("x3y4z5_prop64", "x3y4z5_prop64", "c2_sphere70k_128"):
    v, t, o, dx, d = meshgen.workload(name)
    try:
        got = _lib.make_level_set3(v, t, o, dx, *d, 1, _lib.LAYOUT_ARRAY3)
    except Exception as e:
        print(f"{variant}: {name} ERROR {e}", flush=True)
        continue
    h = hashlib.sha256(np.asfortranarray(got).ravel(order="F").astype("<f4").tobytes()).hexdigest()
    print(f"{variant}: {name} {'ok' if h == rec[name]['sha256_phi'] else 'MISMATCH'}", flush=True)
