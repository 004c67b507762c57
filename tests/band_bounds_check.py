"""The band, ray-parity, sign and soup kernels on the bounds-checked library (run by
tests/test_gpu_bounds.py with SDFGEN_LIB_OVERRIDE=libsdfgen_hip_bounds.so; prints one line per case and
"OK <library>" at the end if every case matched and no index left its buffer).

Covers every index k_prep_soup, k_band_lds (the batch's pair -> triangle search, the LDS table, the
global flush), k_band_big, the ray-parity counts, k_sign and k_sign_kfast form (geom.hpp SDF_CHK sites
40-50, sdfgen_hip.hip): stage 1 of the golden and edge fixtures against oracle.band, coarse random soups
(both work classes in one call), and whole calls in both output layouts against the reference's output.
An out-of-range index makes the library return an error naming the site, so it fails here as an
exception instead of faulting the GPU."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from conftest import EDGE_CASES, GOLDEN_CASES, bits_equal  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import _lib  # noqa: E402


def stage1_equal(got, want):
    phi, ct, cnt, _ = got
    wphi, wct, wcnt = want
    return (np.array_equal(np.asarray(phi).view(np.uint32), np.asarray(wphi).view(np.uint32))
            and np.array_equal(ct, wct) and np.array_equal(cnt.astype(np.int64), wcnt.astype(np.int64)))


def main():
    bad = 0
    for c in GOLDEN_CASES + EDGE_CASES:
        with np.errstate(all="ignore"):
            want = O.band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, exact_band=c.exact_band)
            got = _lib.debug_band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band)
        ok = stage1_equal(got, want)
        for layout in (_lib.LAYOUT_ARRAY3, _lib.LAYOUT_KFAST):
            out = _lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, layout)
            ok = ok and bits_equal(out, c.phi)
        print(("ok   " if ok else "FAIL ") + c.name)
        bad += not ok
    for seed in range(4):   # coarse soups with bands 0-6: batched and big triangles in one call
        rng = np.random.default_rng(7000 + seed)
        nt = int(rng.integers(20, 200))
        v = rng.uniform(-1, 1, size=(nt * 2, 3)).astype(np.float32)
        t = rng.integers(0, len(v), size=(nt, 3)).astype(np.uint32)
        dims = tuple(int(x) for x in rng.integers(24, 40, size=3))   # (large enough for big triangles)
        o = np.array([-1.1, -1.1, -1.1], np.float32)
        dx = float(np.float32(2.2 / min(dims)))
        band = int(rng.integers(2, 7))
        want = O.band(v, t, o, dx, *dims, exact_band=band)
        got = _lib.debug_band(v, t, o, dx, *dims, band)
        same = stage1_equal(got, want)
        ok = same and got[3] > 0   # (the big-triangle list was exercised)
        print(("ok   " if ok else "FAIL ") + f"coarse seed {seed} dims {dims} band {band} big {got[3]} stage1 {'equal' if same else 'DIFFERS'}")
        bad += not ok
    print(("OK " if bad == 0 else f"MISMATCH {bad} ") + _lib.LIB_PATH)


if __name__ == "__main__":
    main()
