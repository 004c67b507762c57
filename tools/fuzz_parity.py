"""Time-bounded randomized parity check of the GPU path against the C oracle (diagnostics).
python tools/fuzz_parity.py SECONDS SEED [wide] -> one line per failure, a summary at the end.
Random triangle soups and bumpy spheres, random (ragged) grid sizes and band widths; "wide": rows of 2 to 700
cells on 2 to 24 rows and planes (several row segments of the second pass's k-streaming scan)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen

secs, seed = float(sys.argv[1]), int(sys.argv[2])
wide = len(sys.argv) > 3 and sys.argv[3] == "wide"
rng = np.random.default_rng(seed)
t_end = time.time() + secs
n = bad = cells = 0
t_note = time.time() + 30
while time.time() < t_end:
    if time.time() > t_note:   # progress line: a silent GPU command is taken for hung after 180 s
        print(f"... {n} cases, {bad} mismatches", flush=True)
        t_note = time.time() + 30
    if rng.random() < 0.5:
        nv = int(rng.integers(10, 3000))
        v = rng.normal(size=(nv, 3)).astype(np.float32)
        t = rng.integers(0, nv, size=(int(rng.integers(1, 4000)), 3)).astype(np.uint32)
    else:
        v, t = meshgen.bumpy_sphere(int(rng.integers(8, 200)), int(rng.integers(4, 80)))
    dims = tuple(int(x) for x in rng.integers(2, 90, size=3))
    if wide:
        dims = (int(rng.integers(2, 701)), int(rng.integers(2, 25)), int(rng.integers(2, 25)))
    o, dx = meshgen.grid_mode2b(v, max(dims[0], 4), max(dims[1], 4), max(dims[2], 4), int(rng.integers(0, 3)))
    if not (np.isfinite(dx) and dx > 0):
        continue
    band = int(rng.integers(0, 4))
    want = np.ascontiguousarray(O.make_level_set3(v, t, o, dx, *dims, exact_band=band))
    got = np.ascontiguousarray(_lib.make_level_set3(v, t, o, dx, *dims, band))
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    n += 1
    cells += got.size
    if not same.all():
        bad += 1
        print(f"MISMATCH case {n}: dims {dims} tris {t.shape[0]} band {band}: {(~same).sum()} cells", flush=True)
print(f"fuzz seed {seed}{' (wide rows)' if wide else ''}: {n} cases, {cells} cells, {bad} mismatches", flush=True)
sys.exit(1 if bad else 0)
