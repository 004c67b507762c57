"""Mixed-size stress of the one-GPU host entry point (diagnostics): golden and edge fixtures, the
reference's benchmark grids and bumpy spheres, in a shuffled order, each result checked bit for bit.
Stops at the first error or mismatch and prints what ran before it.
    python tools/stress_mix.py SECONDS [SEED]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import EDGE_CASES, GOLDEN_CASES  # noqa: E402
from sdfgenfast_amd import _lib, meshgen  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
hashes = json.load(open(os.path.join(ROOT, "tests", "golden", "hashes.json")))
items = []
for c in GOLDEN_CASES + EDGE_CASES:
    want = np.ascontiguousarray(c.phi).view(np.uint32)
    items.append((c.name, c.vertices, c.triangles, c.origin, c.dx, c.dims, c.exact_band,
                  lambda got, w=want: np.array_equal(np.ascontiguousarray(got).view(np.uint32), w)))
for name in ("x3y4z5_prop64", "x3y4z5_prop128", "c2_sphere70k_128"):
    v, t, o, dx, dims = meshgen.workload(name)
    h = hashes[name]["sha256_phi"]
    chk = (lambda got, h=h: hashlib.sha256(np.asfortranarray(got).ravel(order="F").astype("<f4").tobytes()).hexdigest() == h)
    items.append((name, v, t, o, dx, dims, 1, chk))
    items.append((name, v, t, o, dx, dims, 1, chk))   # twice the weight
t_end = time.time() + secs
n = 0
hist = []
while time.time() < t_end:
    name, v, t, o, dx, dims, band, chk = items[int(rng.integers(len(items)))]
    n += 1
    hist.append(name)
    try:
        with np.errstate(all="ignore"):
            got = _lib.make_level_set3(v, t, o, dx, *dims, band, int(rng.integers(2)))   # either layout
    except Exception as e:
        print(f"ERROR at call {n} ({name} {dims}): {type(e).__name__}: {e}\nlast calls: {hist[-12:]}", flush=True)
        sys.exit(1)
    if not chk(got):
        print(f"MISMATCH at call {n} ({name} {dims})\nlast calls: {hist[-12:]}", flush=True)
        sys.exit(1)
    if n % 200 == 0:
        print(f"{n} calls ok", flush=True)
print(f"OK {n} calls", flush=True)
