"""Repeated full calls with parity checks (diagnostics): python tools/stress.py WORKLOAD REPS"""
import hashlib, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _lib, meshgen
name, reps = sys.argv[1], int(sys.argv[2])
db = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "hashes.json")))
v, t, o, dx, dims = meshgen.workload(name)
bad = 0
t0 = time.time()
for r in range(reps):
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    h = hashlib.sha256(np.asfortranarray(got).ravel(order="F").astype("<f4").tobytes()).hexdigest()
    bad += h != db[name]["sha256_phi"]
print(f"{name}: {reps} calls, {bad} mismatches, {time.time() - t0:.1f} s, last {_lib.last_profile()['total_ms']:.2f} ms", flush=True)
sys.exit(1 if bad else 0)
