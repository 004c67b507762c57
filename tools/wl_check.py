"""Run one named workload (sdfgenfast_amd.meshgen.WORKLOADS) through the host entry point and check
it against the reference digest in tests/golden/hashes.json.  Diagnostics for a GPU session: the
environment picks the library (SDFGEN_LIB_OVERRIDE) and sweep variants (SDFGEN_*).
    python tools/wl_check.py WORKLOAD [REPEATS]"""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sdfgenfast_amd import _lib, meshgen  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rec = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "hashes.json"))).get(name)
v, t, o, dx, dims = meshgen.workload(name)
env = {k: v_ for k, v_ in os.environ.items() if k.startswith("SDFGEN_")}
for r in range(reps):
    t0 = time.perf_counter()
    try:
        phi = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    except Exception as e:  # reported, not raised: the next variant still runs
        print(f"{name} {env} ERROR {type(e).__name__}: {e}", flush=True)
        sys.exit(3)
    el = time.perf_counter() - t0
    h = hashlib.sha256(np.asfortranarray(phi).ravel(order="F").astype("<f4").tobytes()).hexdigest()
    p = _lib.last_profile()
    ok = rec is not None and h == rec["sha256_phi"]
    print(f"{name} {env} dims={dims} host {el*1e3:.2f} ms device {p['total_ms']:.3f} ms band {p['band_ms']:.3f} "
          f"sweep {p['sweep_ms']:.3f} evals {p['band_evals']} match={ok}", flush=True)
