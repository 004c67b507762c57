"""Diagnostics: the call time when the first pass's LAST sweeps also run as Jacobi + repair
(SDFGEN_SPARSE_FROM = 8, 7, 6, ...), with the repair statistics of each setting and a digest
check against the default split.
    python tools/sparse_from.py [WORKLOAD] [FROM ...]"""
import hashlib
import json
import os
import sys
import time

os.environ.setdefault("SDFGEN_SWEEP_EVENTS", "1")   # per-sweep times of the second-pass sweeps (before the first call)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sdfgenfast_amd import _lib, meshgen  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
froms = [int(x) for x in sys.argv[2:]] or [8, 7, 6, 5, 4]
v, t, o, dx, dims = meshgen.workload(name)
ref = None
for f in froms:
    os.environ["SDFGEN_SPARSE_FROM"] = str(f)
    ts = []
    for rep in range(6):
        phi = _lib.make_level_set3(v, t, o, dx, *dims, 1)
        ts.append(_lib.last_profile()["total_ms"])
    p = _lib.last_profile()
    dig = hashlib.sha256(np.ascontiguousarray(phi).tobytes()).hexdigest()[:16]
    ref = ref or dig
    print(f"from {f}: total {np.median(ts[2:]):.3f} ms (min {min(ts[2:]):.3f})  sweep {p['sweep_ms']:.3f}  rechecks {p['sparse_rechecks']} claims {p['sparse_claims']}  "
          f"digest {dig} {'OK' if dig == ref else 'MISMATCH'}", flush=True)
    print("   per sweep ms:", " ".join(f"{x:.3f}" for x in p["sweep_launch_ms"]), flush=True)
    print("JSON " + json.dumps({"workload": name, "from": f, "total_ms": float(np.median(ts[2:])), "sweep_ms": p["sweep_ms"],
                                "sweep_launch_ms": [round(x, 4) for x in p["sweep_launch_ms"]],
                                "rechecks": p["sparse_rechecks"], "claims": p["sparse_claims"], "tile_cfg": p["tile_cfg"],
                                "digest_ok": dig == ref}), flush=True)
