"""Run make_level_set3 REPS times on WORKLOAD with the current lib (under rocprofv3 for per-kernel A/B)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen
wl = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
v, t, o, dx, dims = meshgen.workload(wl)
for _ in range(reps):
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
print(wl, reps, "calls done", _lib.last_profile()["total_ms"])
