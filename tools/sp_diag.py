"""Second-pass diagnostics: per-sweep launch times and repair counters of one workload
(run with SDFGEN_LIB_OVERRIDE=ab/spprof.so for the SP_PROF cycle split)."""
import sys, os
os.environ.setdefault("SDFGEN_SWEEP_EVENTS", "1")   # per-sweep launch times (the library's default times them together)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen

for wl in sys.argv[1:] or ["c3_sphere1m_256"]:
    v, t, o, dx, dims = meshgen.workload(wl)
    for _ in range(2):
        _lib.make_level_set3(v, t, o, dx, *dims, 1)
        p = _lib.last_profile()
        print(wl, "sparse sweeps ms", [round(x, 3) for x in p["sweep_launch_ms"][8:]], "rechecks", p["sparse_rechecks"],
              "claims", p["sparse_claims"], flush=True)
