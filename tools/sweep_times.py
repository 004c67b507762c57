"""Per-sweep device times and sparse-repair statistics for one workload (diagnostics)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen

name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
v, t, o, dx, dims = meshgen.workload(name)
for rep in range(2):
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
p = _lib.last_profile()
print(json.dumps({k: p[k] for k in ("total_ms", "band_ms", "sweep_ms", "sweep_impl", "sparse_sweeps", "sparse_first",
                                    "sparse_rechecks", "sparse_claims")}))
print("per sweep ms:", " ".join(f"{x:.3f}" for x in p["sweep_launch_ms"]), flush=True)
