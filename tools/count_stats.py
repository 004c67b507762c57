import os, sys
sys.path.insert(0, "/root/repo")
os.environ["SDFGEN_COUNT_EVALS"] = "1"
from sdfgenfast_amd import _lib, meshgen
v, t, o, dx, dims = meshgen.workload("c3_sphere1m_256")
for r in range(2):
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
p = _lib.last_profile()
print({k: p[k] for k in ("sweep_evals", "sweep_stalls", "own_waits", "helper_polls", "band_evals", "sparse_rechecks")})
