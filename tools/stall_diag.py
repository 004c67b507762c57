"""First-pass wait breakdown (SDFGEN_COUNT_EVALS=1): compute-wave polls, of them the ones waiting
for the helper's own-column data, and helper idle polls, for the isolated tile and a workload."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen  # noqa: E402

cases = [("isolated", *meshgen.bumpy_sphere(200, 61), (1024, 9, 9))]
for wl in sys.argv[1:]:
    v, t, o, dx, dims = meshgen.workload(wl)
    cases.append((wl, v, t, dims))
for name, v, t, dims in cases:
    o, dx = meshgen.grid_mode2b(v, *dims, 2) if name == "isolated" else meshgen.workload(name)[2:4]
    for _ in range(2):
        _lib.make_level_set3(v, t, o, dx, *dims, 1)
    p = _lib.last_profile()
    print(f"{name}: tile ms {p['sweep_launch_ms'][0]:.3f} evals {p['sweep_evals']} compute polls {p['sweep_stalls']} "
          f"(own-data waits {p['own_waits']}) helper idle polls {p['helper_polls']}", flush=True)
