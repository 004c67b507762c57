"""Step-profile diagnostics (build: tools/ab_build.sh prof -DST_STEP_PROF; run with
SDFGEN_LIB_OVERRIDE=ab/prof.so SDFGEN_COUNT_EVALS=1): the library prints where a compute
step's cycles go for the first-pass tile sweep launch.  Grids: the isolated one-tile grid
(bench.py step_latency) and the workloads named on the command line."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen

v, t = meshgen.bumpy_sphere(200, 61)
dims = (1024, 9, 9)
o, dx = meshgen.grid_mode2b(v, *dims, 2)
for _ in range(2):
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
    print("isolated", dims, "tile ms", round(_lib.last_profile()["sweep_launch_ms"][0], 3), flush=True)
for wl in sys.argv[1:]:
    v, t, o, dx, dims = meshgen.workload(wl)
    for _ in range(2):
        _lib.make_level_set3(v, t, o, dx, *dims, 1)
        print(wl, "tile ms", round(_lib.last_profile()["sweep_launch_ms"][0], 3), flush=True)
