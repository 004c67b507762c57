"""tools/step_prof.py under each tile configuration, with the step-profile library (tools/ab_build.sh prof
-DST_STEP_PROF):  python tools/step_prof_cfgs.py CFG [CFG ...] [WORKLOAD ...]   (SDFGEN_TILE_CFG values: the
leading numeric arguments)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfgs = [a for a in sys.argv[1:] if a.isdigit()]
wls = [a for a in sys.argv[1:] if not a.isdigit()]
for c in cfgs:
    env = dict(os.environ, SDFGEN_LIB_OVERRIDE=os.path.join(ROOT, "ab", "prof.so"), SDFGEN_COUNT_EVALS="1", SDFGEN_TILE_CFG=c)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_prof.py"), *wls], env=env,
                       capture_output=True, text=True, timeout=600)
    print(f"==== SDFGEN_TILE_CFG={c} (rc {r.returncode})", flush=True)
    print(r.stdout + r.stderr, flush=True)
