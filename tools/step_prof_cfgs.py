"""tools/step_prof.py under each tile configuration, with the step-profile library (tools/ab_build.sh prof
-DST_STEP_PROF):  python tools/step_prof_cfgs.py CFG [CFG ...] [WORKLOAD ...] [lib=NAME ...]   (SDFGEN_TILE_CFG
values: the numeric arguments; lib=NAME: profile ab/NAME.so instead of ab/prof.so, one run per library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfgs = [a for a in sys.argv[1:] if a.isdigit()]
libs = [a[4:] for a in sys.argv[1:] if a.startswith("lib=")] or ["prof"]
wls = [a for a in sys.argv[1:] if not a.isdigit() and not a.startswith("lib=")]
for c in cfgs:
    for lib in libs:
        env = dict(os.environ, SDFGEN_LIB_OVERRIDE=os.path.join(ROOT, "ab", lib + ".so"), SDFGEN_COUNT_EVALS="1",
                   SDFGEN_TILE_CFG=c)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "step_prof.py"), *wls], env=env,
                           capture_output=True, text=True, timeout=600)
        print(f"==== SDFGEN_TILE_CFG={c} ab/{lib}.so (rc {r.returncode})", flush=True)
        print(r.stdout + r.stderr, flush=True)
