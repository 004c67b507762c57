"""Repair-iteration profile (build: tools/ab_build.sh iterprof -DSP_ITER_PROF): the library prints, per
iteration of k_sp_recheck with >= 1 evaluating lane and per idle one, the cycles of each phase.
    python tools/iter_prof.py [WORKLOAD ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys; sys.path.insert(0, %r); from sdfgenfast_amd import _lib, meshgen; "
        "v, t, o, dx, dims = meshgen.workload(%r); [_lib.make_level_set3(v, t, o, dx, *dims, 1) for _ in range(2)]; "
        "print('second pass ms', sum(_lib.last_profile()['sweep_launch_ms'][8:]))")
for wl in sys.argv[1:] or ["c3_sphere1m_256"]:
    env = dict(os.environ, SDFGEN_LIB_OVERRIDE=os.path.join(ROOT, "ab", "iterprof.so"))
    r = subprocess.run([sys.executable, "-c", code % (ROOT, wl)], env=env, capture_output=True, text=True, timeout=600)
    print(f"==== {wl} (rc {r.returncode})\n" + r.stdout + r.stderr[-3000:], flush=True)
