"""Sweep diagnostics on the GPU: per-sweep times, evaluation and stall counts.
python tools/sweep_diag.py [workload] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sdfgen_amd import _lib, meshgen  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
v, t, o, dx, dims = meshgen.workload(name)
for mode in ("timing", "count"):
    if mode == "count":
        os.environ["SDFGEN_COUNT_EVALS"] = "1"
    for r in range(reps):
        t0 = time.perf_counter()
        _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
        el = time.perf_counter() - t0
        p = _lib.last_profile()
        print(f"{mode} rep{r}: wall {el*1e3:.1f} ms  total {p['total_ms']:.2f}  band {p['band_ms']:.2f}  "
              f"sweep {p['sweep_ms']:.2f}  sign {p['sign_ms']:.3f}  impl {p['sweep_impl']}  "
              f"band_evals {p['band_evals']}  sweep_evals {p['sweep_evals']}  stalls {p['sweep_stalls']} "
              f"(own {p['own_waits']})  helper_idle {p['helper_polls']}",
              flush=True)
    print("per-sweep ms:", [round(x, 3) for x in p["sweep_launch_ms"]], flush=True)
ncell = np.prod(dims)
print(f"cells {ncell}  sweep evals/cell/sweep = {p['sweep_evals']/ncell/16:.3f}")
