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

# per-task trace of one sweep (0 = first +++ sweep, 8 = first sweep of pass 2)
for sw in (0, 8):
    os.environ["SDFGEN_TRACE_SWEEP"] = str(sw)
    _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    tr = _lib.debug_sweep_trace().astype(np.int64)
    B = dims[1] - 1
    C = dims[2] - 1
    nJ = (B + 7) // 8
    nK = (C + 7) // 8
    order = [(J, d - J) for d in range(nJ + nK - 1) for J in range(nJ) if 0 <= d - J < nK]
    tr = tr[: len(order)]
    t0 = tr[:, 0].min()
    start = (tr[:, 0] - t0) / 100.0  # us
    end = (tr[:, 1] - t0) / 100.0
    dur = end - start
    pos = {jk: q for q, jk in enumerate(order)}
    print(f"sweep {sw}: span {end.max():.1f} us; task duration min/med/max {dur.min():.1f}/{np.median(dur):.1f}/{dur.max():.1f} us")
    for jk in [(0, 0), (1, 0), (0, 1), (1, 1), (2, 2), (4, 4), (8, 8), (16, 16), (nJ - 1, nK - 1)]:
        if jk in pos:
            q = pos[jk]
            print(f"   task {jk}: start {start[q]:8.1f}  end {end[q]:8.1f}  dur {dur[q]:7.1f} us")
    # how many tasks were active (started, not ended) over time
    ts = np.linspace(0, end.max(), 12)
    print("   active tasks over time:", [int(((start <= x) & (end > x)).sum()) for x in ts])
del os.environ["SDFGEN_TRACE_SWEEP"]
