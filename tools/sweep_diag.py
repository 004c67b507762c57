"""Sweep diagnostics on the GPU: per-sweep times, evaluation and stall counts.
python tools/sweep_diag.py [workload] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sdfgenfast_amd import _lib, meshgen  # noqa: E402

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
for grid in ("",):
    if grid:
        os.environ["SDFGEN_TILE_GRID"] = grid
    for sw in (0, 8):
        os.environ["SDFGEN_TRACE_SWEEP"] = str(sw)
        _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
        p = _lib.last_profile()
        tr = _lib.debug_sweep_trace().astype(np.int64)
        B = dims[1] - 1
        C = dims[2] - 1
        nJ = (B + 7) // 8
        nK = (C + 7) // 8
        order = [(J, d - J) for d in range(nJ + nK - 1) for J in range(nJ) if 0 <= d - J < nK]
        tr = tr[: len(order)]
        t0 = tr[:, 0].min()
        st = (tr[:, :4] - t0) / 100.0  # us: start, first step, mid, end
        wt = tr[:, 4] / 100.0          # us waiting in polls
        wo, wh = tr[:, 5] & 0xffffffff, tr[:, 5] >> 32   # steps that waited on own data / on halo
        clk = tr[:, 6] / np.maximum(tr[:, 7], 1) / 10.0  # shader clock (GHz) during compute
        pos = {jk: q for q, jk in enumerate(order)}
        nsteps = dims[0] - 1 + 14
        half = nsteps / 2
        print(f"grid={grid or 'auto'} sweep {sw}: sweep_ms {p['sweep_launch_ms'][sw]:.3f} span {st[:, 3].max():.1f} us")
        for jk in [(0, 0), (1, 0), (2, 2), (4, 4), (6, 6), (8, 8), (12, 12), (16, 16), (24, 24), (nJ - 1, nK - 1)]:
            if jk in pos:
                q = pos[jk]
                s0, s1, s2, s3 = st[q]
                print(f"   task {jk}: start {s0:7.1f} first {s1:7.1f} mid {s2:7.1f} end {s3:7.1f}  "
                      f"us/step 1st half {(s2 - s1) / half:5.2f}  2nd half {(s3 - s2) / half:5.2f}  "
                      f"wait {wt[q]:7.1f} us (own {wo[q]}, halo {wh[q]} steps)  "
                      f"busy/step {((s3 - s0) - wt[q]) / nsteps:5.2f}  compute/step {tr[q, 7] / 100.0 / nsteps:5.2f}  clk {clk[q]:.2f} GHz")
    os.environ.pop("SDFGEN_TILE_GRID", None)
del os.environ["SDFGEN_TRACE_SWEEP"]
