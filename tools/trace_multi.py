"""Timeline of the one-launch first pass (diagnostics; SDFGEN_TRACE_MULTI): per task its claim, start
(dependencies + setup done), first step and end, from the device wall clock (100 MHz).  Prints the
resident / computing task counts over time, each sweep's span, and the diagonal tiles' hand-off lags.
    python tools/trace_multi.py [WORKLOAD]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SDFGEN_TRACE_MULTI"] = "1"
import numpy as np  # noqa: E402

from sdfgenfast_amd import _lib, meshgen  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
v, t, o, dx, dims = meshgen.workload(name)
for _ in range(2):
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
p = _lib.last_profile()
B, C = dims[1] - 1, dims[2] - 1
ntasks = 8 * ((B + 7) // 8) * ((C + 7) // 8)
tr = _lib.debug_sweep_trace(max_entries=8 * ntasks).astype(np.int64).reshape(-1, 8)[:ntasks]
claim, start, first, end = tr[:, 7], tr[:, 0], tr[:, 1], tr[:, 3]
halo1, own1, step8 = tr[:, 2], tr[:, 4], tr[:, 5]   # first halo / own entries landed, step 8 done
sw, J, K = tr[:, 6] >> 32, (tr[:, 6] >> 16) & 0xffff, tr[:, 6] & 0xffff
t0 = claim.min()
us = lambda x: (x - t0) / 100.0
nsteps = dims[0] - 1 + 14
print(f"{name}: first-pass launch {p['sweep_launch_ms'][0]:.3f} ms, tile_cfg {p['tile_cfg']}, tasks {ntasks}, "
      f"span {us(end.max()):.1f} us, chain model {p['chain_steps']:.0f} steps")
ts = np.linspace(0, us(end.max()), 25)
print("resident (claimed, not ended):", [int(((us(claim) <= x) & (us(end) > x)).sum()) for x in ts])
print("computing (first step .. end): ", [int(((us(first) <= x) & (us(end) > x)).sum()) for x in ts])
print(f"claim -> start (deps + setup): median {np.median(start - claim) / 100:.1f} us, p90 {np.percentile(start - claim, 90) / 100:.1f}")
print(f"start -> first step: median {np.median(first - start) / 100:.1f} us, p90 {np.percentile(first - start, 90) / 100:.1f}")
print(f"us per step (first .. end): median {np.median((end - first) / 100 / nsteps):.2f}")
for q in range(8):
    m = sw == q
    print(f"sweep {q}: claims {us(claim[m].min()):8.1f} .. {us(claim[m].max()):8.1f}  first steps {us(first[m].min()):8.1f} .. "
          f"{us(first[m].max()):8.1f}  ends {us(end[m].min()):8.1f} .. {us(end[m].max()):8.1f} us")
    idx = {(int(j), int(k)): i for i, (j, k) in enumerate(zip(J[m], K[m]))}
    sub = np.nonzero(m)[0]
    lags = []
    for d in range(1, min(B, C) // 8):
        a, b = idx.get((d, d)), idx.get((d - 1, d - 1))
        if a is not None and b is not None:
            ia, ib = sub[a], sub[b]
            lags.append((us(first[ia]) - us(first[ib]), us(claim[ia]) - us(first[ib])))
    if lags:
        la = np.array(lags)
        print(f"    diagonal hop (J,J)->(J+1,J+1) first-step lag: median {np.median(la[:, 0]):.1f} us "
              f"(16 steps); claimed {np.median(la[:, 1]):+.1f} us after its upstream's first step")
    # one tile hop along the K = 0 row (its c-side is the boundary plane): (J-1, 0) -> (J, 0)
    hops = []
    for j in range(1, (B + 7) // 8):
        a, b = idx.get((j, 0)), idx.get((j - 1, 0))
        if a is None or b is None:
            continue
        ia, ib = sub[a], sub[b]
        hops.append(((first[ia] - first[ib]) / 100, (step8[ib] - first[ib]) / 100, (halo1[ia] - step8[ib]) / 100,
                     (first[ia] - halo1[ia]) / 100, (first[ia] - own1[ia]) / 100))
    if hops:
        h = np.median(np.array(hops), axis=0)
        print(f"    K=0 row hop (J-1,0)->(J,0): step-0 lag {h[0]:.1f} us = producer steps 0..8 {h[1]:.1f} + "
              f"halo landed {h[2]:+.1f} after producer step 8 + consumer step 0 {h[3]:+.1f} after the halo "
              f"(own entries landed {h[4]:.1f} us before step 0)")
