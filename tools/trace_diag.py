"""Tile-wavefront timeline: first/last step of the diagonal tasks of one sweep."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _lib, meshgen
name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
sw = int(sys.argv[2]) if len(sys.argv) > 2 else 0
v, t, o, dx, dims = meshgen.workload(name)
os.environ["SDFGEN_SPARSE_FROM"] = "16"
os.environ["SDFGEN_TRACE_SWEEP"] = str(sw)
_lib.make_level_set3(v, t, o, dx, *dims, 1)
_lib.make_level_set3(v, t, o, dx, *dims, 1)
p = _lib.last_profile()
tr = _lib.debug_sweep_trace().astype(np.int64)
B, C = dims[1] - 1, dims[2] - 1
nJ, nK = (B + 7) // 8, (C + 7) // 8
order = [(J, d - J) for d in range(nJ + nK - 1) for J in range(nJ) if 0 <= d - J < nK]
tr = tr[: len(order)]
t0 = tr[:, 0].min()
st = (tr[:, :4] - t0) / 100.0
pos = {jk: q for q, jk in enumerate(order)}
nsteps = dims[0] - 1 + 14
print(f"sweep {sw}: {p['sweep_launch_ms'][sw]:.3f} ms, span {st[:, 3].max():.1f} us, tasks {len(order)}")
prev = None
for J in range(nJ):
    q = pos[(J, J)]
    s0, s1, s2, s3 = st[q]
    lag = f"{s1 - prev:6.1f}" if prev is not None else "     -"
    print(f"  ({J:2d},{J:2d}) start {s0:8.1f} first {s1:8.1f} (+{lag}) end {s3:8.1f}  dur {s3 - s1:7.1f} "
          f"us/step {(s3 - s1) / nsteps:5.2f} wait {tr[q, 4] / 100:7.1f} compute/step {tr[q, 7] / 100.0 / nsteps:5.2f} "
          f"waits own/other {tr[q, 5] & 0xffffffff}/{tr[q, 5] >> 32}")
    prev = s1
# concurrency profile: number of tasks between first and end over time
ts = np.linspace(0, st[:, 3].max(), 12)
print("active tasks over time:", [int(((st[:, 1] <= x) & (st[:, 3] >= x)).sum()) for x in ts])
