"""Host-buffer (PCIe-inclusive) rate of sdfgen_hip_make_level_set3: host mesh in, host phi out.
python tools/host_rate.py [workload] [reps] -> one line per layout (Array3f i-fastest, numpy k-fastest)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _lib, meshgen

wl = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
v, t, o, dx, dims = meshgen.workload(wl)
n = dims[0] * dims[1] * dims[2]
for name, layout in (("array3 (i-fastest)", _lib.LAYOUT_ARRAY3), ("numpy (k-fastest)", _lib.LAYOUT_KFAST)):
    _lib.make_level_set3(v, t, o, dx, *dims, 1, layout)   # warm-up (allocations)
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.make_level_set3(v, t, o, dx, *dims, 1, layout)
        best = min(best, time.perf_counter() - t0)
    dev = _lib.last_profile()["total_ms"]
    print(f"{wl} {name}: host-to-host {best * 1e3:.2f} ms = {n / best / 1e6:.1f} Mvoxels/s "
          f"(device part {dev:.2f} ms; {12 * (v.shape[0] + t.shape[0]) / 1e6:.0f} MB in, {4 * n / 1e6:.0f} MB out)",
          flush=True)
