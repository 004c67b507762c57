"""Sign pass time per output layout (profile sign_ms): i-fastest Array3f vs k-fastest numpy/.sdf.
    python tools/sign_rate.py [WORKLOAD ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdfgenfast_amd import _hiprt, _lib, meshgen  # noqa: E402

for wl in sys.argv[1:] or ["c3_sphere1m_256"]:
    v, t, o, dx, dims = meshgen.workload(wl)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    out = _hiprt.DeviceBuffer(dims[0] * dims[1] * dims[2] * 4)
    for name, lay in (("array3", _lib.LAYOUT_ARRAY3), ("kfast", _lib.LAYOUT_KFAST)):
        best = None
        for _ in range(3):
            _lib.make_level_set3_device(0, dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, *dims, 1, lay, out.ptr, 0)
            p = _lib.last_profile()
            best = p if best is None or p["sign_ms"] < best["sign_ms"] else best
        print(f"{wl} {name:7s} sign {best['sign_ms']:.3f} ms  total {best['total_ms']:.3f} ms", flush=True)
    for b in (dv, dt, out):
        b.close()
