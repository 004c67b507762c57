"""One C5-size call (1024^3 grid, 4M-triangle sphere) on one GPU: device time, phases, and the
reference digest check (tests/golden/hashes.json)."""
import hashlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _hiprt, _lib, meshgen

name = sys.argv[1] if len(sys.argv) > 1 else "c5_sphere4m_1024"
v, t, o, dx, dims = meshgen.workload(name)
ni, nj, nk = dims
dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
out = _hiprt.DeviceBuffer(ni * nj * nk * 4)
for r in range(2):
    _lib.make_level_set3_device(0, dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, ni, nj, nk, 1, _lib.LAYOUT_ARRAY3, out.ptr, 0)
    p = _lib.last_profile()
    print(f"{name} call {r}: total {p['total_ms']:.1f} ms band {p['band_ms']:.1f} tile {sum(p['sweep_launch_ms'][:8]):.1f} "
          f"sparse {sum(p['sweep_launch_ms'][8:]):.1f}", flush=True)
rec = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "hashes.json"))).get(name)
if rec:
    got = out.download(np.float32, ni * nj * nk)
    print("digest", "MATCH" if hashlib.sha256(got.astype("<f4").tobytes()).hexdigest() == rec["sha256_phi"] else "MISMATCH", flush=True)
