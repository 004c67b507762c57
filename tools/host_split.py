"""Where the host-buffer call's time goes (C3): the whole host call, its device part, and the raw
PCIe copies of the same sizes (pageable and pinned) and a host memcpy of the output size.
python tools/host_split.py [workload]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sdfgenfast_amd import _lib, meshgen

wl = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
v, t, o, dx, dims = meshgen.workload(wl)
n = dims[0] * dims[1] * dims[2]
out = np.empty(n, np.float32)


def best(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, sorted(ts)[len(ts) // 2] * 1e3


h = best(lambda: _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out))
dev = _lib.last_profile()["total_ms"]
print(f"host call: best {h[0]:.3f} median {h[1]:.3f} ms; device part (last call) {dev:.3f} ms", flush=True)
d_out = torch.empty(n, dtype=torch.float32, device="cuda")
page = torch.from_numpy(out)
pin = torch.empty(n, dtype=torch.float32, pin_memory=True)


def d2h(dst):
    dst.copy_(d_out)
    torch.cuda.synchronize()


r = best(lambda: d2h(page)); print(f"D2H {4 * n / 1e6:.0f} MB pageable: {r[0]:.3f} ms ({4 * n / r[0] / 1e6:.1f} GB/s)", flush=True)
r = best(lambda: d2h(pin)); print(f"D2H {4 * n / 1e6:.0f} MB pinned:   {r[0]:.3f} ms ({4 * n / r[0] / 1e6:.1f} GB/s)", flush=True)
src = np.empty_like(out); src[:] = 1.0
r = best(lambda: np.copyto(out, src)); print(f"host memcpy {4 * n / 1e6:.0f} MB (1 thread): {r[0]:.3f} ms", flush=True)
nin = 12 * (v.shape[0] + t.shape[0])
hin = torch.from_numpy(np.ones(nin // 4, np.float32)); din = torch.empty(nin // 4, dtype=torch.float32, device="cuda")


def h2d():
    din.copy_(hin)
    torch.cuda.synchronize()


r = best(h2d); print(f"H2D {nin / 1e6:.0f} MB pageable: {r[0]:.3f} ms", flush=True)
del d_out, din, pin
if len(sys.argv) > 2:   # the same host call after a larger grid grew the workspace (bench's order)
    v4, t4, o4, dx4, dims4 = meshgen.workload(sys.argv[2])
    _lib.make_level_set3(v4, t4, o4, dx4, *dims4, 1)
    h = best(lambda: _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out))
    print(f"host call after {sys.argv[2]}: best {h[0]:.3f} median {h[1]:.3f} ms; device part {_lib.last_profile()['total_ms']:.3f} ms", flush=True)
