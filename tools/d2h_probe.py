"""PCIe copy paths of the ROCm 7.2 runtime the library links (no torch in the process): pageable
hipMemcpy D2H / H2D, the same after hipHostRegister of the host buffer (register + copy + unregister
timed together, and the copy alone), and into hipHostMalloc'd memory.  python tools/d2h_probe.py [MB]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _hiprt

rt = _hiprt._rt
rt.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
rt.hipHostUnregister.argtypes = [ctypes.c_void_p]
rt.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
mb = float(sys.argv[1]) if len(sys.argv) > 1 else 67.1
n = int(mb * 1e6) // 4 * 4
d = _hiprt.DeviceBuffer(n)
h = np.ones(n // 4, np.float32)
hp = h.ctypes.data


def best(f, reps=7):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    ts.sort()
    return f"best {ts[0] * 1e3:.3f} ms ({n / ts[0] / 1e9:.1f} GB/s), median {ts[len(ts) // 2] * 1e3:.3f} ms"


print(f"{n / 1e6:.1f} MB  GPU_PINNED_MIN_XFER_SIZE={os.environ.get('GPU_PINNED_MIN_XFER_SIZE')}", flush=True)
print("D2H pageable           ", best(lambda: rt.hipMemcpy(hp, d.ptr, n, 2)), flush=True)
print("H2D pageable           ", best(lambda: rt.hipMemcpy(d.ptr, hp, n, 1)), flush=True)


def reg_copy(kind):
    assert rt.hipHostRegister(hp, n, 0) == 0
    rt.hipMemcpy(hp, d.ptr, n, 2) if kind == 2 else rt.hipMemcpy(d.ptr, hp, n, 1)
    rt.hipHostUnregister(hp)


print("D2H register+copy+unreg", best(lambda: reg_copy(2)), flush=True)
print("H2D register+copy+unreg", best(lambda: reg_copy(1)), flush=True)
assert rt.hipHostRegister(hp, n, 0) == 0
print("D2H registered (copy)  ", best(lambda: rt.hipMemcpy(hp, d.ptr, n, 2)), flush=True)
rt.hipHostUnregister(hp)
p = ctypes.c_void_p()
assert rt.hipHostMalloc(ctypes.byref(p), n, 0) == 0
print("D2H hipHostMalloc      ", best(lambda: rt.hipMemcpy(p.value, d.ptr, n, 2)), flush=True)
src = np.empty_like(h)
print("host memcpy (1 thread) ", best(lambda: np.copyto(h, src)), flush=True)
