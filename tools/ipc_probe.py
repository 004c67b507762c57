"""Probe: can HIP IPC export device memory allocated with hipExtMallocWithFlags flags?"""
import ctypes
hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
for name, flag in [("coarse hipMalloc", None), ("finegrained", 1), ("uncached", 3)]:
    p = ctypes.c_void_p()
    if flag is None:
        rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
    else:
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(flag))
    h = (ctypes.c_char * 64)()
    rc2 = hip.hipIpcGetMemHandle(h, p)
    print(f"{name}: malloc rc={rc} ipc rc={rc2}", flush=True)
