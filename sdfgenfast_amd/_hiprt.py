"""Minimal device-buffer plumbing through the HIP runtime libsdfgen_hip.so links.

Used by bench.py and the tests to hold inputs/outputs in HBM for the
device-resident entry point.  It deliberately binds the SAME libamdhip64.so.7
instance as the backend (dlopen by soname), so no second HIP runtime is
created in the process (torch wheels bundle their own).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib  # noqa: F401  (loads libsdfgen_hip.so and with it libamdhip64.so.7)

_rt = ctypes.CDLL("libamdhip64.so.7")
_rt.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
_rt.hipMalloc.restype = ctypes.c_int
_rt.hipFree.argtypes = [ctypes.c_void_p]
_rt.hipFree.restype = ctypes.c_int
_rt.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_rt.hipMemcpy.restype = ctypes.c_int
_rt.hipSetDevice.argtypes = [ctypes.c_int]
_rt.hipSetDevice.restype = ctypes.c_int
_rt.hipDeviceSynchronize.restype = ctypes.c_int

H2D, D2H = 1, 2


def set_device(dev: int) -> None:
    rc = _rt.hipSetDevice(int(dev))
    if rc != 0:
        raise RuntimeError(f"hipSetDevice({dev}) failed: {rc}")


def synchronize() -> None:
    rc = _rt.hipDeviceSynchronize()
    if rc != 0:
        raise RuntimeError(f"hipDeviceSynchronize failed: {rc}")


class DeviceBuffer:
    """A raw hipMalloc'd buffer (freed on close/GC)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        rc = _rt.hipMalloc(ctypes.byref(p), max(self.nbytes, 1))
        if rc != 0:
            raise MemoryError(f"hipMalloc({nbytes}) failed: {rc}")
        self.ptr = p.value

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        rc = _rt.hipMemcpy(self.ptr, a.ctypes.data, a.nbytes, H2D)
        if rc != 0:
            raise RuntimeError(f"hipMemcpy H2D failed: {rc}")

    def download(self, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        assert out.nbytes <= self.nbytes
        rc = _rt.hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H)
        if rc != 0:
            raise RuntimeError(f"hipMemcpy D2H failed: {rc}")
        return out

    def close(self) -> None:
        if self.ptr:
            _rt.hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
