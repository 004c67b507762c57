"""ctypes front-end for the CPU parity checkers.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package (sdfgenfast_amd) never does.

* ``liboracle.so``  -- oracle/sdf_oracle.c, the C restatement of
  cpu_lib/makelevelset3.cpp:192-304 (single-thread semantics).
* ``_ref/libsdfref.so`` -- the reference's own cpu_lib/makelevelset3.cpp
  compiled from /root/reference by ``make -C oracle ref`` (``__graft_entry__.build``
  runs it where /root/reference exists).  The built library is git-ignored but
  travels with the working tree to the GPU box, where bench.py times it as the
  CPU baseline (kind "reference"); without it the baseline is the library's own
  native CPU backend on the same full workload (kind "port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ORACLE_SO = os.path.join(_HERE, "liboracle.so")
_REF_SO = os.path.join(_HERE, "_ref", "libsdfref.so")
_MESHREF_SO = os.path.join(_HERE, "_ref", "libmeshref.so")

_P = ctypes.c_void_p
_oracle = None
_ref = None
_meshref = None


def build(ref: bool = False) -> None:
    """Compile the C restatement (and, if asked and available, the reference)."""
    targets = ["all"] + (["ref"] if ref else [])
    subprocess.run(["make", "-s", "-C", _HERE] + targets, check=True)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


def lib():
    global _oracle
    if _oracle is None:
        if not os.path.exists(_ORACLE_SO):
            build()
        L = ctypes.CDLL(_ORACLE_SO)
        L.oracle_make_level_set3.argtypes = [_P, ctypes.c_uint64, _P, ctypes.c_uint64, _P, ctypes.c_float,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]
        L.oracle_make_level_set3.restype = ctypes.c_int
        L.oracle_band.argtypes = [_P, ctypes.c_uint64, _P, ctypes.c_uint64, _P, ctypes.c_float,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P]
        L.oracle_band.restype = ctypes.c_int
        L.oracle_band_mt.argtypes = L.oracle_band.argtypes + [ctypes.c_int]
        L.oracle_band_mt.restype = ctypes.c_int
        L.oracle_sweep.argtypes = [_P, _P, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   _P, _P, ctypes.c_int]
        L.oracle_sweep.restype = None
        L.oracle_sign.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P]
        L.oracle_sign.restype = None
        L.oracle_ptd_batch.argtypes = [ctypes.c_uint64, _P, _P]
        L.oracle_ptd_batch.restype = None
        L.oracle_pit2d_batch.argtypes = [ctypes.c_uint64, _P, _P]
        L.oracle_pit2d_batch.restype = None
        _oracle = L
    return _oracle


def ref_available() -> bool:
    return os.path.exists(_REF_SO)


def ref_lib():
    global _ref
    if _ref is None:
        if not os.path.exists(_REF_SO):
            raise FileNotFoundError(f"{_REF_SO} not built (needs /root/reference; `make -C oracle ref`)")
        L = ctypes.CDLL(_REF_SO)
        L.ref_make_level_set3.argtypes = [_P, ctypes.c_uint64, _P, ctypes.c_uint64, _P, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, _P]
        L.ref_make_level_set3.restype = ctypes.c_int
        L.ref_ptd_batch.argtypes = [ctypes.c_uint64, _P, _P]
        L.ref_ptd_batch.restype = None
        L.ref_pit2d_batch.argtypes = [ctypes.c_uint64, _P, _P]
        L.ref_pit2d_batch.restype = None
        _ref = L
    return _ref


def _prep(vertices, triangles, origin):
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(triangles, dtype=np.uint32).reshape(-1, 3)
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
    return v, t, o


def make_level_set3(vertices, triangles, origin, dx, ni, nj, nk, exact_band=1) -> np.ndarray:
    """Oracle phi, returned as a (ni, nj, nk) view of the i-fastest Array3f buffer
    (i.e. phi[i, j, k] == Array3f(i, j, k)); Fortran-ordered."""
    v, t, o = _prep(vertices, triangles, origin)
    out = np.empty(ni * nj * nk, dtype=np.float32)
    rc = lib().oracle_make_level_set3(_ptr(t), t.shape[0], _ptr(v), v.shape[0], _ptr(o),
                                      ctypes.c_float(dx), ni, nj, nk, exact_band, _ptr(out))
    if rc != 0:
        raise ValueError(f"oracle_make_level_set3 failed rc={rc}")
    return out.reshape((ni, nj, nk), order="F")


def band(vertices, triangles, origin, dx, ni, nj, nk, exact_band=1):
    """Stage 1 only: (phi, closest_tri, intersection_count), each (ni,nj,nk) F-order."""
    v, t, o = _prep(vertices, triangles, origin)
    n = ni * nj * nk
    phi = np.empty(n, np.float32)
    ct = np.empty(n, np.int32)
    cnt = np.empty(n, np.int32)
    rc = lib().oracle_band(_ptr(t), t.shape[0], _ptr(v), v.shape[0], _ptr(o), ctypes.c_float(dx),
                           ni, nj, nk, exact_band, _ptr(phi), _ptr(ct), _ptr(cnt))
    if rc != 0:
        raise ValueError(f"oracle_band failed rc={rc}")
    f = lambda a: a.reshape((ni, nj, nk), order="F")
    return f(phi), f(ct), f(cnt)


def band_mt(vertices, triangles, origin, dx, ni, nj, nk, exact_band=1, threads=None):
    """Stage 1 split over host threads by planes (oracle_band_mt) -- bit-identical to band();
    for parity cases with billions of band evaluations."""
    v, t, o = _prep(vertices, triangles, origin)
    n = ni * nj * nk
    phi = np.empty(n, np.float32)
    ct = np.empty(n, np.int32)
    cnt = np.empty(n, np.int32)
    if threads is None:
        threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64") or 64)))
    rc = lib().oracle_band_mt(_ptr(t), t.shape[0], _ptr(v), v.shape[0], _ptr(o), ctypes.c_float(dx),
                              ni, nj, nk, exact_band, _ptr(phi), _ptr(ct), _ptr(cnt), int(threads))
    if rc != 0:
        raise ValueError(f"oracle_band_mt failed rc={rc}")
    f = lambda a: a.reshape((ni, nj, nk), order="F")
    return f(phi), f(ct), f(cnt)


def sweep(vertices, triangles, origin, dx, phi, ct, nsweeps=16):
    """Stage 2 in place on F-ordered (ni,nj,nk) phi / ct arrays (returns copies)."""
    v, t, o = _prep(vertices, triangles, origin)
    ni, nj, nk = phi.shape
    p = np.asfortranarray(phi, dtype=np.float32).copy(order="F")
    c = np.asfortranarray(ct, dtype=np.int32).copy(order="F")
    lib().oracle_sweep(_ptr(t), _ptr(v), _ptr(o), ctypes.c_float(dx), ni, nj, nk,
                       p.ctypes.data_as(_P), c.ctypes.data_as(_P), nsweeps)
    return p, c


def ptd_batch(pts: np.ndarray) -> np.ndarray:
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 12)
    out = np.empty(pts.shape[0], np.float32)
    lib().oracle_ptd_batch(pts.shape[0], _ptr(pts), _ptr(out))
    return out


def pit2d_batch(pit: np.ndarray) -> np.ndarray:
    pit = np.ascontiguousarray(pit, dtype=np.float64).reshape(-1, 8)
    out = np.empty((pit.shape[0], 4), np.float64)
    lib().oracle_pit2d_batch(pit.shape[0], _ptr(pit), _ptr(out))
    return out


def ref_pit2d_batch(pit: np.ndarray) -> np.ndarray:
    pit = np.ascontiguousarray(pit, dtype=np.float64).reshape(-1, 8)
    out = np.empty((pit.shape[0], 4), np.float64)
    ref_lib().ref_pit2d_batch(pit.shape[0], _ptr(pit), _ptr(out))
    return out


def ref_make_level_set3(vertices, triangles, origin, dx, ni, nj, nk, exact_band=1, num_threads=1):
    """The REFERENCE implementation (built in the development container; bench.py's
    cpu_baseline also times it, multi-threaded, on the GPU box)."""
    v, t, o = _prep(vertices, triangles, origin)
    out = np.empty(ni * nj * nk, dtype=np.float32)
    ref_lib().ref_make_level_set3(_ptr(t), t.shape[0], _ptr(v), v.shape[0], _ptr(o), ctypes.c_float(dx),
                                  ni, nj, nk, exact_band, num_threads, _ptr(out))
    return out.reshape((ni, nj, nk), order="F")


def ref_ptd_batch(pts: np.ndarray) -> np.ndarray:
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 12)
    out = np.empty(pts.shape[0], np.float32)
    ref_lib().ref_ptd_batch(pts.shape[0], _ptr(pts), _ptr(out))
    return out


def meshref_available() -> bool:
    return os.path.exists(_MESHREF_SO)


def meshref_lib():
    global _meshref
    if _meshref is None:
        if not os.path.exists(_MESHREF_SO):
            raise FileNotFoundError(f"{_MESHREF_SO} not built (needs /root/reference; `make -C oracle ref`)")
        L = ctypes.CDLL(_MESHREF_SO)
        L.ref_mesh_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(_P)]
        L.ref_mesh_load.restype = ctypes.c_int
        L.ref_mesh_info.argtypes = [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), _P]
        L.ref_mesh_info.restype = None
        L.ref_mesh_copy.argtypes = [_P, _P, _P]
        L.ref_mesh_copy.restype = None
        L.ref_mesh_log.argtypes = [_P]
        L.ref_mesh_log.restype = ctypes.c_char_p
        L.ref_mesh_free.argtypes = [_P]
        L.ref_mesh_free.restype = None
        _meshref = L
    return _meshref


def ref_load_mesh(path: str):
    """The REFERENCE loader meshio::load_mesh (common/mesh_io.cpp:29-48) ->
    (rc, vertices (N,3) f32, triangles (M,3) u32, bounds (6,) f32 = min_box, max_box, log);
    rc 1 = loaded, 0 = the reference returned false, 2 = it threw (a bad OBJ face index).
    The vectors are whatever the reference left in them, also when it failed."""
    L = meshref_lib()
    h = _P()
    ok = L.ref_mesh_load(os.fsencode(path), ctypes.byref(h))
    try:
        nv, nt = ctypes.c_uint64(), ctypes.c_uint64()
        b = np.empty(6, np.float32)
        L.ref_mesh_info(h, ctypes.byref(nv), ctypes.byref(nt), _ptr(b))
        v = np.empty((nv.value, 3), np.float32)
        t = np.empty((nt.value, 3), np.uint32)
        L.ref_mesh_copy(h, _ptr(v), _ptr(t))
        log = L.ref_mesh_log(h).decode(errors="replace")
    finally:
        L.ref_mesh_free(h)
    return int(ok), v, t, b, log
