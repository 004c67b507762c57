"""ctypes binding of the C-ABI in include/sdfgen_hip.h (libsdfgen_hip.so, built in-tree).

The product path: every generate call goes through this library.  There is no
CPU fallback here -- if the shared library is missing, importing this module
raises ImportError, and a GPU request without a usable device raises
RuntimeError (the reference's "GPU requested but unavailable" contract,
common/sdfgen_unified.cpp:60-63; python/tests/test_sdfgen.py:1030-1049).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDFGEN_LIB_OVERRIDE") or os.path.join(_HERE, "libsdfgen_hip.so")   # override: diagnostics only

OK, EINVAL, EINDEX, ENODEV, ERUNTIME, ENOMEM = 0, -1, -2, -3, -4, -5
LAYOUT_ARRAY3, LAYOUT_KFAST = 0, 1
NGPU_ALL, NGPU_CURRENT = 0, 1      # sdfgen_hip_make_level_set3 ngpu (include/sdfgen_hip.h)

_P = ctypes.c_void_p
_u64 = ctypes.c_uint64

# Every symbol include/sdfgen_hip.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "sdfgen_hip_abi_version",
    "sdfgen_hip_build_id",
    "sdfgen_hip_device_count",
    "sdfgen_hip_topology",
    "sdfgen_hip_make_level_set3",
    "sdfgen_hip_make_level_set3_device",
    "sdfgen_hip_last_profile",
    "sdfgen_hip_release",
    "sdfgen_hip_debug_ptd",
    "sdfgen_hip_debug_pit2d",
    "sdfgen_hip_debug_band",
    "sdfgen_cpu_make_level_set3",
    "sdfgen_hip_debug_sweep_trace",
    "sdfgen_hip_slab_create",
    "sdfgen_hip_slab_range",
    "sdfgen_hip_slab_export",
    "sdfgen_hip_slab_connect_ipc",
    "sdfgen_hip_slab_connect_local",
    "sdfgen_hip_slab_enqueue",
    "sdfgen_hip_slab_finish",
    "sdfgen_hip_slab_run",
    "sdfgen_hip_slab_destroy",
    "sdfgen_hip_slab_prepare",
    "sdfgen_hip_slab_close_imports",
    "sdfgen_hip_slab_debug_dump",
    "sdfgen_cpu_slab_create",
    "sdfgen_cpu_slab_range",
    "sdfgen_cpu_slab_band",
    "sdfgen_cpu_slab_sweep",
    "sdfgen_cpu_slab_sign",
    "sdfgen_cpu_slab_destroy",
    "sdfgen_mesh_load",
    "sdfgen_mesh_info",
    "sdfgen_mesh_copy",
    "sdfgen_mesh_free",
)
IPC_HANDLE_BYTES = 64


class Profile(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double),
        ("prep_ms", ctypes.c_double),
        ("band_ms", ctypes.c_double),
        ("sweep_ms", ctypes.c_double),
        ("sign_ms", ctypes.c_double),
        ("sweep_launch_ms", ctypes.c_double * 16),
        ("sweep_launches", ctypes.c_int),
        ("sweep_impl", ctypes.c_int),
        ("band_evals", ctypes.c_uint64),
        ("sweep_evals", ctypes.c_uint64),
        ("sweep_stalls", ctypes.c_uint64),
        ("helper_polls", ctypes.c_uint64),
        ("own_waits", ctypes.c_uint64),
        ("sparse_sweeps", ctypes.c_int),
        ("sparse_first", ctypes.c_int),
        ("sparse_rechecks", ctypes.c_uint64),
        ("sparse_claims", ctypes.c_uint64),
        ("tile_multi", ctypes.c_int),
        ("slabs", ctypes.c_int),
        ("chain_steps", ctypes.c_double),
        ("slab_wait_done_ms", ctypes.c_double * 8),
        ("slab_wait_ready_ms", ctypes.c_double * 8),
        ("slab_repair_ms", ctypes.c_double * 8),
        ("slab_inbound_ms", ctypes.c_double * 8),
        ("slab_inbound_entries", ctypes.c_uint64 * 8),
        ("slab_inbox_idle_ms", ctypes.c_double),
        ("slab_other_idle_ms", ctypes.c_double),
        ("slab_inbox_tasks", ctypes.c_uint64),
        ("slab_other_tasks", ctypes.c_uint64),
        ("tile_cfg", ctypes.c_int),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        for f, t in self._fields_:
            if hasattr(t, "_length_"):
                d[f] = list(getattr(self, f))
        return d


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP backend first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C sdfgenfast_amd)")
    L = ctypes.CDLL(LIB_PATH)
    L.sdfgen_hip_abi_version.restype = ctypes.c_int
    L.sdfgen_hip_build_id.restype = ctypes.c_char_p
    L.sdfgen_hip_device_count.restype = ctypes.c_int
    if hasattr(L, "sdfgen_hip_topology"):   # (absent from pre-ABI-4 libraries loaded for A/B comparisons)
        L.sdfgen_hip_topology.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), _P, _P]
        L.sdfgen_hip_topology.restype = ctypes.c_int
    L.sdfgen_hip_make_level_set3.argtypes = [_P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P,
                                             ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_hip_make_level_set3.restype = ctypes.c_int
    L.sdfgen_hip_make_level_set3_device.argtypes = [ctypes.c_int, _P, _u64, _P, _u64, _P, ctypes.c_float,
                                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int, _P, _P, ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_hip_make_level_set3_device.restype = ctypes.c_int
    L.sdfgen_hip_last_profile.argtypes = [ctypes.POINTER(Profile)]
    L.sdfgen_hip_last_profile.restype = ctypes.c_int
    L.sdfgen_hip_release.restype = ctypes.c_int
    if hasattr(L, "sdfgen_hip_slab_close_imports"):   # (absent from pre-ABI-5 libraries loaded for A/B runs)
        L.sdfgen_hip_slab_close_imports.restype = ctypes.c_int
    L.sdfgen_cpu_make_level_set3.argtypes = [_P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P,
                                             ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_cpu_make_level_set3.restype = ctypes.c_int
    L.sdfgen_hip_debug_ptd.argtypes = [ctypes.c_int, ctypes.c_int, _u64, _P, _P, ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_hip_debug_ptd.restype = ctypes.c_int
    L.sdfgen_hip_debug_pit2d.argtypes = [ctypes.c_int, _u64, _P, _P, ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_hip_debug_pit2d.restype = ctypes.c_int
    if hasattr(L, "sdfgen_hip_debug_band"):   # (absent from A/B builds of older sources)
        L.sdfgen_hip_debug_band.argtypes = [_P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, _P, _P, _P, ctypes.POINTER(_u64),
                                            ctypes.c_char_p, ctypes.c_size_t]
        L.sdfgen_hip_debug_band.restype = ctypes.c_int
    L.sdfgen_hip_debug_sweep_trace.argtypes = [ctypes.c_int, _P, _u64, ctypes.POINTER(_u64)]
    L.sdfgen_hip_debug_sweep_trace.restype = ctypes.c_int
    _E = [ctypes.c_char_p, ctypes.c_size_t]
    L.sdfgen_hip_slab_create.argtypes = [ctypes.c_int] * 6 + [ctypes.POINTER(_P)] + _E
    L.sdfgen_hip_slab_range.argtypes = [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.sdfgen_hip_slab_export.argtypes = [_P, _P] + _E
    L.sdfgen_hip_slab_connect_ipc.argtypes = [_P, _P, _P] + _E
    L.sdfgen_hip_slab_connect_local.argtypes = [_P, _P, _P] + _E
    L.sdfgen_hip_slab_enqueue.argtypes = [_P, _P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                          _P] + _E
    L.sdfgen_hip_slab_finish.argtypes = [_P, _u64, ctypes.POINTER(Profile)] + _E
    L.sdfgen_hip_slab_run.argtypes = [_P, _P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int, ctypes.c_int, _P,
                                      ctypes.POINTER(Profile)] + _E
    L.sdfgen_hip_slab_destroy.argtypes = [_P]
    L.sdfgen_hip_slab_debug_dump.argtypes = [_P, ctypes.c_int, _P, _u64, ctypes.POINTER(_u64)]
    L.sdfgen_hip_slab_prepare.argtypes = [_P, _u64] + _E
    for f in ("create", "range", "export", "connect_ipc", "connect_local", "enqueue", "finish", "run", "destroy",
              "debug_dump", "prepare"):
        getattr(L, "sdfgen_hip_slab_" + f).restype = ctypes.c_int
    L.sdfgen_cpu_slab_create.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(_P)] + _E
    L.sdfgen_cpu_slab_range.argtypes = [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.sdfgen_cpu_slab_band.argtypes = [_P, _P, _u64, _P, _u64, _P, ctypes.c_float, ctypes.c_int] + _E
    L.sdfgen_cpu_slab_sweep.argtypes = [_P, ctypes.c_int, _P, _P] + _E
    L.sdfgen_cpu_slab_sign.argtypes = [_P, ctypes.c_int, _P] + _E
    L.sdfgen_cpu_slab_destroy.argtypes = [_P]
    for f in ("create", "range", "band", "sweep", "sign", "destroy"):
        getattr(L, "sdfgen_cpu_slab_" + f).restype = ctypes.c_int
    L.sdfgen_mesh_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(_P)] + _E
    L.sdfgen_mesh_info.argtypes = [_P, ctypes.POINTER(_u64), ctypes.POINTER(_u64), _P, ctypes.POINTER(ctypes.c_int)]
    L.sdfgen_mesh_copy.argtypes = [_P, _P, _P]
    L.sdfgen_mesh_free.argtypes = [_P]
    for f in ("load", "info", "copy", "free"):
        getattr(L, "sdfgen_mesh_" + f).restype = ctypes.c_int
    return L


lib = _load()


class HipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def _raise(code: int, buf) -> None:
    msg = buf.value.decode(errors="replace") if buf is not None else ""
    if code == EINVAL:
        raise ValueError(msg or "invalid argument")
    if code == EINDEX:
        raise IndexError(msg or "triangle vertex index out of range")
    if code == ENODEV:
        raise RuntimeError(msg or "GPU backend requested but no HIP GPU is available")
    raise HipError(code, msg or f"GPU (HIP) backend error {code}")


MESH_AUTO, MESH_OBJ, MESH_STL, MESH_STL_BINARY, MESH_STL_ASCII = 0, 1, 2, 3, 4


def mesh_load(path: str, fmt: int = MESH_AUTO):
    """Native mesh loader (include/sdfgen_meshio.h) -> (vertices (n,3) f32, triangles (m,3) u32,
    bounds (min xyz, max xyz) as float32, detected format).  Raises RuntimeError on failure,
    like the reference's loaders returning false (common/mesh_io.cpp:29-48)."""
    h = _P()
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_mesh_load(os.fsencode(path), int(fmt), ctypes.byref(h), err, ctypes.sizeof(err))
    if rc != OK:
        raise RuntimeError(err.value.decode(errors="replace") or f"Failed to load mesh: {path}")
    try:
        nv, nt, f = _u64(), _u64(), ctypes.c_int()
        b = np.empty(6, np.float32)
        lib.sdfgen_mesh_info(h, ctypes.byref(nv), ctypes.byref(nt), b.ctypes.data_as(_P), ctypes.byref(f))
        v = np.empty((nv.value, 3), np.float32)
        t = np.empty((nt.value, 3), np.uint32)
        lib.sdfgen_mesh_copy(h, v.ctypes.data_as(_P), t.ctypes.data_as(_P))
    finally:
        lib.sdfgen_mesh_free(h)
    return v, t, b, f.value


def build_id() -> str:
    """The loaded library's build identity (sdfgen_hip_build_id: SHA-256 prefix of its sources)."""
    return lib.sdfgen_hip_build_id().decode()


def device_count() -> int:
    return int(lib.sdfgen_hip_device_count())


PCI_ID_BYTES = 32   # SDFGEN_HIP_PCI_ID_BYTES


def topology(max_dev: int = 16) -> dict:
    """sdfgen_hip_topology: the visible devices' PCI bus ids and the hipDeviceCanAccessPeer matrix
    (bench.py --gpus N records it, so that a mapping failure on a multi-GPU node names the pair)."""
    n = ctypes.c_int(0)
    ids = ctypes.create_string_buffer(PCI_ID_BYTES * max_dev)
    peer = (ctypes.c_int * (max_dev * max_dev))()
    rc = lib.sdfgen_hip_topology(max_dev, ctypes.byref(n), ids, peer)
    if rc:
        raise RuntimeError(f"sdfgen_hip_topology failed ({rc})")
    m = min(n.value, max_dev)
    pci = [ids.raw[PCI_ID_BYTES * i:PCI_ID_BYTES * (i + 1)].split(b"\0", 1)[0].decode() for i in range(m)]
    return {"devices": n.value, "pci_bus_ids": pci,
            "peer_access": [[int(peer[i * max_dev + j]) for j in range(m)] for i in range(m)]}


def make_level_set3(vertices: np.ndarray, triangles: np.ndarray, origin, dx: float, ni: int, nj: int, nk: int,
                    exact_band: int = 1, layout: int = LAYOUT_KFAST, ngpu: int = 1,
                    out: np.ndarray | None = None) -> np.ndarray:
    """Host-memory entry (sdfgen_hip_make_level_set3).  Returns phi as a (ni,nj,nk)
    array: C-ordered for LAYOUT_KFAST, a Fortran-ordered view of the i-fastest
    Array3f buffer for LAYOUT_ARRAY3 -- either way phi[i, j, k].  `out`: an optional
    contiguous float32 buffer of ni*nj*nk elements to write into (reused across calls)."""
    v = np.ascontiguousarray(vertices, dtype=np.float32)
    t = np.ascontiguousarray(triangles, dtype=np.uint32)
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
    if out is None:
        out = np.empty(int(ni) * int(nj) * int(nk), dtype=np.float32)
    elif out.dtype != np.float32 or out.size != int(ni) * int(nj) * int(nk) or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous float32 array of ni*nj*nk elements")
    out = out.reshape(-1)
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_hip_make_level_set3(t.ctypes.data_as(_P), t.shape[0] if t.ndim == 2 else t.size // 3,
                                        v.ctypes.data_as(_P), v.shape[0] if v.ndim == 2 else v.size // 3,
                                        o.ctypes.data_as(_P), ctypes.c_float(dx), int(ni), int(nj), int(nk),
                                        int(exact_band), int(ngpu), int(layout), out.ctypes.data_as(_P), err,
                                        ctypes.sizeof(err))
    if rc != OK:
        _raise(rc, err)
    if layout == LAYOUT_KFAST:
        return out.reshape((ni, nj, nk))
    return out.reshape((ni, nj, nk), order="F")


def cpu_make_level_set3(vertices: np.ndarray, triangles: np.ndarray, origin, dx: float, ni: int, nj: int, nk: int,
                        exact_band: int = 1, num_threads: int = 0, layout: int = LAYOUT_KFAST) -> np.ndarray:
    """The library's native CPU backend (include/sdfgen_cpu.h); same return convention."""
    v = np.ascontiguousarray(vertices, dtype=np.float32)
    t = np.ascontiguousarray(triangles, dtype=np.uint32)
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
    out = np.empty(int(ni) * int(nj) * int(nk), dtype=np.float32)
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_cpu_make_level_set3(t.ctypes.data_as(_P), t.size // 3, v.ctypes.data_as(_P), v.size // 3,
                                        o.ctypes.data_as(_P), ctypes.c_float(dx), int(ni), int(nj), int(nk),
                                        int(exact_band), int(num_threads), int(layout), out.ctypes.data_as(_P),
                                        err, ctypes.sizeof(err))
    if rc != OK:
        _raise(rc, err)
    if layout == LAYOUT_KFAST:
        return out.reshape((ni, nj, nk))
    return out.reshape((ni, nj, nk), order="F")


def make_level_set3_device(device: int, d_tri: int, ntri: int, d_xyz: int, nvert: int, origin, dx: float,
                           ni: int, nj: int, nk: int, exact_band: int, layout: int, d_out: int,
                           stream: int = 0) -> None:
    """Device-resident entry: raw device pointers (ints), optional hipStream_t."""
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_hip_make_level_set3_device(int(device), _P(d_tri), int(ntri), _P(d_xyz), int(nvert),
                                               o.ctypes.data_as(_P), ctypes.c_float(dx), int(ni), int(nj),
                                               int(nk), int(exact_band), int(layout), _P(d_out),
                                               _P(stream) if stream else None, err, ctypes.sizeof(err))
    if rc != OK:
        _raise(rc, err)


def last_profile() -> dict:
    p = Profile()
    lib.sdfgen_hip_last_profile(ctypes.byref(p))
    return p.as_dict()


def release() -> None:
    """Free the cached device workspaces (the slab communication pool and IPC mappings stay)."""
    lib.sdfgen_hip_release()


def slab_close_imports() -> int:
    """Opt-in: close the IPC mappings of neighbour slabs' blocks once no slab session is alive
    (sdfgen_hip_slab_close_imports; for long-lived processes whose peers are replaced between jobs)."""
    return int(lib.sdfgen_hip_slab_close_imports())


def debug_ptd(pts: np.ndarray, device: int = 0, variant: int = 0) -> np.ndarray:
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 12)
    out = np.empty(pts.shape[0], np.float32)
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_hip_debug_ptd(device, variant, pts.shape[0], pts.ctypes.data_as(_P), out.ctypes.data_as(_P),
                                  err, 512)
    if rc != OK:
        _raise(rc, err)
    return out


def debug_band(vertices, triangles, origin, dx: float, ni: int, nj: int, nk: int, exact_band: int = 1):
    """Stage 1 only on the current device (sdfgen_hip_debug_band) -> (phi, closest_tri, counts, big_n):
    the pre-sweep state as (ni,nj,nk) Fortran-ordered views of the i-fastest buffers (the layout of
    oracle.band), and the number of triangles the band phase treated as big."""
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(triangles, dtype=np.uint32).reshape(-1, 3)
    o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
    n = int(ni) * int(nj) * int(nk)
    phi, ct, cnt = np.empty(n, np.float32), np.empty(n, np.int32), np.empty(n, np.uint32)
    big = _u64(0)
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_hip_debug_band(t.ctypes.data_as(_P), t.shape[0], v.ctypes.data_as(_P), v.shape[0],
                                   o.ctypes.data_as(_P), ctypes.c_float(dx), int(ni), int(nj), int(nk),
                                   int(exact_band), phi.ctypes.data_as(_P), ct.ctypes.data_as(_P),
                                   cnt.ctypes.data_as(_P), ctypes.byref(big), err, ctypes.sizeof(err))
    if rc != OK:
        _raise(rc, err)
    f = lambda a: a.reshape((ni, nj, nk), order="F")
    return f(phi), f(ct), f(cnt), int(big.value)


def debug_sweep_trace(device: int = 0, max_entries: int = 1 << 22) -> np.ndarray:
    out = np.zeros(max_entries, np.uint64)
    n = _u64(0)
    rc = lib.sdfgen_hip_debug_sweep_trace(device, out.ctypes.data_as(_P), max_entries, ctypes.byref(n))
    if rc != OK:
        raise RuntimeError("no sweep trace recorded (set SDFGEN_TRACE_SWEEP)")
    return out[: n.value].reshape(-1, 8)


def debug_pit2d(pit: np.ndarray, device: int = 0) -> np.ndarray:
    pit = np.ascontiguousarray(pit, dtype=np.float64).reshape(-1, 8)
    out = np.empty((pit.shape[0], 4), np.float64)
    err = ctypes.create_string_buffer(512)
    rc = lib.sdfgen_hip_debug_pit2d(device, pit.shape[0], pit.ctypes.data_as(_P), out.ctypes.data_as(_P), err, 512)
    if rc != OK:
        _raise(rc, err)
    return out


class Slab:
    """One Z-slab session (sdfgen_hip_slab_*): planes k in [k_begin, k_end) on `device`."""

    def __init__(self, device: int, nslabs: int, slab: int, ni: int, nj: int, nk: int):
        self.dims = (int(ni), int(nj), int(nk))
        self.device, self.nslabs, self.slab = int(device), int(nslabs), int(slab)
        h = _P()
        err = ctypes.create_string_buffer(512)
        rc = lib.sdfgen_hip_slab_create(self.device, self.nslabs, self.slab, *self.dims, ctypes.byref(h), err,
                                        ctypes.sizeof(err))
        if rc != OK:
            _raise(rc, err)
        self.h = h
        kb, ke = ctypes.c_int(), ctypes.c_int()
        lib.sdfgen_hip_slab_range(self.h, ctypes.byref(kb), ctypes.byref(ke))
        self.k_begin, self.k_end = kb.value, ke.value

    def _check(self, rc, err):
        if rc != OK:
            _raise(rc, err)

    def export(self) -> bytes:
        buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_export(self.h, buf, err, ctypes.sizeof(err)), err)
        return buf.raw

    def connect_ipc(self, lower: bytes | None, upper: bytes | None) -> None:
        err = ctypes.create_string_buffer(512)
        lo = ctypes.create_string_buffer(lower, IPC_HANDLE_BYTES) if lower else None
        up = ctypes.create_string_buffer(upper, IPC_HANDLE_BYTES) if upper else None
        self._check(lib.sdfgen_hip_slab_connect_ipc(self.h, lo, up, err, ctypes.sizeof(err)), err)

    def connect_local(self, lower: "Slab | None", upper: "Slab | None") -> None:
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_connect_local(self.h, lower.h if lower else None, upper.h if upper else None,
                                                      err, ctypes.sizeof(err)), err)

    def prepare(self, ntri: int) -> None:
        """Allocate for a call with ntri triangles; with several slabs in one thread, prepare
        every slab before enqueuing any (sdfgen_hip_slab_prepare)."""
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_prepare(self.h, int(ntri), err, ctypes.sizeof(err)), err)

    def enqueue(self, d_tri: int, ntri: int, d_xyz: int, nvert: int, origin, dx: float, exact_band: int,
                layout: int, d_out: int) -> None:
        o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_enqueue(self.h, _P(d_tri), int(ntri), _P(d_xyz), int(nvert),
                                                o.ctypes.data_as(_P), ctypes.c_float(dx), int(exact_band),
                                                int(layout), _P(d_out), err, ctypes.sizeof(err)), err)

    def finish(self, nvert: int = 0) -> dict:
        p = Profile()
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_finish(self.h, int(nvert), ctypes.byref(p), err, ctypes.sizeof(err)), err)
        return p.as_dict()

    def run(self, vertices, triangles, origin, dx: float, exact_band: int = 1, layout: int = LAYOUT_ARRAY3):
        """Host arrays in; returns (phi slab (ni,nj,k_end-k_begin) indexed [i,j,k-k_begin], profile)."""
        v = np.ascontiguousarray(vertices, dtype=np.float32)
        t = np.ascontiguousarray(triangles, dtype=np.uint32)
        o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
        ni, nj, _ = self.dims
        nks = self.k_end - self.k_begin
        out = np.empty(ni * nj * nks, dtype=np.float32)
        p = Profile()
        err = ctypes.create_string_buffer(512)
        self._check(lib.sdfgen_hip_slab_run(self.h, t.ctypes.data_as(_P), t.size // 3, v.ctypes.data_as(_P),
                                            v.size // 3, o.ctypes.data_as(_P), ctypes.c_float(dx), int(exact_band),
                                            int(layout), out.ctypes.data_as(_P), ctypes.byref(p), err,
                                            ctypes.sizeof(err)), err)
        if layout == LAYOUT_KFAST:
            return out.reshape((ni, nj, nks)), p.as_dict()
        return out.reshape((ni, nj, nks), order="F"), p.as_dict()

    def debug_dump(self, which: int, max_bytes: int = 1 << 26) -> bytes:
        """Diagnostics (sdfgen_hip_slab_debug_dump): 0 comm block, 1 tile control words,
        2 first-pass completion flags, 3 task table, 4 dependency table."""
        buf = ctypes.create_string_buffer(max_bytes)
        n = _u64()
        rc = lib.sdfgen_hip_slab_debug_dump(self.h, int(which), buf, max_bytes, ctypes.byref(n))
        if rc != OK:
            raise HipError(rc, "debug dump failed")
        return buf.raw[:n.value]

    def close(self) -> None:
        if getattr(self, "h", None):
            lib.sdfgen_hip_slab_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CpuSlab:
    """CPU Z-slab session (sdfgen_cpu_slab_*); sweeps one at a time with explicit planes."""

    SWEEP_DIRS = ((1, 1, 1), (-1, -1, -1), (1, 1, -1), (-1, -1, 1), (1, -1, 1), (-1, 1, -1), (1, -1, -1), (-1, 1, 1))

    def __init__(self, nslabs: int, slab: int, ni: int, nj: int, nk: int):
        self.dims = (int(ni), int(nj), int(nk))
        self.nslabs, self.slab = int(nslabs), int(slab)
        h = _P()
        err = ctypes.create_string_buffer(512)
        rc = lib.sdfgen_cpu_slab_create(self.nslabs, self.slab, *self.dims, ctypes.byref(h), err, ctypes.sizeof(err))
        if rc != OK:
            _raise(rc, err)
        self.h = h
        kb, ke = ctypes.c_int(), ctypes.c_int()
        lib.sdfgen_cpu_slab_range(self.h, ctypes.byref(kb), ctypes.byref(ke))
        self.k_begin, self.k_end = kb.value, ke.value

    def band(self, vertices, triangles, origin, dx: float, exact_band: int = 1) -> None:
        self._v = np.ascontiguousarray(vertices, dtype=np.float32)   # kept alive for the sweeps
        self._t = np.ascontiguousarray(triangles, dtype=np.uint32)
        o = np.ascontiguousarray(np.asarray(origin, dtype=np.float32).reshape(3))
        err = ctypes.create_string_buffer(512)
        rc = lib.sdfgen_cpu_slab_band(self.h, self._t.ctypes.data_as(_P), self._t.size // 3,
                                      self._v.ctypes.data_as(_P), self._v.size // 3, o.ctypes.data_as(_P),
                                      ctypes.c_float(dx), int(exact_band), err, ctypes.sizeof(err))
        if rc != OK:
            _raise(rc, err)

    def upstream_is_below(self, sweep: int) -> bool:
        return self.SWEEP_DIRS[sweep % 8][2] > 0

    def sweep(self, sweep: int, plane_in: np.ndarray | None, want_out: bool) -> np.ndarray | None:
        ni, nj, _ = self.dims
        pin = None if plane_in is None else np.ascontiguousarray(plane_in, dtype=np.uint64)
        pout = np.empty(ni * nj, dtype=np.uint64) if want_out else None
        err = ctypes.create_string_buffer(512)
        rc = lib.sdfgen_cpu_slab_sweep(self.h, int(sweep), None if pin is None else pin.ctypes.data_as(_P),
                                       None if pout is None else pout.ctypes.data_as(_P), err, ctypes.sizeof(err))
        if rc != OK:
            _raise(rc, err)
        return pout

    def sign(self, layout: int = LAYOUT_ARRAY3) -> np.ndarray:
        ni, nj, _ = self.dims
        nks = self.k_end - self.k_begin
        out = np.empty(ni * nj * nks, dtype=np.float32)
        err = ctypes.create_string_buffer(512)
        rc = lib.sdfgen_cpu_slab_sign(self.h, int(layout), out.ctypes.data_as(_P), err, ctypes.sizeof(err))
        if rc != OK:
            _raise(rc, err)
        if layout == LAYOUT_KFAST:
            return out.reshape((ni, nj, nks))
        return out.reshape((ni, nj, nks), order="F")

    def close(self) -> None:
        if getattr(self, "h", None):
            lib.sdfgen_cpu_slab_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
