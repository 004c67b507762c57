"""sdfgenfast_amd -- MI355X-native signed distance fields, drop-in for ``sdfgen``.

Mirrors the reference Python surface (sdfgen/__init__.py:29-279 and the
nanobind module python/sdfgen_py.cpp:316-411):

    load_mesh, generate_sdf, save_sdf, load_sdf, is_gpu_available,
    generate_from_mesh, generate_from_file

``generate_sdf`` calls the hand-written gfx950 HIP kernels through the C-ABI of
include/sdfgen_hip.h (libsdfgen_hip.so), asking the device to write phi
directly in numpy's (nx, ny, nz) C order, so there is no host transpose
(python/sdfgen_py.cpp:71-98 in the reference).  ``backend="cpu"`` runs the
library's native multi-threaded CPU implementation (deterministic: identical
bits for any thread count).  ``backend="auto"`` picks the GPU when one is
visible, else the CPU backend, as the reference does
(common/sdfgen_unified.cpp:42-48).
"""
from __future__ import annotations

__version__ = "0.1.0"

import os
from typing import Optional, Tuple

import numpy as np

from . import _lib
from .meshio import load_mesh as _load_mesh
from .meshio import read_sdf as _read_sdf
from .meshio import write_sdf as _write_sdf

__all__ = [
    "load_mesh",
    "generate_sdf",
    "save_sdf",
    "load_sdf",
    "is_gpu_available",
    "generate_from_mesh",
    "generate_from_file",
    "last_profile",
]


def is_gpu_available() -> bool:
    """True when a HIP device is visible (python/sdfgen_py.cpp:311-313)."""
    return _lib.device_count() > 0


def load_mesh(filename: str):
    """-> (vertices (N,3) float32, triangles (M,3) uint32, ((minx,miny,minz),(maxx,maxy,maxz)))."""
    return _load_mesh(filename)


def _as_nx3(a, dtype, name):
    arr = np.asarray(a)
    if arr.ndim != 2 or arr.shape[1] != 3:
        raise TypeError(f"{name} must have shape (N, 3), got {arr.shape}")
    return np.ascontiguousarray(arr, dtype=dtype)


def _ngpu_from_env() -> int:
    """SDFGEN_NGPU, the drop-in's GPU-count knob (the reference's signature has no device argument):
    unset or "1" = the current device, "all" or "0" = every visible device, n > 1 = devices 0..n-1 with
    the grid split into Z-slabs -- the same rule as sdfgen::make_level_set3
    (csrc/sdfgen_unified.cpp ngpu_from_env)."""
    e = os.environ.get("SDFGEN_NGPU", "")
    if e == "":
        return _lib.NGPU_CURRENT
    if e == "all":
        return _lib.NGPU_ALL
    if not e.isdigit():
        raise ValueError(f"SDFGEN_NGPU = {e!r} (expected 'all', 0, 1 or a device count)")
    return int(e)


def generate_sdf(vertices, triangles, origin, dx, nx, ny, nz, exact_band=1, backend="auto", num_threads=0):
    """Generate a signed distance field (python/sdfgen_py.cpp:160-218).

    Returns a float32 array of shape (nx, ny, nz), C-ordered, sdf[i,j,k] = phi(i,j,k):
    negative inside, positive outside, bit-identical to the reference CPU
    implementation (cpu_lib/makelevelset3.cpp:192-304, single-thread semantics)."""
    v = _as_nx3(vertices, np.float32, "vertices")
    t = _as_nx3(triangles, np.uint32, "triangles")
    if v.shape[0] == 0 or t.shape[0] == 0:
        raise ValueError("Cannot generate SDF from empty mesh (vertices or triangles are empty)")
    nx, ny, nz = int(nx), int(ny), int(nz)
    if nx <= 0 or ny <= 0 or nz <= 0:
        raise ValueError("Grid dimensions must be positive (nx, ny, nz > 0)")
    dxf = np.float32(dx)
    if not dxf > 0.0:
        raise ValueError("Cell spacing dx must be positive")
    o = tuple(float(np.float32(origin[c])) for c in range(3))
    if backend not in ("auto", "cpu", "gpu"):
        raise ValueError(f"Invalid backend: {backend} (must be 'auto', 'cpu', or 'gpu')")
    if backend == "auto":
        backend = "gpu" if is_gpu_available() else "cpu"
    if backend == "gpu":
        if not is_gpu_available():
            raise RuntimeError("GPU backend requested but no HIP GPU device is available. "
                               "Use backend='cpu'.")
        return _lib.make_level_set3(v, t, o, float(dxf), nx, ny, nz, int(exact_band), _lib.LAYOUT_KFAST,
                                    ngpu=_ngpu_from_env())
    return _lib.cpu_make_level_set3(v, t, o, float(dxf), nx, ny, nz, int(exact_band), int(num_threads),
                                    _lib.LAYOUT_KFAST)


def save_sdf(filename: str, sdf_array, origin, dx) -> None:
    """Write a .sdf file (python/sdfgen_py.cpp:221-278; common/sdf_io.cpp:10-74)."""
    a = np.asarray(sdf_array)
    if a.ndim != 3:
        raise ValueError("SDF array must be 3-dimensional")
    _write_sdf(filename, a.astype(np.float32, copy=False), origin, float(np.float32(dx)))


def load_sdf(filename: str):
    """-> (sdf (nx,ny,nz) float32, origin, dx, bounds)   (python/sdfgen_py.cpp:281-308)."""
    sdf, mn, mx = _read_sdf(filename)
    dx = float(np.float32(np.float32(mx[0]) - np.float32(mn[0])) / np.float32(sdf.shape[0]))
    return sdf, tuple(mn), dx, (tuple(mn), tuple(mx))


def generate_from_mesh(vertices: np.ndarray, triangles: np.ndarray, nx: int, ny: Optional[int] = None,
                       nz: Optional[int] = None, dx: Optional[float] = None, padding: int = 1,
                       exact_band: int = 1, backend: str = "auto", num_threads: int = 0) -> Tuple[np.ndarray, dict]:
    """Grid sizing from mesh bounds, then generate (sdfgen/__init__.py:47-142)."""
    vertices = np.asarray(vertices)
    min_box = vertices.min(axis=0)
    max_box = vertices.max(axis=0)
    extents = max_box - min_box
    if ny is None or nz is None:
        if dx is None:
            dx = extents[0] / nx
        ny = int(np.ceil(extents[1] / dx)) if ny is None else ny
        nz = int(np.ceil(extents[2] / dx)) if nz is None else nz
    else:
        if dx is None:
            dx = max(extents[0] / nx, extents[1] / ny, extents[2] / nz)
    nx += 2 * padding
    ny += 2 * padding
    nz += 2 * padding
    origin = min_box - padding * dx
    sdf = generate_sdf(vertices, triangles, tuple(origin), dx, nx, ny, nz, exact_band=exact_band,
                       backend=backend, num_threads=num_threads)
    meta = {"origin": tuple(origin), "dx": dx, "bounds": (tuple(min_box), tuple(max_box)), "backend": backend}
    return sdf, meta


def generate_from_file(filename: str, nx: Optional[int] = None, ny: Optional[int] = None, nz: Optional[int] = None,
                       dx: Optional[float] = None, padding: int = 1, exact_band: int = 1, backend: str = "auto",
                       num_threads: int = 0) -> Tuple[np.ndarray, dict]:
    """Load a mesh file, size the grid, generate (sdfgen/__init__.py:145-265)."""
    vertices, triangles, bounds = load_mesh(filename)
    min_box = np.array(bounds[0], dtype=np.float32)
    max_box = np.array(bounds[1], dtype=np.float32)
    extents = max_box - min_box
    if dx is not None:
        if nx is None:
            nx = int(np.ceil(extents[0] / dx))
        if ny is None:
            ny = int(np.ceil(extents[1] / dx))
        if nz is None:
            nz = int(np.ceil(extents[2] / dx))
    elif nx is not None:
        if ny is None or nz is None:
            if dx is None:
                dx = extents[0] / nx
            ny = int(np.ceil(extents[1] / dx)) if ny is None else ny
            nz = int(np.ceil(extents[2] / dx)) if nz is None else nz
        else:
            if dx is None:
                dx = max(extents[0] / nx, extents[1] / ny, extents[2] / nz)
    else:
        raise ValueError("Must specify either 'dx' or 'nx' (or 'nx', 'ny', 'nz') for grid sizing")
    nx += 2 * padding
    ny += 2 * padding
    nz += 2 * padding
    origin = min_box - padding * dx
    sdf = generate_sdf(vertices, triangles, tuple(origin), dx, nx, ny, nz, exact_band=exact_band,
                       backend=backend, num_threads=num_threads)
    meta = {"origin": tuple(origin), "dx": dx, "bounds": (tuple(min_box), tuple(max_box)), "backend": backend}
    return sdf, meta


def last_profile() -> dict:
    """Per-phase device timings (HIP events) of the last GPU call in this process."""
    return _lib.last_profile()
