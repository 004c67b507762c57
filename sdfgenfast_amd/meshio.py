"""Host-side mesh and .sdf file I/O (the callers either side of the hot path).

* ``load_mesh``  -- the library's native loaders (include/sdfgen_meshio.h,
  csrc/meshio.cpp: whole-file read, text parsed in parallel line chunks, correctly
  rounded from_chars floats, update_minmax bounds in file order), restating
  common/mesh_io.cpp:29-48 (dispatch on extension), binary STL
  common/mesh_io_stl.cpp:98-173 (no vertex de-duplication), ASCII STL :179-303,
  format detection :42-92, OBJ common/mesh_io_obj.cpp:21-157 (fan :115-121), bounds
  common/mesh_io.h:101-108.  Pinned bit for bit to the reference loaders compiled
  from their sources (tests/test_meshio_ref.py).
* ``write_sdf`` / ``read_sdf`` -- common/sdf_io.cpp:10-147: a 36-byte header
  (3 x int32 dims, 3 x f32 min, 3 x f32 max = min + n*dx) followed by float32
  data written k-fastest (for i, for j, for k), i.e. exactly a C-ordered
  (ni, nj, nk) numpy array -- one bulk write instead of one 4-byte write per
  value.
"""
from __future__ import annotations

import os
import struct

import numpy as np


def load_mesh(filename: str):
    """Load an OBJ or STL mesh -> (vertices (N,3) f32, triangles (M,3) u32, bounds).

    Mirrors python/sdfgen_py.cpp:101-157 (``sdfgen.load_mesh``): bounds are the loader's
    min_box / max_box (update_minmax over the vertices in file order)."""
    from . import _lib
    path = os.fspath(filename)
    ext = os.path.splitext(path)[1].lower()
    if not os.path.isfile(path) or ext not in (".obj", ".stl"):
        raise RuntimeError(f"Failed to load mesh: {path}")
    try:
        v, t, b, _ = _lib.mesh_load(path)
    except RuntimeError as e:
        raise RuntimeError(f"Failed to load mesh: {path} ({e})") from e
    return v, t, (tuple(float(a) for a in b[:3]), tuple(float(a) for a in b[3:]))


def write_sdf(filename: str, sdf: np.ndarray, origin, dx: float) -> int:
    """Write ``sdf`` (C-ordered (ni,nj,nk) float32) as a .sdf file; returns the
    inside count (``val < 0``, common/sdf_io.cpp:53)."""
    a = np.ascontiguousarray(sdf, dtype=np.float32)
    if a.ndim != 3:
        raise ValueError("SDF array must be 3-dimensional")
    ni, nj, nk = a.shape
    if ni == 0 or nj == 0 or nk == 0:
        raise ValueError("SDF array dimensions cannot be zero")
    o = np.asarray(origin, dtype=np.float32).reshape(3)
    dxf = np.float32(dx)
    mx = np.array([o[0] + np.float32(ni) * dxf, o[1] + np.float32(nj) * dxf, o[2] + np.float32(nk) * dxf],
                  dtype=np.float32)
    try:
        with open(filename, "wb") as f:
            f.write(struct.pack("<3i", ni, nj, nk))
            f.write(o.astype("<f4").tobytes())
            f.write(mx.astype("<f4").tobytes())
            a.astype("<f4", copy=False).tofile(f)
    except OSError as e:
        raise RuntimeError(f"Failed to write SDF file: {filename}") from e
    return int(np.count_nonzero(a < 0.0))


def read_sdf(filename: str):
    """Read a .sdf file -> (sdf (ni,nj,nk) float32 C-order, min_box, max_box)."""
    try:
        with open(filename, "rb") as f:
            head = f.read(36)
            if len(head) < 36:
                raise RuntimeError(f"Failed to read SDF file: {filename}")
            ni, nj, nk = struct.unpack("<3i", head[:12])
            if ni <= 0 or nj <= 0 or nk <= 0:
                raise RuntimeError(f"Failed to read SDF file: {filename} (bad dims)")
            mn = struct.unpack("<3f", head[12:24])
            mx = struct.unpack("<3f", head[24:36])
            n = ni * nj * nk
            data = np.fromfile(f, dtype="<f4", count=n)
    except OSError as e:
        raise RuntimeError(f"Failed to read SDF file: {filename}") from e
    if data.size != n:
        raise RuntimeError(f"Failed to read SDF file: {filename} (truncated)")
    return data.astype(np.float32).reshape(ni, nj, nk), mn, mx
