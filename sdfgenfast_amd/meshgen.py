"""Deterministic synthetic meshes and grid recipes for tests and the bench.

The bumpy UV-sphere is the 1M-triangle workload of BASELINE.json:
triangles = 2*nu*(nv-1), vertices = nu*(nv-1)+2.  Every coordinate is built
from IEEE-754 double +, -, *, / and round() only (no libm transcendental), so
the float32 vertices are bit-identical on any host -- the golden SHA-256 of the
reference output (tests/golden/hashes.json) therefore pins the HIP output at
full size on the GPU box.

Radius r = 1 + 0.15*s(5u)*s(4v) + 0.05*s(17u+3)*c(13v), z scaled by 1.3,
with s/c the polynomial sine/cosine below.
"""
from __future__ import annotations

import numpy as np

_TWO_PI = 6.283185307179586
_PI = 3.141592653589793


def _sin(x: np.ndarray) -> np.ndarray:
    """sin via reduction to [-pi, pi] and an odd Taylor polynomial (degree 21)."""
    x = np.asarray(x, dtype=np.float64)
    y = x - _TWO_PI * np.round(x / _TWO_PI)
    y2 = y * y
    # Horner on the Taylor coefficients 1/(2k+1)!  (k = 10 .. 0)
    acc = np.zeros_like(y)
    for k in range(10, -1, -1):
        f = 1.0
        for q in range(2, 2 * k + 2):
            f = f * q
        c = (1.0 / f) if k % 2 == 0 else (-1.0 / f)
        acc = acc * y2 + c
    return acc * y


def _cos(x: np.ndarray) -> np.ndarray:
    return _sin(np.asarray(x, dtype=np.float64) + _PI / 2.0)


def bumpy_sphere(nu: int = 1000, nv: int = 501):
    """Closed bumpy UV-sphere -> (vertices (V,3) f32, triangles (T,3) u32)."""
    if nu < 3 or nv < 2:
        raise ValueError("need nu >= 3 and nv >= 2")
    a = np.arange(nu, dtype=np.float64)
    b = np.arange(1, nv, dtype=np.float64)
    u = a * (_TWO_PI / nu)
    v = b * (_PI / nv)
    U, V = np.meshgrid(u, v)  # (nv-1, nu): ring-major
    r = 1.0 + 0.15 * _sin(5.0 * U) * _sin(4.0 * V) + 0.05 * _sin(17.0 * U + 3.0) * _cos(13.0 * V)
    sv, cv = _sin(V), _cos(V)
    x = r * sv * _cos(U)
    y = r * sv * _sin(U)
    z = 1.3 * r * cv
    ring = np.stack([x, y, z], axis=-1).reshape(-1, 3)
    rp = 1.0 + 0.05 * float(_sin(np.array([3.0]))[0])
    north = np.array([[0.0, 0.0, 1.3 * rp]])
    south = np.array([[0.0, 0.0, -1.3 * rp]])
    verts = np.concatenate([north, ring, south]).astype(np.float32)

    nr = nv - 1
    ia = np.arange(nu, dtype=np.int64)
    ia1 = (ia + 1) % nu
    tris = []
    r0 = 1
    tris.append(np.stack([np.zeros(nu, np.int64), r0 + ia, r0 + ia1], axis=1))  # north cap
    for bb in range(nr - 1):
        p = 1 + bb * nu
        q = 1 + (bb + 1) * nu
        t1 = np.stack([p + ia, q + ia, q + ia1], axis=1)
        t2 = np.stack([p + ia, q + ia1, p + ia1], axis=1)
        band = np.empty((2 * nu, 3), np.int64)
        band[0::2] = t1
        band[1::2] = t2
        tris.append(band)
    last = 1 + (nr - 1) * nu
    sp = 1 + nr * nu
    tris.append(np.stack([np.full(nu, sp, np.int64), last + ia1, last + ia], axis=1))  # south cap
    tri = np.concatenate(tris).astype(np.uint32)
    assert tri.shape[0] == 2 * nu * (nv - 1)
    return verts, tri


def unit_cube():
    """The 12-triangle cube of tests/test_correctness.cpp:30-62."""
    v = np.array([[-0.5, -0.5, -0.5], [0.5, -0.5, -0.5], [0.5, 0.5, -0.5], [-0.5, 0.5, -0.5],
                  [-0.5, -0.5, 0.5], [0.5, -0.5, 0.5], [0.5, 0.5, 0.5], [-0.5, 0.5, 0.5]], np.float32)
    t = np.array([[0, 1, 2], [0, 2, 3], [4, 6, 5], [4, 7, 6], [0, 5, 1], [0, 4, 5],
                  [2, 7, 3], [2, 6, 7], [0, 3, 7], [0, 7, 4], [1, 6, 2], [1, 5, 6]], np.uint32)
    return v, t


def bounds(v: np.ndarray):
    return np.fmin.reduce(v, axis=0).astype(np.float32), np.fmax.reduce(v, axis=0).astype(np.float32)


def grid_mode2b(vertices: np.ndarray, nx: int, ny: int, nz: int, padding: int):
    """CLI mode 2b sizing (app/main.cpp:180-185, 240-245), all float32:
    dx = max over axes of extent/(n-2*padding); grid centred on the mesh box.
    Returns (origin f32[3], dx f32)."""
    mn, mx = bounds(vertices)
    size = (mx - mn).astype(np.float32)
    f = np.float32
    dxs = [size[0] / f(nx - 2 * padding), size[1] / f(ny - 2 * padding), size[2] / f(nz - 2 * padding)]
    dx = dxs[0] if not (dxs[0] < max(dxs[1], dxs[2])) else max(dxs[1], dxs[2])
    dx = f(dx)
    gsize = np.array([f(nx) * dx, f(ny) * dx, f(nz) * dx], np.float32)
    center = ((mn + mx) * f(0.5)).astype(np.float32)
    origin = (center - gsize * f(0.5)).astype(np.float32)
    return origin, dx


def grid_proportional(vertices: np.ndarray, target_nx: int, padding: int):
    """tests/test_utils.cpp:276-305 calculate_grid_parameters -> (origin, dx, (nx,ny,nz))."""
    mn, mx = bounds(vertices)
    size = (mx - mn).astype(np.float32)
    f = np.float32
    dx = f(size[0] / f(target_nx - 2 * padding))
    ny = int(np.int32(size[1] / dx + f(0.5))) + 2 * padding
    nz = int(np.int32(size[2] / dx + f(0.5))) + 2 * padding
    gsize = np.array([f(target_nx) * dx, f(ny) * dx, f(nz) * dx], np.float32)
    center = ((mn + mx) * f(0.5)).astype(np.float32)
    origin = (center - gsize * f(0.5)).astype(np.float32)
    return origin, dx, (target_nx, ny, nz)


def tetrahedron():
    """A regular tetrahedron on alternate corners of the cube [-1, 1]^3: every face holds three
    corners, so every face's bounding box -- and band box -- spans the whole grid (the coarse-mesh
    extreme of the band phase: 4 triangles, 4 x the grid's cells of band work)."""
    v = np.array([[-1, -1, -1], [1, 1, -1], [1, -1, 1], [-1, 1, 1]], np.float32)
    t = np.array([[0, 2, 1], [0, 1, 3], [0, 3, 2], [1, 2, 3]], np.uint32)
    return v, t


# The reference's benchmark mesh tests/resources/test_x3y4z5_bin.stl as data: 36 triangles, 108 unshared
# vertices in file order (the binary STL's vertex coordinates are small integers), so the package needs no
# test tree (tests/test_api.py checks it against the loader on tests/golden/resources/test_x3y4z5_bin.stl).
_X3Y4Z5_XYZ = (
    -1, -1, -1, -1, -1, 1, -1, 1, 1, -1, -1, -1, -1, 1, 1, -1, 1, -1, -1, 1, 1, 1, 1, 1, 1, 3, 1,
    -1, 1, 1, 1, 3, 1, -1, 3, 1, 1, -1, 1, 1, -1, -1, 2, -1, -1, 1, -1, 1, 2, -1, -1, 2, -1, 1,
    1, -1, -1, 1, -1, 1, -1, -1, 1, 1, -1, -1, -1, -1, 1, -1, -1, -1, -1, 1, -1, 1, 1, -1, 1, -1, -1,
    -1, 1, -1, 1, -1, -1, -1, -1, -1, 1, 1, 1, -1, 1, 1, -1, 1, 4, 1, 1, 1, -1, 1, 4, 1, 1, 4,
    2, 1, -1, 2, 1, 1, 2, -1, 1, 2, 1, -1, 2, -1, 1, 2, -1, -1, 1, -1, -1, 1, 1, -1, 2, 1, -1,
    1, -1, -1, 2, 1, -1, 2, -1, -1, 1, 1, 1, 1, -1, 1, 2, -1, 1, 1, 1, 1, 2, -1, 1, 2, 1, 1,
    1, 1, -1, 1, 1, 1, 2, 1, 1, 1, 1, -1, 2, 1, 1, 2, 1, -1, -1, 3, -1, -1, 3, 1, 1, 3, 1,
    -1, 3, -1, 1, 3, 1, 1, 3, -1, -1, 1, -1, -1, 1, 1, -1, 3, 1, -1, 1, -1, -1, 3, 1, -1, 3, -1,
    1, 1, 1, 1, 1, -1, 1, 3, -1, 1, 1, 1, 1, 3, -1, 1, 3, 1, 1, 1, -1, -1, 1, -1, -1, 3, -1,
    1, 1, -1, -1, 3, -1, 1, 3, -1, 1, 1, 4, -1, 1, 4, -1, -1, 4, 1, 1, 4, -1, -1, 4, 1, -1, 4,
    1, -1, 1, 1, 1, 1, 1, 1, 4, 1, -1, 1, 1, 1, 4, 1, -1, 4, -1, 1, 1, -1, -1, 1, -1, -1, 4,
    -1, 1, 1, -1, -1, 4, -1, 1, 4, -1, -1, 1, 1, -1, 1, 1, -1, 4, -1, -1, 1, 1, -1, 4, -1, -1, 4,
)


def x3y4z5():
    """The reference's benchmark mesh tests/resources/test_x3y4z5_bin.stl (36 triangles), embedded: the
    vertices and faces the native loader returns for that file (bit-identical to the reference's
    meshio::load_stl, tests/test_meshio_ref.py)."""
    v = np.array(_X3Y4Z5_XYZ, np.float32).reshape(-1, 3)
    t = np.arange(v.shape[0], dtype=np.uint32).reshape(-1, 3)
    return v, t


# Named workloads: BASELINE.json's configs, the reference's own published benchmark
# (tests/benchmark_performance.cpp:151, 181-185: test_x3y4z5_bin.stl on proportional grids with padding
# 2, README.md:256-260) and a coarse-mesh extreme for the band phase.
WORKLOADS = {
    "c2_sphere70k_128": dict(nu=350, nv=101, n=128, padding=2),
    "c3_sphere1m_256": dict(nu=1000, nv=501, n=256, padding=2),
    "c4_sphere1m_512": dict(nu=1000, nv=501, n=512, padding=2),
    "c5_sphere4m_1024": dict(nu=2000, nv=1001, n=1024, padding=2),
    "x3y4z5_prop64": dict(mesh="x3y4z5", n=64, padding=2, grid="proportional"),     # 64 x 84 x 104
    "x3y4z5_prop128": dict(mesh="x3y4z5", n=128, padding=2, grid="proportional"),   # 128 x 169 x 211
    "x3y4z5_prop256": dict(mesh="x3y4z5", n=256, padding=2, grid="proportional"),   # 256 x 340 x 424
    "tetra_512": dict(mesh="tetrahedron", n=512, padding=2),
    # tile-configuration crossover (diagnostics): 1,600 and 2,304 tiles per sweep
    "sphere1m_320": dict(nu=1000, nv=501, n=320, padding=2),
    "sphere1m_384": dict(nu=1000, nv=501, n=384, padding=2),
}


def workload_mesh(name: str):
    w = WORKLOADS[name]
    m = w.get("mesh")
    if m == "x3y4z5":
        return x3y4z5()
    if m == "tetrahedron":
        return tetrahedron()
    return bumpy_sphere(w["nu"], w["nv"])


def workload(name: str):
    """-> (vertices, triangles, origin, dx, (ni, nj, nk)) for a named workload."""
    w = WORKLOADS[name]
    v, t = workload_mesh(name)
    n = w["n"]
    if w.get("grid") == "proportional":
        origin, dx, dims = grid_proportional(v, n, w["padding"])
        return v, t, origin, dx, dims
    origin, dx = grid_mode2b(v, n, n, n, w["padding"])
    return v, t, origin, dx, (n, n, n)
