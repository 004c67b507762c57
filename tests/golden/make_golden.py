"""Generate the golden fixtures in tests/golden/ from the REFERENCE implementation.

Run in the development container only (needs /root/reference):

    make -C oracle all ref
    python tests/golden/make_golden.py --small          # cases.npz (full phi arrays)
    python tests/golden/make_golden.py --edge           # edge_cases.npz (far / NaN / Inf vertices, wrapping bands)
    python tests/golden/make_golden.py --large c2 c3 c4 # hashes.json (SHA-256 of phi)
    python tests/golden/make_golden.py --large x3y4z5_prop64 tetra_512   # any meshgen.WORKLOADS name

Every expected output comes from ``sdfgen::cpu::make_level_set3(..., num_threads=1)``
(/root/reference/cpu_lib/makelevelset3.cpp:192, compiled by oracle/Makefile into
oracle/_ref/libsdfref.so).  Inputs are the reference's own test meshes
(tests/resources, tests/test_correctness.cpp:30-62) plus deterministic synthetic
meshes from sdfgenfast_amd/meshgen.py.  Only data (inputs + outputs) is stored.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import meshgen  # noqa: E402

RES = "/root/reference/tests/resources"


def _ref_load(path):
    """The reference's own loader (common/mesh_io.cpp via oracle/_ref/libmeshref.so). The native
    loader gives the same bits on these files (tests/test_meshio_ref.py::test_reference_resources_live),
    so fixtures made before round 3 with meshio.load_mesh are unchanged."""
    rc, v, t, _, _ = O.ref_load_mesh(path)
    assert rc == 1, path
    return v, t, None


def small_cases():
    """(name, vertices, triangles, origin, dx, (ni,nj,nk), exact_band)."""
    cases = []
    v, t, _ = _ref_load(os.path.join(RES, "test_x3y4z5_bin.stl"))
    o, dx = meshgen.grid_mode2b(v, 32, 32, 32, 1)
    cases.append(("x3y4z5_stl_32", v, t, o, dx, (32, 32, 32), 1))           # SURVEY 8.c fixture (1)
    o, dx, dims = meshgen.grid_proportional(v, 32, 1)
    cases.append(("x3y4z5_stl_prop32", v, t, o, dx, dims, 1))               # 32x42x52
    vq, tq, _ = _ref_load(os.path.join(RES, "test_x3y4z5_quads.obj"))
    o, dx = meshgen.grid_mode2b(vq, 24, 20, 28, 2)
    cases.append(("x3y4z5_quads_obj", vq, tq, o, dx, (24, 20, 28), 1))
    vc, tc = meshgen.unit_cube()
    o, dx, dims = meshgen.grid_proportional(vc, 64, 2)
    cases.append(("cube_64", vc, tc, o, dx, dims, 1))                        # fixture (2)
    vs, ts = meshgen.bumpy_sphere(60, 31)                                    # 3,600 tris
    o, dx = meshgen.grid_mode2b(vs, 40, 44, 52, 2)
    cases.append(("sphere3600_40x44x52", vs, ts, o, dx, (40, 44, 52), 1))   # fixture (3)
    cases.append(("sphere3600_band0", vs, ts, o, dx, (40, 44, 52), 0))
    cases.append(("sphere3600_band3", vs, ts, o, dx, (40, 44, 52), 3))
    # mesh partly outside the grid: triangles clamped onto boundary cells
    o2 = (o + np.float32(9) * dx).astype(np.float32)
    cases.append(("sphere3600_shifted", vs, ts, o2, dx, (40, 44, 52), 1))
    # tiny and degenerate grids (python/tests/test_sdfgen.py:925-936)
    for dims in [(1, 1, 1), (2, 3, 1), (1, 5, 4), (3, 3, 3), (5, 2, 7)]:
        oo, dd = meshgen.grid_mode2b(vc, max(dims[0], 3), max(dims[1], 3), max(dims[2], 3), 1)
        cases.append((f"cube_tiny_{dims[0]}x{dims[1]}x{dims[2]}", vc, tc, oo, dd, dims, 1))
    # single triangle + degenerate (zero-area, repeated-vertex) triangles
    v1 = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0.5, 0.5, 0.5], [0.5, 0.5, 0.5], [0.2, 0.9, 0.1]],
                  np.float32)
    t1 = np.array([[0, 1, 2], [3, 4, 5], [3, 3, 3], [0, 1, 1]], np.uint32)
    o, dx = meshgen.grid_mode2b(v1, 17, 19, 13, 2)
    cases.append(("degenerate_tris", v1, t1, o, dx, (17, 19, 13), 1))
    # mesh far from the origin (python/tests/test_sdfgen.py:960-990)
    vf = (vc + np.float32(1000.0)).astype(np.float32)
    o, dx = meshgen.grid_mode2b(vf, 20, 20, 20, 2)
    cases.append(("cube_far", vf, tc, o, dx, (20, 20, 20), 1))
    # random triangle soup (open, self-intersecting): distances exact, signs = parity rule
    rng = np.random.default_rng(20251205)
    vr = rng.uniform(-1, 1, size=(300, 3)).astype(np.float32)
    tr = rng.integers(0, 300, size=(200, 3)).astype(np.uint32)
    o, dx = meshgen.grid_mode2b(vr, 30, 26, 22, 1)
    cases.append(("random_soup", vr, tr, o, dx, (30, 26, 22), 2))
    return cases


def run_small(out_path):
    data = {}
    names = []
    for name, v, t, o, dx, dims, band in small_cases():
        t0 = time.time()
        phi = O.ref_make_level_set3(v, t, o, dx, *dims, exact_band=band, num_threads=1)
        mine = O.make_level_set3(v, t, o, dx, *dims, exact_band=band)
        same = np.array_equal(phi.view(np.uint32), mine.view(np.uint32))
        print(f"{name:28s} dims={dims} tris={t.shape[0]:6d} band={band} ref {time.time()-t0:.2f}s "
              f"oracle==ref: {same}")
        if not same:
            raise SystemExit(f"oracle restatement differs from reference on {name}")
        names.append(name)
        data[f"{name}/vertices"] = v
        data[f"{name}/triangles"] = t
        data[f"{name}/origin"] = np.asarray(o, np.float32)
        data[f"{name}/dx"] = np.float32(dx)
        data[f"{name}/dims"] = np.asarray(dims, np.int32)
        data[f"{name}/exact_band"] = np.int32(band)
        data[f"{name}/phi"] = np.ascontiguousarray(phi)  # sdf[i,j,k] (C order)
    data["names"] = np.array(names)
    np.savez_compressed(out_path, **data)
    print("wrote", out_path, os.path.getsize(out_path), "bytes")


INT_MAX = 2**31 - 1


def edge_cases():
    """Inputs whose band boxes and ray lattices go through C++ int(double) out of range, NaN and
    +-Inf, and the +band+1 wrap (cpu_lib/makelevelset3.cpp:206-212, 222-233; SURVEY App. A "Edge
    semantics").  x86 cvttsd2si gives INT_MIN there; the boxes follow from clamp() after the wrap."""
    cases = []
    vc, tc = meshgen.unit_cube()
    dims = (20, 22, 24)
    o, dx = meshgen.grid_mode2b(vc, *dims, 2)
    f32 = np.float32

    def with_tris(extra_v, extra_t):
        v = np.concatenate([vc, np.asarray(extra_v, np.float32)]).astype(np.float32)
        t = np.concatenate([tc, np.asarray(extra_t, np.uint32) + len(vc)]).astype(np.uint32)
        return v, t

    base = np.array([[0.1, 0.05, 0.1], [0.3, 0.2, 0.15], [0.05, 0.3, 0.25]], np.float32)
    # one vertex more than 2^31 cells from the grid, on each axis and sign (fi = +-3e9 and just past
    # the int range)
    for axis in range(3):
        for sgn, mag in ((1, 3.0e9), (-1, 3.0e9), (1, 2.2e9), (-1, 2.16e9)):
            far = base[2].copy()
            far[axis] = f32(o[axis] + f32(sgn * mag) * f32(dx))
            v, t = with_tris([base[0], base[1], far], [[0, 1, 2]])
            cases.append((f"far_{'xyz'[axis]}{'+' if sgn > 0 else '-'}{int(mag / 1e7)}", v, t, o, dx, dims, 1))
    # all three vertices far (the whole triangle off the grid, boxes from INT_MIN on every axis)
    v, t = with_tris([[3e9 * dx, 1e10 * dx, -5e9 * dx], [-4e9 * dx, 2e9 * dx, 3.1e9 * dx], [1.0, 2.5e9 * dx, 0.2]],
                     [[0, 1, 2]])
    cases.append(("far_all", v, t, o, dx, dims, 1))
    # NaN and +-Inf coordinates
    for axis in range(3):
        for name, val in (("nan", np.nan), ("pinf", np.inf), ("ninf", -np.inf)):
            bad = base[2].copy()
            bad[axis] = f32(val)
            v, t = with_tris([base[0], base[1], bad], [[0, 1, 2]])
            cases.append((f"{name}_{'xyz'[axis]}", v, t, o, dx, dims, 1))
    v, t = with_tris([[np.nan, np.nan, np.nan], [np.inf, -np.inf, np.inf], [0.2, 0.2, 0.2]], [[0, 1, 2], [1, 2, 0]])
    cases.append(("nan_inf_mixed", v, t, o, dx, dims, 1))
    # exact_band large enough that int(max) + band + 1 wraps, very wide, zero and negative
    for band in (INT_MAX, INT_MAX - 1, 2**30, 1000, 0, -1, -5, -(2**31) + 1):
        cases.append((f"cube_band_{band}", vc, tc, o, dx, dims, band))
    # far / non-finite vertices together with a band wide enough that every box is big
    v, t = with_tris([base[0], base[1], [f32(o[0] - f32(3e9) * f32(dx)), 0.1, 0.1], [np.nan, 0.0, 0.0],
                      [0.1, f32(o[1] + f32(2.5e9) * f32(dx)), 0.2]], [[0, 1, 2], [0, 1, 3], [4, 1, 0]])
    cases.append(("far_nan_band40", v, t, o, dx, (48, 40, 44), 40))
    vs, ts = meshgen.bumpy_sphere(40, 17)
    os_, dxs = meshgen.grid_mode2b(vs, 36, 30, 40, 2)
    v = np.concatenate([vs, [[np.nan, 0, 0], [0, np.inf, 0], [0, 0, f32(os_[2] + f32(2.3e9) * dxs)]]]).astype(np.float32)
    t = np.concatenate([ts, [[len(vs), len(vs) + 1, len(vs) + 2], [0, 1, len(vs) + 2]]]).astype(np.uint32)
    cases.append(("sphere_with_bad_tris", v, t, os_, dxs, (36, 30, 40), 2))
    return cases


def run_edge(out_path):
    data = {}
    names = []
    with np.errstate(all="ignore"):
        for name, v, t, o, dx, dims, band in edge_cases():
            phi = O.ref_make_level_set3(v, t, o, dx, *dims, exact_band=band, num_threads=1)
            mine = O.make_level_set3(v, t, o, dx, *dims, exact_band=band)
            same = np.array_equal(phi.view(np.uint32), mine.view(np.uint32))
            print(f"{name:24s} dims={dims} tris={t.shape[0]:5d} band={band} oracle==ref: {same}")
            if not same:
                raise SystemExit(f"oracle restatement differs from reference on {name}")
            names.append(name)
            data[f"{name}/vertices"] = v
            data[f"{name}/triangles"] = t
            data[f"{name}/origin"] = np.asarray(o, np.float32)
            data[f"{name}/dx"] = np.float32(dx)
            data[f"{name}/dims"] = np.asarray(dims, np.int32)
            data[f"{name}/exact_band"] = np.int32(band)
            data[f"{name}/phi"] = np.ascontiguousarray(phi)
    data["names"] = np.array(names)
    np.savez_compressed(out_path, **data)
    print("wrote", out_path, os.path.getsize(out_path), "bytes")


def digest(phi_f: np.ndarray) -> dict:
    """phi_f: (ni,nj,nk) array; hashes are over the i-fastest (Array3f) byte order."""
    flat = np.asfortranarray(phi_f).ravel(order="F").astype("<f4")
    sb = np.signbit(flat)
    return {
        "sha256_phi": hashlib.sha256(flat.tobytes()).hexdigest(),
        "sha256_signbit": hashlib.sha256(np.packbits(sb).tobytes()).hexdigest(),
        "inside_lt0": int(np.count_nonzero(flat < 0)),
        "signbit_count": int(np.count_nonzero(sb)),
        "sum_abs_f64": float(np.abs(flat.astype(np.float64)).sum()),
    }


LARGE = {"c2": "c2_sphere70k_128", "c3": "c3_sphere1m_256", "c4": "c4_sphere1m_512",
         "c5": "c5_sphere4m_1024"}


def run_large(keys, out_path):
    db = {}
    if os.path.exists(out_path):
        with open(out_path) as f:
            db = json.load(f)
    for key in keys:
        name = LARGE.get(key, key)   # a short key or any meshgen.WORKLOADS name
        v, t, o, dx, dims = meshgen.workload(name)
        t0 = time.time()
        phi = O.ref_make_level_set3(v, t, o, dx, *dims, exact_band=1, num_threads=1)
        el = time.time() - t0
        rec = digest(phi)
        rec.update({"dims": [int(d) for d in dims], "triangles": int(t.shape[0]), "vertices": int(v.shape[0]),
                    "origin": [float(a) for a in o], "dx": float(dx),
                    "mesh_sha256": hashlib.sha256(v.tobytes() + t.tobytes()).hexdigest(),
                    "ref_seconds_1thread": round(el, 2)})
        db[name] = rec
        print(name, json.dumps(rec))
        with open(out_path, "w") as f:
            json.dump(db, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--large", nargs="*", default=[])
    ap.add_argument("--edge", action="store_true")
    a = ap.parse_args()
    if a.small:
        run_small(os.path.join(HERE, "cases.npz"))
    if a.edge:
        run_edge(os.path.join(HERE, "edge_cases.npz"))
    if a.large:
        run_large(a.large, os.path.join(HERE, "hashes.json"))
