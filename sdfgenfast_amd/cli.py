"""Command-line front end: the reference's SDFGen tool (app/main.cpp) on this backend.

    python -m sdfgenfast_amd <file.obj> <dx> <padding> [threads]          mode 1
    python -m sdfgenfast_amd <file.stl> <Nx> [padding] [threads]           mode 2a
    python -m sdfgenfast_amd <file.stl> <Nx> <Ny> <Nz> [padding] [threads] mode 2b

Same argument grammar (including the argc == 5 heuristic of app/main.cpp:107,
"second value < 20 means mode 2a"), the same float32 grid sizing
(mode 1 :214-245 -- box padded by padding*dx, sizes = (max-min)/dx truncated;
mode 2a :109-131; mode 2b :150-176, dx = max over axes), the same output names
(`<base>.sdf`, or `<base>_sdf_NIxNJxNK.sdf` in mode 2, :309-316) and the same
.sdf file (36-byte header + k-fastest float32, common/sdf_io.cpp:10-60).

Additions for this backend (options go before the positional arguments):
  --backend {auto,gpu,cpu}   hardware selection (reference: always Auto, :255)
  --gpus N                   split the grid into N Z-slabs over GPUs 0..N-1 (GPU backend)
  -o/--output PATH           output file instead of the derived name
  -q/--quiet                 summary line only
The VTK writer of the reference (HAVE_VTK builds) is out of scope.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import _lib, generate_sdf, is_gpu_available, meshio

_f = np.float32


def _atoi(s: str) -> int:
    """C atoi: leading integer prefix, 0 when there is none (app/main.cpp uses atoi)."""
    s = s.strip()
    n = 0
    sign = 1
    i = 0
    if i < len(s) and s[i] in "+-":
        sign = -1 if s[i] == "-" else 1
        i += 1
    digits = ""
    while i < len(s) and s[i].isdigit():
        digits += s[i]
        i += 1
    if digits:
        n = int(digits)
    return sign * n


def plan(argv: list[str]):
    """Parse the positional arguments exactly as app/main.cpp:28-186 does.

    Returns dict(mode, filename, padding, threads, and either dx (mode 1) or
    target dims) -- or raises SystemExit with the usage text."""
    argc = len(argv) + 1
    filename = argv[0] if argv else ""
    is_stl = filename.endswith(".stl")
    mode_precise = is_stl and argc >= 3
    if (not mode_precise and argc < 4) or (mode_precise and argc < 3):
        raise SystemExit(__doc__)
    p = {"filename": filename, "padding": 1, "threads": 0}
    if mode_precise:
        is_2a = argc in (3, 4) or (argc == 5 and _atoi(argv[2]) < 20)
        if is_2a:
            p["mode"] = "2a"
            p["nx"] = _atoi(argv[1])
            if argc >= 4:
                p["padding"] = _atoi(argv[2])
            if argc == 5:
                p["threads"] = _atoi(argv[3])
            if p["nx"] <= 0:
                raise SystemExit("Error: Grid dimension must be a positive integer.")
        else:
            p["mode"] = "2b"
            p["nx"], p["ny"], p["nz"] = _atoi(argv[1]), _atoi(argv[2]), _atoi(argv[3])
            if argc >= 6:
                p["padding"] = _atoi(argv[4])
            if argc == 7:
                p["threads"] = _atoi(argv[5])
            if min(p["nx"], p["ny"], p["nz"]) <= 0:
                raise SystemExit("Error: Grid dimensions must be positive integers.")
    else:
        p["mode"] = "1"
        if not filename.endswith(".obj") or len(filename) < 5:
            raise SystemExit("Error: Mode 1 requires OBJ file (.obj extension).")
        try:
            p["dx"] = _f(float(argv[1]))    # stringstream >> float
        except ValueError:
            p["dx"] = _f(0.0)
        p["padding"] = _atoi(argv[2])
        if argc >= 5:
            p["threads"] = _atoi(argv[3])
    if p["padding"] < 1:
        p["padding"] = 1
    return p


def grid(p: dict, mn: np.ndarray, mx: np.ndarray):
    """(origin f32[3], dx f32, (ni,nj,nk)) for a parsed plan and the mesh's bounds."""
    mn = np.asarray(mn, _f)
    mx = np.asarray(mx, _f)
    pad = p["padding"]
    if p["mode"] == "1":
        dx = _f(p["dx"])
        off = _f(_f(pad) * dx)                      # padding*dx*unit (:236-238)
        lo = (mn - off).astype(_f)
        hi = (mx + off).astype(_f)
        ext = ((hi - lo).astype(_f) / dx).astype(_f)
        dims = tuple(int(np.uint32(x)) for x in ext)   # Vec3ui(...): truncation (:239)
        return lo, dx, dims
    size = (mx - mn).astype(_f)
    if p["mode"] == "2a":
        nx = p["nx"]
        dx = _f(size[0] / _f(nx - 2 * pad))
        ny = int(np.int32(_f(size[1] / dx) + _f(0.5))) + 2 * pad
        nz = int(np.int32(_f(size[2] / dx) + _f(0.5))) + 2 * pad
        dims = (nx, ny, nz)
    else:
        dims = (p["nx"], p["ny"], p["nz"])
        dxs = [_f(size[a] / _f(dims[a] - 2 * pad)) for a in range(3)]
        m = dxs[2] if dxs[1] < dxs[2] else dxs[1]     # std::max(dx_y, dx_z)
        dx = m if dxs[0] < m else dxs[0]              # std::max(dx_x, .)
    gsize = np.array([_f(dims[0]) * dx, _f(dims[1]) * dx, _f(dims[2]) * dx], _f)
    center = ((mn + mx).astype(_f) * _f(0.5)).astype(_f)
    origin = (center - (gsize * _f(0.5)).astype(_f)).astype(_f)
    return origin, _f(dx), dims


def output_name(p: dict, dims) -> str:
    base = p["filename"][: p["filename"].rfind(".")] if "." in p["filename"] else p["filename"]
    if p["mode"] == "1":
        return base + ".sdf"
    return f"{base}_sdf_{dims[0]}x{dims[1]}x{dims[2]}.sdf"


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m sdfgenfast_amd", add_help=True,
                                 description="SDFGen on MI355X (see module docstring for the modes)")
    ap.add_argument("--backend", choices=["auto", "gpu", "cpu"], default="auto")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("-o", "--output", default=None)
    ap.add_argument("-q", "--quiet", action="store_true")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    ns = ap.parse_args(argv)
    p = plan(ns.args)
    say = (lambda *a: None) if ns.quiet else print
    try:
        v, t, (mn, mx) = meshio.load_mesh(p["filename"])
    except RuntimeError as e:
        print(f"Failed to load mesh: {e}", file=sys.stderr)
        return 255
    origin, dx, dims = grid(p, mn, mx)
    gpu = is_gpu_available()
    impl = "GPU (HIP, MI355X)" if (ns.backend == "gpu" or (ns.backend == "auto" and gpu)) else "CPU (multi-threaded)"
    say(f"Mode {p['mode']}: {p['filename']} ({t.shape[0]} triangles)")
    say(f"  Grid dimensions: {dims[0]} x {dims[1]} x {dims[2]}  dx = {float(dx):.9g}  padding = {p['padding']}")
    say(f"  Padded bounds: ({origin[0]:.6g}, {origin[1]:.6g}, {origin[2]:.6g})")
    say(f"  Implementation: {impl}")
    t0 = time.perf_counter()
    if ns.gpus > 1 and ns.backend != "cpu":
        impl = f"GPU (HIP, MI355X) x{ns.gpus} Z-slabs"
        sdf = _lib.make_level_set3(v, t, origin, float(dx), *dims, 1, _lib.LAYOUT_KFAST, ngpu=ns.gpus)
    else:
        sdf = generate_sdf(v, t, origin, float(dx), *dims, exact_band=1, backend=ns.backend,
                           num_threads=p["threads"])
    el = time.perf_counter() - t0
    out = ns.output or output_name(p, dims)
    inside = meshio.write_sdf(out, sdf, origin, float(dx))
    total = dims[0] * dims[1] * dims[2]
    print(f"{out}: {dims[0]}x{dims[1]}x{dims[2]}, inside {inside} / {total} "
          f"({100.0 * inside / total:.2f}%), {el * 1e3:.1f} ms, {total / el / 1e6:.1f} Mvoxels/s ({impl})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
