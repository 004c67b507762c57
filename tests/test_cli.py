"""CLI (sdfgenfast_amd/cli.py) against app/main.cpp's grammar, sizing and output file.

The x3y4z5 fixture mesh is written back out as a binary STL; running mode 2b
(`SDFGen test_x3y4z5_bin.stl 32 32 32 1 1`) must reproduce the reference tool's
.sdf bytes, SHA-256 426adb5c....  The CPU tests use
--backend cpu; the GPU test runs the same command on the HIP backend."""
import hashlib
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN_CASES, ROOT
from sdfgenfast_amd import cli, meshgen

REF_SHA = "426adb5ca3b0aa53834ec05384a6aedefb58f16a6581ae0b80b37c26b5147d9b"


def _write_stl(path, v, t):
    with open(path, "wb") as f:
        f.write(b"\0" * 80)
        f.write(struct.pack("<I", t.shape[0]))
        for tri in t:
            f.write(struct.pack("<3f", 0, 0, 0))
            for q in tri:
                f.write(struct.pack("<3f", *v[q]))
            f.write(b"\0\0")


@pytest.fixture
def x3y4z5_stl(tmp_path):
    c = next(g for g in GOLDEN_CASES if g.name == "x3y4z5_stl_32")
    p = tmp_path / "test_x3y4z5_bin.stl"
    _write_stl(p, c.vertices, c.triangles)
    return p, c


def _run(args, cwd):
    return subprocess.run([sys.executable, "-m", "sdfgenfast_amd", *args], cwd=cwd, capture_output=True, text=True,
                          env=dict(os.environ, PYTHONPATH=ROOT), timeout=300)


def test_plan_grammar():
    assert cli.plan(["m.obj", "0.1", "2"])["mode"] == "1"
    assert cli.plan(["m.obj", "0.1", "0", "4"])["padding"] == 1      # padding < 1 -> 1
    p = cli.plan(["m.stl", "64"])
    assert p["mode"] == "2a" and p["nx"] == 64 and p["padding"] == 1
    p = cli.plan(["m.stl", "64", "3", "8"])                            # argc 5, 3 < 20 -> 2a
    assert p["mode"] == "2a" and p["padding"] == 3 and p["threads"] == 8
    p = cli.plan(["m.stl", "64", "32", "48"])                          # argc 5, 32 >= 20 -> 2b
    assert p["mode"] == "2b" and (p["nx"], p["ny"], p["nz"]) == (64, 32, 48)
    p = cli.plan(["m.stl", "64", "32", "48", "2", "4"])
    assert p["padding"] == 2 and p["threads"] == 4
    for bad in ([], ["m.obj", "0.1"], ["m.stl"], ["m.ply", "1", "2"]):
        with pytest.raises(SystemExit):
            cli.plan(bad)
    with pytest.raises(SystemExit):
        cli.plan(["m.stl", "0"])


def test_grid_matches_mode2b_and_proportional():
    v, _ = meshgen.bumpy_sphere(40, 21)
    mn, mx = meshgen.bounds(v)
    o, dx, dims = cli.grid(cli.plan(["m.stl", "40", "36", "44", "2"]), mn, mx)
    o2, dx2 = meshgen.grid_mode2b(v, 40, 36, 44, 2)
    assert dims == (40, 36, 44) and dx == dx2 and np.array_equal(o, o2)
    o, dx, dims = cli.grid(cli.plan(["m.stl", "40", "2"]), mn, mx)
    o3, dx3, dims3 = meshgen.grid_proportional(v, 40, 2)
    assert dims == dims3 and dx == dx3 and np.array_equal(o, o3)


def test_grid_mode1_padding_and_truncation():
    mn, mx = np.array([0, 0, 0], np.float32), np.array([1, 0.5, 0.25], np.float32)
    o, dx, dims = cli.grid(cli.plan(["m.obj", "0.1", "2"]), mn, mx)
    assert np.allclose(o, [-0.2, -0.2, -0.2]) and dims == (14, 9, 6)


def test_cli_reproduces_reference_sdf_file_cpu(x3y4z5_stl, tmp_path):
    p, _ = x3y4z5_stl
    r = _run(["--backend", "cpu", "-q", p.name, "32", "32", "32", "1", "1"], tmp_path)
    assert r.returncode == 0, r.stderr
    out = tmp_path / "test_x3y4z5_bin_sdf_32x32x32.sdf"
    assert hashlib.sha256(out.read_bytes()).hexdigest() == REF_SHA


@pytest.mark.gpu
def test_cli_reproduces_reference_sdf_file_gpu(x3y4z5_stl, tmp_path):
    p, _ = x3y4z5_stl
    r = _run(["--backend", "gpu", p.name, "32", "32", "32", "1", "1"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "GPU (HIP" in r.stdout
    out = tmp_path / "test_x3y4z5_bin_sdf_32x32x32.sdf"
    assert hashlib.sha256(out.read_bytes()).hexdigest() == REF_SHA


def test_cli_mode2a_proportional_dims_and_header(x3y4z5_stl, tmp_path):
    """tests/test_cli_modes.cpp:94-100: `Nx=32` on the x3y4z5 mesh -> a 32x42x52 grid,
    named <base>_sdf_32x42x52.sdf, header dims match; values = the prop32 fixture."""
    p, _ = x3y4z5_stl
    r = _run(["--backend", "cpu", "-q", p.name, "32"], tmp_path)
    assert r.returncode == 0, r.stderr
    out = tmp_path / "test_x3y4z5_bin_sdf_32x42x52.sdf"
    raw = out.read_bytes()
    assert struct.unpack("<3i", raw[:12]) == (32, 42, 52)
    c = next(g for g in GOLDEN_CASES if g.name == "x3y4z5_stl_prop32")
    got = np.frombuffer(raw[36:], dtype="<f4").reshape(32, 42, 52)
    assert np.array_equal(got.view(np.uint32), np.ascontiguousarray(c.phi, np.float32).view(np.uint32))
    mn = struct.unpack("<3f", raw[12:24])
    assert np.allclose(mn, c.origin)


def test_cli_mode1_obj(tmp_path):
    """Mode 1 (legacy OBJ + dx + padding): <base>.sdf, sizes = padded box / dx (truncated)."""
    v, t = meshgen.bumpy_sphere(30, 11)
    obj = tmp_path / "sphere.obj"
    with open(obj, "w") as f:
        for x in v:
            f.write(f"v {x[0]:.9g} {x[1]:.9g} {x[2]:.9g}\n")
        for tri in t:
            f.write(f"f {tri[0] + 1} {tri[1] + 1} {tri[2] + 1}\n")
    r = _run(["--backend", "cpu", "-q", obj.name, "0.1", "2"], tmp_path)
    assert r.returncode == 0, r.stderr
    raw = (tmp_path / "sphere.sdf").read_bytes()
    dims = struct.unpack("<3i", raw[:12])
    from sdfgenfast_amd import meshio
    _, _, (mn, mx) = meshio.load_mesh(str(obj))
    o, dx, want = cli.grid(cli.plan([obj.name, "0.1", "2"]), mn, mx)
    assert dims == want and len(raw) == 36 + 4 * int(np.prod(dims))
    phi = np.frombuffer(raw[36:], dtype="<f4").reshape(dims)
    assert phi[dims[0] // 2, dims[1] // 2, dims[2] // 2] < 0 and phi[0, 0, 0] > 0


def test_cli_errors(tmp_path):
    """test_cli_errors: usage text for too few arguments, failure for a missing mesh."""
    r = _run([], tmp_path)
    assert r.returncode != 0 and "mode 1" in (r.stdout + r.stderr).lower()
    r = _run(["--backend", "cpu", "missing.stl", "32"], tmp_path)
    assert r.returncode != 0 and "Failed to load mesh" in r.stderr
    r = _run(["--backend", "cpu", "m.stl", "0"], tmp_path)
    assert r.returncode != 0
