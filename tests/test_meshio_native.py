"""Native mesh loaders (csrc/meshio.cpp, include/sdfgen_meshio.h) against the Python
restatement of the reference's loaders (meshio.load_mesh_py: common/mesh_io_obj.cpp:21-157,
common/mesh_io_stl.cpp:42-303, per-token strtof): bit-identical vertices, triangles and
update_minmax bounds -- on the reference's own test meshes (tests/golden/resources, copied
from the reference's tests/resources as data) and on generated meshes with awkward number
formats, polygons, index forms and line endings."""
import os

import numpy as np
import pytest

from sdfgenfast_amd import meshio

RES = os.path.join(os.path.dirname(__file__), "golden", "resources")


def _same(path):
    v1, t1, b1 = meshio.load_mesh(path)
    v2, t2, b2 = meshio.load_mesh_py(path)
    assert v1.shape == v2.shape and t1.shape == t2.shape
    assert np.array_equal(v1.view(np.uint32), v2.astype(np.float32).view(np.uint32))
    assert np.array_equal(t1, t2)
    assert np.array_equal(np.float32(b1).view(np.uint32), np.float32(b2).view(np.uint32))
    return v1, t1


@pytest.mark.parametrize("name", sorted(os.listdir(RES)))
def test_reference_resources_native_equals_python(name):
    v, t = _same(os.path.join(RES, name))
    assert t.shape[0] == 36   # the same x3y4z5 box in every format
    if name.endswith(".stl"):
        assert v.shape[0] == 108   # STL repeats vertices per facet (mesh_io_stl.cpp:157-165)


def _fmt_values(rng, n):
    """Floats in the formats meshes carry: %.9g, %.6f, %e, %.17g, integers, '+' signs, tiny
    and huge exponents, negative zero."""
    x = rng.standard_normal(n).astype(np.float64) * 10.0 ** rng.integers(-6, 6, n)
    out = []
    for i, a in enumerate(x):
        k = i % 8
        if k == 0:
            out.append("%.9g" % a)
        elif k == 1:
            out.append("%.6f" % a)
        elif k == 2:
            out.append("%e" % a)
        elif k == 3:
            out.append("%.17g" % a)
        elif k == 4:
            out.append("%d" % int(a))
        elif k == 5:
            out.append("+%.7g" % abs(a))
        elif k == 6:
            out.append("%.3e" % (a * 1e-30))
        else:
            out.append("-0.0" if i % 16 == 7 else "%.12g" % (a * 1e25))
    return out


def test_generated_obj_native_equals_python(tmp_path):
    rng = np.random.default_rng(5)
    nv = 3000
    vals = _fmt_values(rng, 3 * nv)
    lines = ["# generated", "o thing", ""]
    for i in range(nv):
        lines.append("v " + " ".join(vals[3 * i:3 * i + 3]))
        if i % 97 == 0:
            lines.append("vn 0 0 1")
            lines.append("vt 0.5 0.5")
    for f in range(2000):
        k = 3 + f % 4                       # triangles, quads, pentagons, hexagons (fan)
        idx = rng.integers(1, nv + 1, k)
        form = f % 3
        toks = [str(i) if form == 0 else (f"{i}/{i}" if form == 1 else f"{i}//{i}") for i in idx]
        lines.append("f " + " ".join(toks))
    p = tmp_path / "gen.obj"
    p.write_bytes(("\r\n".join(lines) + "\r\n").encode())   # CRLF line ends
    v, t = _same(str(p))
    assert v.shape[0] == nv and t.shape[0] == sum(1 + f % 4 for f in range(2000))


def test_generated_ascii_stl_native_equals_python(tmp_path):
    rng = np.random.default_rng(6)
    ntri = 800
    vals = _fmt_values(rng, 9 * ntri)
    out = ["solid gen"]
    for f in range(ntri):
        out.append("  facet normal 0 0 1")
        out.append("    outer loop")
        for c in range(3):
            out.append("      vertex " + " ".join(vals[9 * f + 3 * c:9 * f + 3 * c + 3]))
        out.append("    endloop")
        out.append("  endfacet")
    out.append("endsolid gen")
    p = tmp_path / "gen.stl"
    p.write_text("\n".join(out) + "\n")
    v, t = _same(str(p))
    assert t.shape[0] == ntri and v.shape[0] == 3 * ntri


def test_generated_binary_stl_native_equals_python(tmp_path):
    rng = np.random.default_rng(7)
    ntri = 5000
    rec = np.zeros(ntri, dtype=[("n", "<f4", 3), ("v", "<f4", 9), ("a", "<u2")])
    rec["v"] = rng.standard_normal((ntri, 9)).astype(np.float32)
    p = tmp_path / "gen.stl"
    with open(p, "wb") as f:
        f.write(b"binary header".ljust(80, b" "))
        f.write(np.uint32(ntri).tobytes())
        f.write(rec.tobytes())
    v, t = _same(str(p))
    assert t.shape[0] == ntri


@pytest.mark.parametrize("body", [
    "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nendloop\nendfacet\nendsolid\n",  # 2 vertices
    "solid s\nvertex 0 0 0\nendsolid\n",                                                            # outside facet
    "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 zero 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid\n",
    "solid s\nendsolid\nfacet normal 0 0 1\n",                                                      # facet outside solid
])
def test_ascii_stl_errors_native_and_python_agree(tmp_path, body):
    """Malformed ASCII STL fails in both loaders (mesh_io_stl.cpp:179-303 returns false)."""
    p = tmp_path / "bad.stl"
    p.write_text(body)
    with pytest.raises(RuntimeError):
        meshio.load_mesh(str(p))
    with pytest.raises(RuntimeError):
        meshio.load_mesh_py(str(p))
