"""Deterministic corpus of mesh files for the loader parity tests (tests/test_meshio_ref.py) and
the reference-digest generator (tests/golden/make_meshio_golden.py).

Every case is (name, file bytes). Names end in the extension the loader dispatches on
(common/mesh_io.cpp:29-48). The corpus aims at the reference grammar's corners:
  * numbers as `istream >> float` reads them (common/mesh_io_obj.cpp:75, mesh_io_stl.cpp:272):
    signs, exponents with and without digits, inf/nan spellings, hex, overflow, denormals;
  * OBJ faces through std::stoi (mesh_io_obj.cpp:97-106): index forms, signs, bad tokens,
    polygons (fan :115-121), short faces;
  * ASCII STL keyword state machine (mesh_io_stl.cpp:216-284) and binary STL detection and
    sizes (:42-92, :98-173), including 0 facets and truncation;
  * bounds (update_minmax, common/mesh_io.h:101-108) with monotone, NaN and signed-zero inputs.
"""
from __future__ import annotations

import struct

import numpy as np

# Tokens `>> float` must treat exactly as libstdc++ num_get does.
ODD_FLOATS = [
    "1", "-1", "+1", "0", "-0", "+0", "-0.0", ".5", "5.", "-.5e-3", "+.25E+2", "00012", "1e0005",
    "1e", "1e+", "2.5E-", "1.5ex", "3e+x", "-", "+", ".", "-.", "+-1", "-+1", "1.5.5", "1,5",
    "inf", "-inf", "+inf", "INF", "-Infinity", "nan", "-nan", "+nan", "NaN", "nan(1)",
    "0x1p3", "-0x10", "0X1", "1e-50", "-1e-50", "4e-45", "1.4e-45", "1e-38", "1e38", "3.4028235e38",
    "3.4028236e38", "1e39", "-1e50", "123456789012345678901234567890", "0.000000000000000000000001",
    "9.99999999999999999999e-1", "1.00000005960464477539062", "16777217", "-16777217", "2e-7x",
    "7abc", "1e2e3", "0e0", "-0e-0",
]


def _fmt_values(rng, n):
    x = rng.standard_normal(n).astype(np.float64) * 10.0 ** rng.integers(-6, 6, n)
    out = []
    for i, a in enumerate(x):
        k = i % 8
        out.append(["%.9g" % a, "%.6f" % a, "%e" % a, "%.17g" % a, "%d" % int(a), "+%.7g" % abs(a),
                    "%.3e" % (a * 1e-30), "%.12g" % (a * 1e25)][k])
    return out


def _obj_values_cases():
    cases = []
    # one vertex line per odd token in each coordinate slot, plus a face so the file loads
    for slot in range(3):
        lines = ["v 0 0 0", "v 1 0 0", "v 0 1 0"]
        for tok in ODD_FLOATS:
            xyz = ["0.5", "0.25", "0.125"]
            xyz[slot] = tok
            lines.append("v " + " ".join(xyz))
        lines.append("v 0 0 1")
        lines.append("f 1 2 3")
        lines.append(f"f 1 2 {len(lines) - 1}")   # the last vertex's index depends on how many lines parsed
        lines.append("f -1 -2 -3")
        cases.append((f"odd_floats_slot{slot}.obj", ("\n".join(lines) + "\n").encode()))
    return cases


def _obj_face_cases():
    base = ["v 0 0 0", "v 1 0 0", "v 0 1 0", "v 0 0 1", "v 1 1 1"]
    faces_ok = [
        "f 1 2 3", "f 1/1 2/2 3/3", "f 1/1/1 2/2/2 3/3/3", "f 1//1 2//2 3//3", "f 1 2 3 4 5",
        "f  1   2\t3  ", "f\t1 2 3", "f +1 +2 +3", "f -1 -2 -3", "f 0 1 2", "f 1.7 2.2 3e1",
        "f 1a 2b 3c", "f 2147483647 1 2", "f -2147483648 1 2", "f 1 2", "f 1", "f", "f ",
        "f 1 2 3 # comment", "fo 1 2 3", "F 1 2 3", " f 1 2 3", "f 1 2 3 4 5 6 7 8 9",
    ]
    cases = []
    for n, fl in enumerate(faces_ok):
        body = base + ["f 1 2 3", fl]
        cases.append((f"face_{n:02d}.obj", ("\n".join(body) + "\n").encode()))
    for n, fl in enumerate(["f a b c", "f 1 2 x", "f /1 2 3", "f 2147483648 1 2", "f -2147483649 1 2",
                            "f 99999999999 1 2", "f 1 2 3 - 4", "f 1 2 +"]):
        body = base + ["f 1 2 3", fl]
        cases.append((f"face_bad_{n:02d}.obj", ("\n".join(body) + "\n").encode()))
    return cases


def _obj_misc_cases(rng):
    cases = []
    lines = ["# generated", "o thing", "", "g group", "usemtl m", "s off", "vx 1 2 3", "v", "v 1 2",
             "v 1 2 3 4", "v\t1\t2\t3", "v  1  2  3", "vn 0 0 1", "vt 0.5 0.5", "vp 1 2 3"]
    nv = 1500
    vals = _fmt_values(rng, 3 * nv)
    for i in range(nv):
        lines.append("v " + " ".join(vals[3 * i:3 * i + 3]))
    for f in range(1200):
        k = 3 + f % 4
        idx = rng.integers(1, nv + 1, k)
        form = f % 3
        toks = [str(i) if form == 0 else (f"{i}/{i}" if form == 1 else f"{i}//{i}") for i in idx]
        lines.append("f " + " ".join(toks))
    cases.append(("mixed_lf.obj", ("\n".join(lines) + "\n").encode()))
    cases.append(("mixed_crlf.obj", ("\r\n".join(lines) + "\r\n").encode()))
    cases.append(("mixed_noeol.obj", "\n".join(lines).encode()))
    # bounds: monotone increasing / decreasing coordinates, NaN and signed zeros
    for name, seq in [("incr", np.arange(20, dtype=np.float32)),
                      ("decr", np.arange(20, 0, -1, dtype=np.float32)),
                      ("single", np.float32([3.0])),
                      ("zeros", np.float32([0.0, -0.0, 0.0, -0.0])),
                      ("negzeros", np.float32([-0.0, 0.0, -0.0]))]:
        ls = [f"v {repr(float(a))} {repr(float(-a))} {repr(float(a))}" for a in seq]
        ls += ["v 0 0 0", "v 0 0 0", "f 1 2 3"]
        cases.append((f"bounds_{name}.obj", ("\n".join(ls) + "\n").encode()))
    cases.append(("empty.obj", b""))
    cases.append(("no_faces.obj", b"v 0 0 0\nv 1 0 0\nv 0 1 0\n"))
    cases.append(("no_verts.obj", b"f 1 2 3\n"))
    cases.append(("only_bad_verts.obj", b"v inf 0 0\nv -nan 0 0\nv 1e 2 3\nf 1 2 3\n"))
    cases.append(("UPPER.OBJ", b"v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n"))
    return cases


def _stl_ascii(facets, name="gen", kw=("solid", "facet normal 0 0 1", "outer loop", "vertex", "endloop",
                                          "endfacet", "endsolid"), eol="\n"):
    s, fn, ol, vx, el, ef, es = kw
    out = [f"{s} {name}"]
    for tri in facets:
        out.append(f"  {fn}")
        out.append(f"    {ol}")
        for v in tri:
            out.append(f"      {vx} " + " ".join(v))
        out.append(f"    {el}")
        out.append(f"  {ef}")
    out.append(f"{es} {name}")
    return (eol.join(out) + eol).encode()


def _stl_ascii_cases(rng):
    cases = []
    ntri = 400
    vals = _fmt_values(rng, 9 * ntri)
    facets = [[vals[9 * f + 3 * c:9 * f + 3 * c + 3] for c in range(3)] for f in range(ntri)]
    cases.append(("gen_ascii.stl", _stl_ascii(facets)))
    cases.append(("gen_ascii_crlf.stl", _stl_ascii(facets, eol="\r\n")))
    cases.append(("gen_ascii_upper.stl", _stl_ascii(
        facets[:20], kw=("SOLID", "FACET NORMAL 0 0 1", "OUTER LOOP", "VERTEX", "ENDLOOP", "ENDFACET", "ENDSOLID"))))
    cases.append(("gen_ascii_tabs.stl", _stl_ascii(facets[:20]).replace(b"  ", b"\t")))
    # one odd token per file in the first vertex's x slot
    good = [["0", "0", "0"], ["1", "0", "0"], ["0", "1", "0"]]
    for n, tok in enumerate(ODD_FLOATS):
        f0 = [[tok, "0", "0"], ["1", "0", "0"], ["0", "1", "0"]]
        cases.append((f"odd_{n:02d}.stl", _stl_ascii([good, f0, good])))
    bad = {
        "two_vertices": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nendloop\nendfacet\nendsolid\n",
        "four_vertices": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nvertex 0 1 0\nvertex 1 1 0\nendloop\nendfacet\nendsolid\n",
        "vertex_outside": "solid s\nvertex 0 0 0\nendsolid\n",
        "vertex_outside_loop": "solid s\nfacet normal 0 0 1\nvertex 0 0 0\nendfacet\nendsolid\n",
        "facet_outside_solid": "solid s\nendsolid\nfacet normal 0 0 1\n",
        "bad_number": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 zero 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid\n",
        "short_vertex": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid\n",
        "no_facets": "solid s\nendsolid s\n",
        "no_endfacet": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendsolid\n",
    }
    for k, body in bad.items():
        cases.append((f"err_{k}.stl", body.encode()))
    quirks = {
        # a facet without endfacet leaves its vertices in the list (mesh_io_stl.cpp:279), then a normal one
        "dangling_vertices": "solid s\nfacet normal 0 0 1\nouter loop\nvertex 9 9 9\nvertex 8 8 8\nendloop\n"
                             "facet normal 0 0 1\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid\n",
        "keyword_prefixes": "solidity\nfacets\nouter loops\nvertexes 0 0 0\nvertex1 1 0 0\nvertex 0 1 0 extra\nendloops\nendfacets\n",
        "outer_tab_loop": "solid s\nfacet normal 0 0 1\nouter\tloop\nvertex 0 0 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid\n",
        "two_solids": "solid a\nfacet\nouter loop\nvertex 0 0 0\nvertex 1 0 0\nvertex 0 1 0\nendloop\nendfacet\nendsolid a\n"
                      "solid b\nfacet\nouter loop\nvertex 0 0 1\nvertex 1 0 1\nvertex 0 1 1\nendloop\nendfacet\nendsolid b\n",
        "blank_lines": "\n\n   \nsolid s\n\t\nfacet normal 0 0 1\n outer loop\n  vertex 0 0 0\n  vertex 1 0 0\n  vertex 0 1 0\n endloop\nendfacet\nendsolid\n\n",
    }
    for k, body in quirks.items():
        cases.append((f"quirk_{k}.stl", body.encode()))
    return cases


def _stl_binary(tris, header=b"binary header", count=None, attr=0, extra=b""):
    n = len(tris)
    rec = np.zeros(n, dtype=[("n", "<f4", 3), ("v", "<f4", 9), ("a", "<u2")])
    if n:
        rec["v"] = np.asarray(tris, np.float32).reshape(n, 9)
        rec["a"] = attr
    return header.ljust(80, b" ")[:80] + struct.pack("<I", n if count is None else count) + rec.tobytes() + extra


def _stl_binary_cases(rng):
    cases = []
    t = rng.standard_normal((300, 9)).astype(np.float32)
    cases.append(("bin_gen.stl", _stl_binary(t)))
    cases.append(("bin_zero.stl", _stl_binary([])))
    cases.append(("bin_solid_header.stl", _stl_binary(t[:10], header=b"solid but binary")))
    cases.append(("bin_truncated.stl", _stl_binary(t[:10], count=11)))
    cases.append(("bin_trailing.stl", _stl_binary(t[:10], extra=b"xx")))
    cases.append(("bin_solid_size_mismatch.stl", _stl_binary(t[:10], header=b"solid x", extra=b"\n")))
    special = np.float32([[np.nan, 0, 0, 1, np.inf, 0, -0.0, 1, -np.inf],
                          [0.0, -0.0, 0.0, -0.0, 0.0, -0.0, 1e-45, -1e-45, 0.0],
                          [5, 4, 3, 2, 1, 0, -1, -2, -3]])
    cases.append(("bin_special.stl", _stl_binary(special)))
    cases.append(("bin_decreasing.stl", _stl_binary(np.arange(90, 0, -1, dtype=np.float32).reshape(10, 9))))
    cases.append(("tiny.stl", b"sol"))
    cases.append(("header_only.stl", b"solid".ljust(80, b" ")))
    cases.append(("count_only.stl", _stl_binary([], header=b"bin")[:82]))
    return cases


def corpus(seed: int = 20261017):
    """All cases for one seed: [(name, bytes)], names unique."""
    rng = np.random.default_rng(seed)
    cases = (_obj_values_cases() + _obj_face_cases() + _obj_misc_cases(rng) + _stl_ascii_cases(rng)
             + _stl_binary_cases(rng))
    names = [c[0] for c in cases]
    assert len(names) == len(set(n.lower() for n in names)), "duplicate case names"
    return cases
