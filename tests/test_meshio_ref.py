"""Native mesh loaders (csrc/meshio.cpp, include/sdfgen_meshio.h) pinned to the REFERENCE loaders
(common/mesh_io.cpp:29-48, mesh_io_obj.cpp:21-157, mesh_io_stl.cpp:42-332) -- bit-identical
vertices, triangles and min_box / max_box, and the same success / failure:

* against the reference's digests committed in tests/golden/meshio_ref.json (made by
  tests/golden/make_meshio_golden.py from the reference compiled here); runs anywhere;
* against the live reference build (oracle/_ref/libmeshref.so) on more seeds of the corpus and on
  files large enough to be parsed in several parallel chunks; skipped where it is not built.

The corpus (tests/meshio_corpus.py) covers the number grammar of `istream >> float` (signed
inf/nan, exponents without digits, hex, overflow, denormals), OBJ face tokens through std::stoi,
the ASCII-STL keyword state machine, binary-STL detection / truncation / 0 facets, and bounds
on monotone, NaN and signed-zero coordinates."""
import hashlib
import json
import os

import numpy as np
import pytest

import meshio_corpus
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen, meshio

HERE = os.path.dirname(__file__)
RES = os.path.join(HERE, "golden", "resources")
with open(os.path.join(HERE, "golden", "meshio_ref.json")) as _f:
    GOLD = json.load(_f)
CASES = dict(meshio_corpus.corpus(GOLD["seed"]))


def _native(path):
    """(rc, v, t, bounds f32[6]) from the native loader; rc 0 on failure."""
    try:
        v, t, b, _ = _lib.mesh_load(path)
    except RuntimeError:
        return 0, None, None, None
    return 1, v, t, np.float32(b)


def _digest(rc, v, t, b):
    if rc != 1:
        return {"rc": 0}
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    return {"rc": 1, "nvert": int(v.shape[0]), "ntri": int(t.shape[0]),
            "xyz_sha256": h(v.astype(np.float32)), "tri_sha256": h(t.astype(np.uint32)),
            "bounds_sha256": h(b)}


def test_corpus_matches_committed_case_list():
    assert sorted(CASES) == sorted(GOLD["cases"]), "tests/meshio_corpus.py changed: rerun make_meshio_golden.py"


@pytest.mark.parametrize("name", sorted(GOLD["cases"]))
def test_native_matches_reference_digest(tmp_path, name):
    p = tmp_path / name
    p.write_bytes(CASES[name])
    want = dict(GOLD["cases"][name])
    want.pop("bounds", None)
    if want["rc"] != 1:
        want = {"rc": 0}   # returned false or threw: the native loader must fail
    assert _digest(*_native(str(p))) == want


def _compare_live(path):
    rc, v, t, b, log = O.ref_load_mesh(path)
    nrc, v1, t1, b1 = _native(path)
    assert (rc == 1) == (nrc == 1), f"reference rc={rc}, native rc={nrc}: {log[-300:]}"
    if rc == 1:
        assert v.shape == v1.shape and t.shape == t1.shape
        assert np.array_equal(v.view(np.uint32), v1.view(np.uint32))
        assert np.array_equal(t, t1)
        assert np.array_equal(b.view(np.uint32), b1.view(np.uint32))
    return rc


needs_ref = pytest.mark.skipif(not O.meshref_available(),
                               reason="oracle/_ref/libmeshref.so not built (needs /root/reference)")


@needs_ref
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_native_matches_live_reference_corpus(tmp_path, seed):
    n_ok = 0
    for name, data in meshio_corpus.corpus(seed):
        p = tmp_path / name
        p.write_bytes(data)
        n_ok += _compare_live(str(p)) == 1
    assert n_ok > 50


@needs_ref
@pytest.mark.parametrize("name", sorted(os.listdir(RES)))
def test_reference_resources_live(name):
    assert _compare_live(os.path.join(RES, name)) == 1


@needs_ref
def test_large_files_live(tmp_path):
    """Files over the 4 MB-per-thread threshold: several parallel chunks split at line starts,
    replayed in file order (OBJ, ASCII STL) and the bulk binary path."""
    v, t = meshgen.bumpy_sphere(400, 301)   # 240,000 triangles
    rng = np.random.default_rng(9)
    obj = tmp_path / "big.obj"
    with open(obj, "w") as f:
        for i, x in enumerate(v):
            f.write(("v %.9g %.9g %.9g\n" if i % 3 else "v %.6e %.7f %r\n") % (x[0], x[1], float(x[2])))
        for i, q in enumerate(t + 1):
            f.write("f %d %d %d\n" % tuple(q) if i % 2 else "f %d/1 %d//2 %d/3/4\n" % tuple(q))
    assert os.path.getsize(obj) > 8 << 20
    assert _compare_live(str(obj)) == 1
    stl = tmp_path / "big_ascii.stl"
    with open(stl, "w") as f:
        f.write("solid big\n")
        for q in t[:60000]:
            f.write("facet normal 0 0 1\n outer loop\n")
            for c in q:
                f.write("  vertex %.9g %.9g %.9g\n" % tuple(v[c] * rng.uniform(0.5, 2)))
            f.write(" endloop\nendfacet\n")
        f.write("endsolid big\n")
    assert os.path.getsize(stl) > 8 << 20
    assert _compare_live(str(stl)) == 1
    tri = v[t].reshape(-1, 9).astype(np.float32)
    binp = tmp_path / "big_bin.stl"
    binp.write_bytes(meshio_corpus._stl_binary(tri))
    assert _compare_live(str(binp)) == 1


def test_load_mesh_api_bounds_are_reference_bounds(tmp_path):
    """meshio.load_mesh (the Python drop-in's sdfgen.load_mesh, python/sdfgen_py.cpp:101-157) returns
    the reference's min_box / max_box: a vertex that lowers the minimum can still raise the maximum
    (common/mesh_io.h:101-108)."""
    p = tmp_path / "decr.obj"
    p.write_bytes(CASES["bounds_decr.obj"])
    _, _, (mn, mx) = meshio.load_mesh(str(p))
    assert GOLD["cases"]["bounds_decr.obj"]["bounds"] == list(mn) + list(mx)
    assert mx[0] == 20.0


def test_zero_facet_binary_stl_loads_empty(tmp_path):
    """mesh_io_stl.cpp:140-172 returns true for 0 facets: an empty mesh, not an error."""
    p = tmp_path / "zero.stl"
    p.write_bytes(CASES["bin_zero.stl"])
    v, t, (mn, mx) = meshio.load_mesh(str(p))
    assert v.shape == (0, 3) and t.shape == (0, 3)
    assert mn == (float(np.finfo(np.float32).max),) * 3 and mx == (float(-np.finfo(np.float32).max),) * 3
