"""Generate tests/golden/meshio_ref.json: the REFERENCE mesh loaders' results on the corpus of
tests/meshio_corpus.py, as digests.

Runs only in the development container, where oracle/_ref/libmeshref.so is compiled from the
reference's own common/mesh_io.cpp, mesh_io_obj.cpp and mesh_io_stl.cpp (`make -C oracle ref`).
For each case it records what meshio::load_mesh (common/mesh_io.cpp:29-48) returned: rc (1 loaded,
0 returned false, 2 threw), vertex and triangle counts and SHA-256 of the vertex (f32), triangle
(u32) and bounds (min_box, max_box as 6 f32) bytes.  tests/test_meshio_ref.py checks the native
loaders against these digests anywhere, and against the live reference where it is built.

    python tests/golden/make_meshio_golden.py
"""
import hashlib
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
import meshio_corpus  # noqa: E402

SEED = 20261017


def digest(rc, v, t, b):
    if rc != 1:
        return {"rc": rc}
    h = lambda a: hashlib.sha256(a.tobytes()).hexdigest()
    return {"rc": 1, "nvert": int(v.shape[0]), "ntri": int(t.shape[0]),
            "xyz_sha256": h(v), "tri_sha256": h(t), "bounds_sha256": h(b),
            "bounds": [float(x) for x in b]}


def main():
    out = {"seed": SEED, "generator": "tests/meshio_corpus.py corpus(seed)",
           "reference": "common/mesh_io.cpp, mesh_io_obj.cpp, mesh_io_stl.cpp via oracle/_ref/libmeshref.so",
           "cases": {}}
    with tempfile.TemporaryDirectory() as d:
        for name, data in meshio_corpus.corpus(SEED):
            p = os.path.join(d, name)
            with open(p, "wb") as f:
                f.write(data)
            rc, v, t, b, _ = O.ref_load_mesh(p)
            out["cases"][name] = digest(rc, v, t, b)
    path = os.path.join(HERE, "meshio_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    n_ok = sum(c["rc"] == 1 for c in out["cases"].values())
    print(f"wrote {path}: {len(out['cases'])} cases, {n_ok} load")


if __name__ == "__main__":
    main()
