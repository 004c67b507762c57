"""Load rate of the native OBJ / ASCII-STL / binary-STL loaders on the C3 mesh (1,000,000-triangle
bumpy sphere written as files), against the REFERENCE loaders compiled from their sources
(oracle/_ref/libmeshref.so: common/mesh_io*.cpp; development container only) on the same files.
python tools/meshio_rate.py [outdir]"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import meshgen, meshio  # noqa: E402


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp()
    v, t, _, _, _ = meshgen.workload("c3_sphere1m_256")
    obj = os.path.join(d, "sphere1m.obj")
    with open(obj, "w") as f:
        f.write("".join("v %.9g %.9g %.9g\n" % tuple(p) for p in v))
        f.write("".join("f %d %d %d\n" % (a + 1, b + 1, c + 1) for a, b, c in t))
    stl = os.path.join(d, "sphere1m_ascii.stl")
    with open(stl, "w") as f:
        f.write("solid s\n")
        for a, b, c in t:
            f.write("facet normal 0 0 0\nouter loop\n")
            for q in (a, b, c):
                f.write("vertex %.9g %.9g %.9g\n" % tuple(v[q]))
            f.write("endloop\nendfacet\n")
        f.write("endsolid s\n")
    for path in (obj, stl):
        t0 = time.perf_counter()
        vn, tn, bn = meshio.load_mesh(path)
        tnat = time.perf_counter() - t0
        t0 = time.perf_counter()
        rc, vr, tr, br, _ = O.ref_load_mesh(path)
        tref = time.perf_counter() - t0
        same = (rc == 1 and np.array_equal(vn.view(np.uint32), vr.view(np.uint32)) and np.array_equal(tn, tr)
                and np.array_equal(np.float32(bn[0] + bn[1]).view(np.uint32), br.view(np.uint32)))
        print(f"{os.path.basename(path)}: {os.path.getsize(path) / 1e6:.0f} MB, {tn.shape[0]} triangles: native "
              f"{tnat:.3f} s, reference {tref:.2f} s, identical={same}", flush=True)


if __name__ == "__main__":
    main()
