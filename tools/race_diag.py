"""Find the first sweep whose GPU result differs from the oracle (debug aid).

    SDFGEN_LIB_OVERRIDE=path/libsdfgen_hip.so python tools/race_diag.py [ns ...]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen

v, t = meshgen.bumpy_sphere(120, 41)
dims = (48, 40, 56)
o, dx = meshgen.grid_mode2b(v, *dims, 2)
phi0, ct0, cnt = O.band(v, t, o, dx, *dims, 1)
par = np.cumsum(cnt, axis=0) % 2 == 1
nss = [int(x) for x in sys.argv[1:]] or [1, 2, 16]
bad = []
for ns in nss:
    os.environ["SDFGEN_DEBUG_NSWEEPS"] = str(ns)
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    p2, _ = O.sweep(v, t, o, dx, phi0, ct0, nsweeps=ns)
    want = np.where(par, -p2, p2)
    bad.append(int((np.asfortranarray(got).view(np.uint32) != np.asfortranarray(want).view(np.uint32)).sum()))
print(os.environ.get("SDFGEN_LIB_OVERRIDE", "default"), os.environ.get("SDFGEN_SWEEP", "tile"),
      "cells differing after", nss, "sweeps:", bad, flush=True)

if os.environ.get("DIAG_MAP"):
    os.environ["SDFGEN_DEBUG_NSWEEPS"] = "1"
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    p2, _ = O.sweep(v, t, o, dx, phi0, ct0, nsweeps=1)
    want = np.where(par, -p2, p2)
    d = np.asfortranarray(got).view(np.uint32) != np.asfortranarray(want).view(np.uint32)
    idx = np.argwhere(d)
    a, b, c = idx[:, 0] - 1, idx[:, 1] - 1, idx[:, 2] - 1
    print("bl hist", np.bincount(b % 8, minlength=8), "cl hist", np.bincount(c % 8, minlength=8))
    print("tiles (J,K) hist:", sorted(set(zip((b // 8).tolist(), (c // 8).tolist())))[:40])
    # first wrong cell in sweep order per tile: minimal a+bl+cl (step)
    for J, K in sorted(set(zip((b // 8).tolist(), (c // 8).tolist())))[:6]:
        m = (b // 8 == J) & (c // 8 == K)
        st = a[m] + b[m] % 8 + c[m] % 8
        i0 = np.argmin(st)
        print(f"tile {J},{K}: n={m.sum()} first step {st[i0]} at a={a[m][i0]} bl={b[m][i0] % 8} cl={c[m][i0] % 8}")
    # is the first error a direct loss of a neighbour's label?

if os.environ.get("DIAG_CELL"):
    # explain the first wrong cell of tile (J,K) in sweep 0 (all directions +1)
    os.environ["SDFGEN_DEBUG_NSWEEPS"] = "1"
    got = np.asfortranarray(_lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3))
    p2, c2 = O.sweep(v, t, o, dx, phi0, ct0, nsweeps=1)
    want = np.where(par, -p2, p2)
    d = got.view(np.uint32) != want.view(np.uint32)
    idx = np.argwhere(d)
    J, K = [int(x) for x in os.environ["DIAG_CELL"].split(",")]
    a, b, c = idx[:, 0] - 1, idx[:, 1] - 1, idx[:, 2] - 1
    m = (b // 8 == J) & (c // 8 == K)
    st = a[m] + b[m] % 8 + c[m] % 8
    order = np.argsort(st, kind="stable")[:4]
    tri = np.asarray(t, np.int64)
    V = np.asarray(v, np.float32)
    for n in order:
        i, j, k = idx[m][n]
        g = np.array([i * dx + o[0], j * dx + o[1], k * dx + o[2]], np.float32)
        pts = np.concatenate([np.broadcast_to(g, (len(tri), 3)), V[tri[:, 0]], V[tri[:, 1]], V[tri[:, 2]]], axis=1)
        dd = O.ptd_batch(pts)
        gv = abs(float(got[i, j, k]))
        cands = np.nonzero(dd == np.float32(gv))[0]
        nbrs = {}
        for di_, dj_, dk_ in [(-1, 0, 0), (0, -1, 0), (-1, -1, 0), (0, 0, -1), (-1, 0, -1), (0, -1, -1), (-1, -1, -1)]:
            nbrs[(di_, dj_, dk_)] = (int(c2[i + di_, j + dj_, k + dk_]), int(ct0[i + di_, j + dj_, k + dk_]))
        print(f"cell ijk=({i},{j},{k}) a={i-1} bl={(j-1)%8} cl={(k-1)%8}: gpu {got[i,j,k]!r} want {want[i,j,k]!r} "
              f"oracle ct {int(c2[i,j,k])} band ct {int(ct0[i,j,k])}; gpu value = ptd of tris {cands[:5].tolist()}")
        print("   oracle neighbour labels after sweep (label, band label):", nbrs)
