"""Diagnostics: run N slabs of one grid in this process on GPU 0 (first pass only matters) and,
on failure, dump each slab's tile-sweep control words, first-pass completion flags and the epoch
tags in its per-sweep inboxes.
    SDFGEN_TILE_GRID=96 python tools/slab_multi_diag.py NSLABS NI NJ NK
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from sdfgenfast_amd import _hiprt, _lib, meshgen  # noqa: E402


def main():
    nslabs, ni, nj, nk = (int(x) for x in sys.argv[1:5])
    v, t = meshgen.bumpy_sphere(90, 31)
    o, dx = meshgen.grid_mode2b(v, max(ni, 8), max(nj, 8), max(nk, 8), 2)
    slabs = [_lib.Slab(0, nslabs, s, ni, nj, nk) for s in range(nslabs)]
    for s, sl in enumerate(slabs):
        sl.connect_local(slabs[s - 1] if s > 0 else None, slabs[s + 1] if s < nslabs - 1 else None)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    outs = [_hiprt.DeviceBuffer(ni * nj * (sl.k_end - sl.k_begin) * 4) for sl in slabs]
    import time
    for sl in slabs:   # every slab set up before any slab's kernels run
        sl.prepare(t.shape[0])
    for s, (sl, d) in enumerate(zip(slabs, outs)):
        t0 = time.perf_counter()
        sl.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_ARRAY3, d.ptr)
        print(f"enqueue slab {s}: {time.perf_counter() - t0:.3f} s", flush=True)
    errs = []
    for sl in slabs:
        try:
            sl.finish(v.shape[0])
            errs.append(None)
        except Exception as e:
            errs.append(str(e))
    print("errors:", errs, flush=True)
    plane = ni * nj
    for s, sl in enumerate(slabs):
        ctrl = np.frombuffer(sl.debug_dump(1), np.int32)
        done = np.frombuffer(sl.debug_dump(2), np.uint32)
        tasks = np.frombuffer(sl.debug_dump(3), np.int32).reshape(-1, 4)
        comm = np.frombuffer(sl.debug_dump(0), np.uint64)
        print(f"slab {s} k=[{sl.k_begin},{sl.k_end}) ctrl={ctrl[:4].tolist()} tasks={len(tasks)} "
              f"done={np.bincount(done.astype(np.int64)).tolist()}", flush=True)
        for i, (tj, tk, q, _) in enumerate(tasks):
            if done[i] != done.max():
                print(f"   not done: rank {i} J={tj} K={tk} sweep={q}", flush=True)
        for q in range(8):
            ep = (comm[q * plane:(q + 1) * plane] >> np.uint64(32)).astype(np.int64)
            vals, cnts = np.unique(ep, return_counts=True)
            print(f"   inbox {q}: epochs {dict(zip(vals.tolist(), cnts.tolist()))}", flush=True)
    return 0 if all(e is None for e in errs) else 1


if __name__ == "__main__":
    sys.exit(main())
