"""Run N slabs of one grid in this process on GPU 0 and compare with the oracle.

Used by tests/test_gpu_slab.py in a subprocess with GPU_MAX_HW_QUEUES raised, so that
every slab's stream gets its own hardware queue (see the test for why).
    python tests/slab_inprocess_check.py NSLABS NI NJ NK
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import bits_equal, diff_report  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import _hiprt, _lib, meshgen  # noqa: E402


def main():
    nslabs, ni, nj, nk = (int(x) for x in sys.argv[1:5])
    v, t = meshgen.bumpy_sphere(90, 31)
    o, dx = meshgen.grid_mode2b(v, max(ni, 8), max(nj, 8), max(nk, 8), 2)
    want = np.asfortranarray(O.make_level_set3(v, t, o, dx, ni, nj, nk, 1))
    slabs = [_lib.Slab(0, nslabs, s, ni, nj, nk) for s in range(nslabs)]
    for s, sl in enumerate(slabs):
        sl.connect_local(slabs[s - 1] if s > 0 else None, slabs[s + 1] if s < nslabs - 1 else None)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    outs = [_hiprt.DeviceBuffer(ni * nj * (sl.k_end - sl.k_begin) * 4) for sl in slabs]
    for rep in range(2):   # twice: the second call reuses the inboxes (epochs keep counting)
        for sl_ in slabs:   # every slab set up before any slab's kernels run
            sl_.prepare(t.shape[0])
        for sl, d in zip(slabs, outs):
            sl.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_ARRAY3, d.ptr)
        errs = []
        for sl in slabs:
            try:
                sl.finish(v.shape[0])
            except Exception as e:   # report every slab's state, not just the first
                errs.append(str(e))
        if errs:
            print("ERROR", errs)
            return 1
        got = np.concatenate([d.download(np.float32, ni * nj * (sl.k_end - sl.k_begin))
                              for sl, d in zip(slabs, outs)]).reshape((ni, nj, nk), order="F")
        if not bits_equal(got, want):
            print("MISMATCH", diff_report(got, want, dx))
            return 1
    print(f"OK {nslabs} slabs {ni}x{nj}x{nk}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
