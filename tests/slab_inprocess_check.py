"""Run N slabs of one grid in this process on GPU 0 and compare with the oracle, or, for a named
full-size workload, with the reference's digests (tests/golden/hashes.json).

Used by tests/test_gpu_slab.py and tests/test_gpu_bounds.py in a subprocess with
GPU_MAX_HW_QUEUES raised, so that every slab's stream gets its own hardware queue (see
test_gpu_slab.py for why); SDFGEN_LIB_OVERRIDE selects the bounds-checked library.
    python tests/slab_inprocess_check.py NSLABS NI NJ NK
    python tests/slab_inprocess_check.py NSLABS WORKLOAD [REPS]
    python tests/slab_inprocess_check.py NSLABS WORKLOAD REPS --cabi
The --cabi form runs the split through sdfgen_hip_make_level_set3(ngpu = NSLABS) -- the C-ABI's own
multi-device path -- with every slab on device 0 (SDFGEN_DEBUG_SLABS_ONE_DEVICE) and host arrays.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import GOLDEN, bits_equal, diff_report  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import _hiprt, _lib, meshgen  # noqa: E402


def main():
    nslabs = int(sys.argv[1])
    if sys.argv[2].isdigit():
        ni, nj, nk = (int(x) for x in sys.argv[2:5])
        v, t = meshgen.bumpy_sphere(90, 31)
        o, dx = meshgen.grid_mode2b(v, max(ni, 8), max(nj, 8), max(nk, 8), 2)
        want = np.asfortranarray(O.make_level_set3(v, t, o, dx, ni, nj, nk, 1))
        rec, reps, name = None, 2, f"{ni}x{nj}x{nk}"
    else:
        name = sys.argv[2]
        reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
        v, t, o, dx, (ni, nj, nk) = meshgen.workload(name)
        with open(os.path.join(GOLDEN, "hashes.json")) as f:
            rec = json.load(f)[name]
        want = None
    print(f"library {os.path.basename(_lib.LIB_PATH)} build {_lib.build_id()}", flush=True)
    if "--cabi" in sys.argv:
        if rec is None:
            print("ERROR --cabi needs a named workload")
            return 1
        os.environ["SDFGEN_DEBUG_SLABS_ONE_DEVICE"] = "1"
        for rep in range(reps):
            phi = _lib.make_level_set3(v, t, o, dx, ni, nj, nk, 1, _lib.LAYOUT_ARRAY3, ngpu=nslabs)
            raw = np.asarray(phi, np.float32).ravel(order="F")   # i-fastest, the Array3f bytes
            got = hashlib.sha256(raw.astype("<f4", copy=False).tobytes()).hexdigest()
            inside = int(np.count_nonzero(raw < 0))
            if got != rec["sha256_phi"] or inside != rec["inside_lt0"]:
                print(f"MISMATCH {name} (C-ABI ngpu={nslabs}): sha256 {got[:16]} inside {inside} vs reference "
                      f"{rec['sha256_phi'][:16]} {rec['inside_lt0']}")
                return 1
        print(f"OK {nslabs} slabs {name} x{reps} (C-ABI ngpu)")
        return 0
    slabs = [_lib.Slab(0, nslabs, s, ni, nj, nk) for s in range(nslabs)]
    for s, sl in enumerate(slabs):
        sl.connect_local(slabs[s - 1] if s > 0 else None, slabs[s + 1] if s < nslabs - 1 else None)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    outs = [_hiprt.DeviceBuffer(ni * nj * (sl.k_end - sl.k_begin) * 4) for sl in slabs]
    for rep in range(reps):   # again: the second call reuses the inboxes (epochs keep counting)
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
        parts = [d.download(np.float32, ni * nj * (sl.k_end - sl.k_begin)) for sl, d in zip(slabs, outs)]
        if rec is None:
            got = np.concatenate(parts).reshape((ni, nj, nk), order="F")
            if not bits_equal(got, want):
                print("MISMATCH", diff_report(got, want, dx))
                return 1
        else:   # the slabs' i-fastest planes in k order are the whole grid's Array3f bytes
            h = hashlib.sha256()
            inside = 0
            for p in parts:
                h.update(p.astype("<f4", copy=False).tobytes())
                inside += int(np.count_nonzero(p < 0))
            if h.hexdigest() != rec["sha256_phi"] or inside != rec["inside_lt0"]:
                print(f"MISMATCH {name}: sha256 {h.hexdigest()[:16]} inside {inside} vs reference "
                      f"{rec['sha256_phi'][:16]} {rec['inside_lt0']}")
                return 1
            del parts
    print(f"OK {nslabs} slabs {name} x{reps}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
