"""The sequence that exposed the freed-uncached-memory failure, in a fresh
process: stage-1 band calls on every golden and edge fixture (they grow the one-GPU workspace), then
in-process two-slab calls on one GPU (their sessions allocate and destroy uncached communication
blocks), then the first one-GPU whole call -- against the reference's digest.  Before the
communication blocks were pooled this failed 3 runs in 3 (a digest mismatch or a tile watchdog).
    python tests/slab_then_one_gpu_check.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from conftest import EDGE_CASES, GOLDEN, GOLDEN_CASES, bits_equal  # noqa: E402
from sdfgenfast_amd import _lib, meshgen  # noqa: E402


def main():
    with np.errstate(all="ignore"):
        for c in GOLDEN_CASES + EDGE_CASES:
            _lib.debug_band(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band)
        os.environ["SDFGEN_DEBUG_SLABS_ONE_DEVICE"] = "1"
        os.environ["SDFGEN_TILE_GRID"] = "96"
        for name in ("far_nan_band40", "sphere_with_bad_tris", "far_z+300", "pinf_z"):
            c = next(e for e in EDGE_CASES if e.name == name)
            got = np.ascontiguousarray(_lib.make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims,
                                                            c.exact_band, _lib.LAYOUT_KFAST, ngpu=2))
            if not bits_equal(got, c.phi):
                print(f"MISMATCH two slabs {name}", flush=True)
                return 1
        del os.environ["SDFGEN_DEBUG_SLABS_ONE_DEVICE"], os.environ["SDFGEN_TILE_GRID"]
    with open(os.path.join(GOLDEN, "hashes.json")) as f:
        rec = json.load(f)["x3y4z5_prop64"]
    v, t, o, dx, dims = meshgen.workload("x3y4z5_prop64")
    got = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3)
    h = hashlib.sha256(np.asfortranarray(got).ravel(order="F").astype("<f4").tobytes()).hexdigest()
    if h != rec["sha256_phi"]:
        print("MISMATCH first one-GPU call after the slab sessions", flush=True)
        return 1
    print("OK", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
