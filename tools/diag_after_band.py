"""Diagnostics (round 4): run right after tests/test_gpu_band.py in the same pytest process, so the
state that made its x3y4z5_prop64 call go wrong is still there; then probe which phase is wrong.
    python -m pytest tests/test_gpu_band.py tools/diag_after_band.py -m gpu -s -k "not batch_boxes_past" """
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import _lib, meshgen  # noqa: E402

pytestmark = pytest.mark.gpu


def _h(a):
    return hashlib.sha256(np.asfortranarray(a).ravel(order="F").astype("<f4").tobytes()).hexdigest()


def test_diag_after(monkeypatch):
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "hashes.json")))["x3y4z5_prop64"]
    v, t, o, dx, d = meshgen.workload("x3y4z5_prop64")
    for r in range(3):
        got = _lib.make_level_set3(v, t, o, dx, *d, 1, _lib.LAYOUT_ARRAY3)
        print(f"\nDIAG full call {r}: {'ok' if _h(got) == rec['sha256_phi'] else 'MISMATCH'}", flush=True)
    phi, ct, cnt, nb = _lib.debug_band(v, t, o, dx, *d, 1)
    wphi, wct, wcnt = O.band(v, t, o, dx, *d, exact_band=1)
    print(f"DIAG band: phi {int((phi.view(np.uint32) != wphi.view(np.uint32)).sum())} ct {int((ct != wct).sum())} "
          f"cnt {int((cnt.astype(np.int64) != wcnt).sum())} cells differ; big {nb}", flush=True)
    for ns in (1, 2, 4, 8, 16):
        monkeypatch.setenv("SDFGEN_DEBUG_NSWEEPS", str(ns))
        got = np.asfortranarray(_lib.make_level_set3(v, t, o, dx, *d, 1, _lib.LAYOUT_ARRAY3))
        p2, c2 = O.sweep(v, t, o, dx, wphi, wct, nsweeps=ns)
        par = np.cumsum(wcnt, axis=0) % 2 == 1
        want = np.where(par, -p2, p2)
        bad = got.view(np.uint32) != np.asfortranarray(want).view(np.uint32)
        idx = np.argwhere(bad)
        print(f"DIAG {ns} sweeps: {int(bad.sum())} cells differ; first {idx[:4].tolist()}; "
              f"multi {_lib.last_profile()['tile_multi']} cfg {_lib.last_profile()['tile_cfg']}", flush=True)
    monkeypatch.delenv("SDFGEN_DEBUG_NSWEEPS")
    monkeypatch.setenv("SDFGEN_SWEEP", "plane")
    got = _lib.make_level_set3(v, t, o, dx, *d, 1, _lib.LAYOUT_ARRAY3)
    print(f"DIAG plane sweeps: {'ok' if _h(got) == rec['sha256_phi'] else 'MISMATCH'}", flush=True)
