"""Shared fixtures.  `-m gpu` tests need a real MI355X and call the HIP path
through the C-ABI; everything else runs on CPU (oracle, host logic, C-ABI
symbol checks, the native CPU backend)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


class GoldenCase:
    def __init__(self, z, name):
        self.name = name
        self.vertices = z[f"{name}/vertices"]
        self.triangles = z[f"{name}/triangles"]
        self.origin = z[f"{name}/origin"]
        self.dx = float(z[f"{name}/dx"])
        self.dims = tuple(int(d) for d in z[f"{name}/dims"])
        self.exact_band = int(z[f"{name}/exact_band"])
        self.phi = z[f"{name}/phi"]  # sdf[i,j,k], C order (reference output)


def load_golden(fname="cases.npz"):
    z = np.load(os.path.join(GOLDEN, fname))
    return [GoldenCase(z, str(n)) for n in z["names"]]


GOLDEN_CASES = load_golden()
# far (> 2^31 cells), NaN and +-Inf vertices, wrapping exact_band values: the reference's own output
# (tests/golden/make_golden.py --edge)
EDGE_CASES = load_golden("edge_cases.npz")


@pytest.fixture(params=GOLDEN_CASES, ids=[c.name for c in GOLDEN_CASES])
def golden_case(request):
    return request.param


@pytest.fixture(params=EDGE_CASES, ids=[c.name for c in EDGE_CASES])
def edge_case(request):
    return request.param


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def diff_report(got, want, dx):
    got = np.asarray(got, np.float32)
    want = np.asarray(want, np.float32)
    bad = got.view(np.uint32) != want.view(np.uint32)
    if not bad.any():
        return "identical"
    idx = np.argwhere(bad)[:5]
    err = np.abs(got.astype(np.float64) - want.astype(np.float64))
    return (f"{bad.sum()} cells differ, max |diff| = {np.nanmax(err)/dx:.3g} dx, "
            f"sign mismatches = {(np.signbit(got) != np.signbit(want)).sum()}, first {idx.tolist()}")
