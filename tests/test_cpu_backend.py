"""The library's native CPU backend (include/sdfgen_cpu.h) reproduces the
reference fixtures bit-for-bit for ANY thread count (the reference's own
multi-threaded sweep races)."""
import numpy as np
import pytest

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import _lib, meshgen


@pytest.mark.parametrize("threads", [1, 2, 5, 8])
def test_cpu_backend_matches_reference(golden_case, threads):
    c = golden_case
    out = _lib.cpu_make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, threads)
    assert bits_equal(out, c.phi), diff_report(out, c.phi, c.dx)


def test_cpu_backend_array3_layout(golden_case):
    c = golden_case
    out = _lib.cpu_make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, 3,
                                   layout=_lib.LAYOUT_ARRAY3)
    assert bits_equal(np.ascontiguousarray(out), c.phi)


def test_cpu_backend_vs_oracle_c2_subsample():
    v, t = meshgen.bumpy_sphere(120, 41)   # 9,600 triangles
    o, dx = meshgen.grid_mode2b(v, 48, 40, 56, 2)
    want = O.make_level_set3(v, t, o, dx, 48, 40, 56, 1)
    got = _lib.cpu_make_level_set3(v, t, o, dx, 48, 40, 56, 1, 0)
    assert bits_equal(got, np.ascontiguousarray(want)), diff_report(got, want, dx)


def test_cpu_backend_bad_index():
    v = np.eye(3, dtype=np.float32)
    t = np.array([[0, 1, 9]], np.uint32)
    with pytest.raises(IndexError):
        _lib.cpu_make_level_set3(v, t, (0, 0, 0), 0.1, 4, 4, 4, 1, 1)


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_backend_edge_semantics(edge_case, threads):
    """Far (> 2^31 cells), NaN and infinite vertices and wrapping exact_band values: the reference's
    own output (cpu_lib/makelevelset3.cpp:206-212, 222-233 on x86: int() -> INT_MIN, wrapping adds)."""
    c = edge_case
    with np.errstate(all="ignore"):
        out = _lib.cpu_make_level_set3(c.vertices, c.triangles, c.origin, c.dx, *c.dims, c.exact_band, threads)
    assert bits_equal(out, c.phi), diff_report(out, c.phi, c.dx)
