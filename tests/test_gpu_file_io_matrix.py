"""The resolution x padding matrix of the reference's file-I/O suite as a GPU parity matrix.

/root/reference/tests/test_file_io.cpp:122 runs grid resolutions {16, 32, 64, 128} at padding 2 and
:138 paddings {1, 2, 3, 5, 10} at resolution 32, sizing each grid with calculate_grid_parameters
(tests/test_utils.cpp:276-305: proportional, centred) on its unit cube (test_file_io.cpp:7-30), then
writes both backends' .sdf files, reads them back and compares them (tests/test_utils.cpp:131-220)
to 25 dx.  Here the same matrix -- on that cube and on the reference's benchmark mesh
test_x3y4z5_bin.stl -- must be BIT-exact against the oracle (pinned to the reference), through the
Python drop-in's generate_sdf -> save_sdf -> load_sdf round trip."""
import numpy as np
import pytest

from conftest import bits_equal, diff_report
from oracle import oracle as O
from sdfgenfast_amd import meshgen

pytestmark = pytest.mark.gpu

MATRIX = [(r, 2) for r in (16, 32, 64, 128)] + [(32, p) for p in (1, 3, 5, 10)]


@pytest.mark.parametrize("mesh", ["unit_cube", "x3y4z5"])
@pytest.mark.parametrize("res,padding", MATRIX, ids=[f"res{r}-pad{p}" for r, p in MATRIX])
def test_gpu_file_io_matrix(tmp_path, mesh, res, padding):
    import sdfgenfast_amd as S
    v, t = meshgen.unit_cube() if mesh == "unit_cube" else meshgen.x3y4z5()
    o, dx, dims = meshgen.grid_proportional(v, res, padding)
    want = O.make_level_set3(v, t, o, dx, *dims, exact_band=1)
    sdf = S.generate_sdf(v, t, tuple(float(x) for x in o), float(dx), *dims, backend="gpu")
    assert sdf.shape == dims
    assert bits_equal(sdf, want), diff_report(sdf, want, dx)
    path = str(tmp_path / "out.sdf")
    S.save_sdf(path, sdf, tuple(float(x) for x in o), float(dx))
    back, o2, dx2 = S.load_sdf(path)[:3]
    assert bits_equal(np.asarray(back), want)
    assert np.array_equal(np.asarray(o2, np.float32), np.asarray(o, np.float32))
