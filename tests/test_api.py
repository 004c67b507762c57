"""The Python drop-in (sdfgenfast_amd, also importable as `sdfgen`) mirrors the
reference's own Python tests (python/tests/test_sdfgen.py, 9 classes / 51 tests):
same call shapes, defaults, dtype conversions and error contracts.  These run
on CPU (backend "cpu", or "auto" on a GPU-less host); the GPU path is covered
by tests/test_gpu_parity.py."""
import os
import tempfile

import numpy as np
import pytest

import sdfgen  # the drop-in package name (sdfgen/__init__.py re-exports sdfgenfast_amd)
import sdfgenfast_amd
from conftest import bits_equal


@pytest.fixture
def simple_cube():
    # python/tests/test_sdfgen.py:15-65
    v = np.array([[-0.5, -0.5, -0.5], [0.5, -0.5, -0.5], [0.5, 0.5, -0.5], [-0.5, 0.5, -0.5],
                  [-0.5, -0.5, 0.5], [0.5, -0.5, 0.5], [0.5, 0.5, 0.5], [-0.5, 0.5, 0.5]], np.float32)
    t = np.array([[0, 1, 2], [0, 2, 3], [4, 6, 5], [4, 7, 6], [0, 3, 7], [0, 7, 4],
                  [1, 5, 6], [1, 6, 2], [0, 4, 5], [0, 5, 1], [3, 2, 6], [3, 6, 7]], np.uint32)
    return v, t


@pytest.fixture
def temp_obj_file(simple_cube):
    v, t = simple_cube
    with tempfile.NamedTemporaryFile(mode="w", suffix=".obj", delete=False) as f:
        for p in v:
            f.write(f"v {p[0]} {p[1]} {p[2]}\n")
        for q in t:
            f.write(f"f {q[0]+1} {q[1]+1} {q[2]+1}\n")
        path = f.name
    yield path
    os.unlink(path)


@pytest.fixture
def temp_sdf_file():
    with tempfile.NamedTemporaryFile(suffix=".sdf", delete=False) as f:
        path = f.name
    yield path
    if os.path.exists(path):
        os.unlink(path)


def test_sdfgen_alias_is_the_same_package():
    assert sdfgen.generate_sdf is sdfgenfast_amd.generate_sdf
    for name in ("load_mesh", "generate_sdf", "save_sdf", "load_sdf", "is_gpu_available",
                 "generate_from_mesh", "generate_from_file"):
        assert hasattr(sdfgen, name)


class TestBasicFunctionality:
    def test_generate_sdf_from_arrays(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, origin=(-1.0, -1.0, -1.0), dx=0.1, nx=20, ny=20, nz=20, backend="cpu")
        assert sdf.shape == (20, 20, 20) and sdf.dtype == np.float32
        assert sdf[10, 10, 10] < 0      # centre inside  (test_sdfgen.py:108-130)
        assert sdf[0, 0, 0] > 0         # corner outside

    def test_load_mesh_from_file(self, temp_obj_file):
        v, t, bounds = sdfgen.load_mesh(temp_obj_file)
        assert v.shape == (8, 3) and v.dtype == np.float32
        assert t.shape == (12, 3) and t.dtype == np.uint32
        assert np.allclose(bounds[0], (-0.5, -0.5, -0.5)) and np.allclose(bounds[1], (0.5, 0.5, 0.5))

    def test_generate_from_file(self, temp_obj_file):
        sdf, meta = sdfgen.generate_from_file(temp_obj_file, nx=16, backend="cpu")
        assert sdf.ndim == 3 and set(meta) == {"origin", "dx", "bounds", "backend"}

    def test_generate_from_mesh(self, simple_cube):
        v, t = simple_cube
        sdf, meta = sdfgen.generate_from_mesh(v, t, nx=32, padding=2, backend="cpu")
        assert sdf.shape == (36, 36, 36)

    def test_save_and_load_sdf(self, simple_cube, temp_sdf_file):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1.0, -1.0, -1.0), 0.1, 20, 20, 20, backend="cpu")
        sdfgen.save_sdf(temp_sdf_file, sdf, origin=(-1.0, -1.0, -1.0), dx=0.1)
        back, origin, dx, bounds = sdfgen.load_sdf(temp_sdf_file)
        assert bits_equal(back, sdf)
        assert np.allclose(origin, (-1, -1, -1)) and abs(dx - 0.1) < 1e-6
        assert os.path.getsize(temp_sdf_file) == 36 + 4 * 20 ** 3


class TestBackends:
    def test_is_gpu_available(self):
        assert isinstance(sdfgen.is_gpu_available(), bool)

    def test_cpu_backend(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, backend="cpu")
        assert sdf.shape == (20, 20, 20)

    def test_auto_backend(self, simple_cube):
        v, t = simple_cube
        a = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, backend="auto")
        b = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, backend="cpu")
        assert bits_equal(a, b)   # every backend gives the same bits (unlike the reference's 25*dx)


class TestParameters:
    @pytest.mark.parametrize("n", [8, 16, 32])
    def test_different_grid_sizes(self, simple_cube, n):
        v, t = simple_cube
        assert sdfgen.generate_sdf(v, t, (-1, -1, -1), 2.0 / n, n, n, n, backend="cpu").shape == (n, n, n)

    def test_non_uniform_grid(self, simple_cube):
        v, t = simple_cube
        assert sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 10, 20, 30, backend="cpu").shape == (10, 20, 30)

    @pytest.mark.parametrize("band", [0, 1, 2, 3, 5])
    def test_exact_band_parameter(self, simple_cube, band):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, exact_band=band, backend="cpu")
        assert np.isfinite(sdf).all()

    @pytest.mark.parametrize("threads", [0, 1, 2, 4, 8, 100])
    def test_num_threads_parameter(self, simple_cube, threads):
        v, t = simple_cube
        a = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, backend="cpu", num_threads=threads)
        b = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 20, 20, 20, backend="cpu", num_threads=1)
        assert bits_equal(a, b)   # deterministic for any thread count


class TestErrorHandling:
    def test_invalid_backend(self, simple_cube):
        v, t = simple_cube
        with pytest.raises(ValueError):
            sdfgen.generate_sdf(v, t, (0, 0, 0), 0.1, 10, 10, 10, backend="invalid")

    def test_invalid_mesh_file(self):
        with pytest.raises(Exception):
            sdfgen.load_mesh("/nonexistent/file.obj")

    def test_invalid_array_shapes(self):
        with pytest.raises(Exception):
            sdfgen.generate_sdf(np.zeros((3, 2), np.float32), np.zeros((1, 3), np.uint32), (0, 0, 0), 0.1,
                                10, 10, 10)

    def test_empty_mesh(self):
        with pytest.raises(ValueError):
            sdfgen.generate_sdf(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32), (0, 0, 0), 0.1,
                                10, 10, 10)

    @pytest.mark.parametrize("dims", [(0, 10, 10), (10, -1, 10), (10, 10, 0)])
    def test_invalid_grid_size(self, simple_cube, dims):
        v, t = simple_cube
        with pytest.raises(ValueError):
            sdfgen.generate_sdf(v, t, (0, 0, 0), 0.1, *dims)

    @pytest.mark.parametrize("dx", [0.0, -0.1])
    def test_bad_dx(self, simple_cube, dx):
        v, t = simple_cube
        with pytest.raises(ValueError):
            sdfgen.generate_sdf(v, t, (0, 0, 0), dx, 10, 10, 10)

    def test_generate_from_file_missing_parameters(self, temp_obj_file):
        with pytest.raises(ValueError):
            sdfgen.generate_from_file(temp_obj_file)

    def test_load_sdf_nonexistent_file(self):
        with pytest.raises(Exception):
            sdfgen.load_sdf("/nonexistent/file.sdf")

    def test_load_sdf_corrupted_file(self):
        with tempfile.NamedTemporaryFile(suffix=".sdf", delete=False) as f:
            f.write(b"garbage")
            path = f.name
        try:
            with pytest.raises(Exception):
                sdfgen.load_sdf(path)
        finally:
            os.unlink(path)

    def test_load_mesh_corrupted_file(self):
        with tempfile.NamedTemporaryFile(mode="w", suffix=".obj", delete=False) as f:
            f.write("this is not an obj file\n")
            path = f.name
        try:
            with pytest.raises(Exception):
                sdfgen.load_mesh(path)
        finally:
            os.unlink(path)

    def test_save_sdf_invalid_path(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 10, 10, 10, backend="cpu")
        with pytest.raises(Exception):
            sdfgen.save_sdf("/nonexistent/dir/x.sdf", sdf, (0, 0, 0), 0.1)

    def test_save_sdf_invalid_array(self, temp_sdf_file):
        with pytest.raises(Exception):
            sdfgen.save_sdf(temp_sdf_file, np.zeros((4, 4), np.float32), (0, 0, 0), 0.1)


class TestDataValidation:
    def test_wrong_vertex_dtype_is_converted(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v.astype(np.int32), t, (0, 0, 0), 0.1, 10, 10, 10, backend="cpu")
        assert sdf.shape == (10, 10, 10) and sdf.dtype == np.float32

    def test_wrong_triangle_dtype_is_converted(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t.astype(np.int32), (0, 0, 0), 0.1, 10, 10, 10, backend="cpu")
        assert sdf.shape == (10, 10, 10)

    def test_non_contiguous_arrays(self, simple_cube):
        v, t = simple_cube
        tmp = np.zeros((16, 3), np.float32)
        tmp[::2] = v
        a = sdfgen.generate_sdf(tmp[::2], t, (-1, -1, -1), 0.1, 10, 10, 10, backend="cpu")
        b = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.1, 10, 10, 10, backend="cpu")
        assert bits_equal(a, b)

    def test_out_of_bounds_indices_raise(self, simple_cube):
        v, _ = simple_cube
        with pytest.raises(IndexError):
            sdfgen.generate_sdf(v, np.array([[0, 1, 999], [1, 2, 3]], np.uint32), (0, 0, 0), 0.1, 10, 10, 10,
                                backend="cpu")

    def test_save_sdf_wrong_dtype(self, simple_cube, temp_sdf_file):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (0, 0, 0), 0.1, 10, 10, 10, backend="cpu")
        sdfgen.save_sdf(temp_sdf_file, sdf.astype(np.int32), (0, 0, 0), 0.1)
        back, _, _, _ = sdfgen.load_sdf(temp_sdf_file)
        assert back.dtype == np.float32 and back.shape == (10, 10, 10)

    def test_1d_arrays_rejected(self, simple_cube):
        v, t = simple_cube
        with pytest.raises(Exception):
            sdfgen.generate_sdf(v.flatten(), t, (0, 0, 0), 0.1, 10, 10, 10)
        with pytest.raises(Exception):
            sdfgen.generate_sdf(v, t.flatten(), (0, 0, 0), 0.1, 10, 10, 10)


class TestEdgeCases:
    def test_single_triangle_mesh(self):
        v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
        t = np.array([[0, 1, 2]], np.uint32)
        sdf = sdfgen.generate_sdf(v, t, (-0.5, -0.5, -0.5), 0.1, 20, 20, 20, backend="cpu")
        assert sdf.shape == (20, 20, 20) and np.isfinite(sdf).all()

    @pytest.mark.parametrize("n", [1, 2, 3])
    def test_minimum_grid_size(self, simple_cube, n):
        v, t = simple_cube
        assert sdfgen.generate_sdf(v, t, (-1, -1, -1), 1.0, n, n, n, backend="cpu").shape == (n, n, n)

    def test_degenerate_triangles(self):
        v = np.array([[0, 0, 0], [1, 0, 0], [2, 0, 0], [0, 1, 0]], np.float32)
        t = np.array([[0, 1, 2], [0, 0, 3], [1, 1, 1]], np.uint32)
        sdf = sdfgen.generate_sdf(v, t, (-1, -1, -1), 0.2, 15, 15, 15, backend="cpu")
        assert sdf.shape == (15, 15, 15)

    def test_mesh_far_from_origin(self, simple_cube):
        v, t = simple_cube
        vf = v + np.float32(1000)
        sdf = sdfgen.generate_sdf(vf, t, (999, 999, 999), 0.1, 20, 20, 20, backend="cpu")
        assert sdf[10, 10, 10] < 0 and sdf[0, 0, 0] > 0

    def test_proportional_sizing_shapes(self, simple_cube):
        v, t = simple_cube
        sdf, meta = sdfgen.generate_from_mesh(v, t, nx=20, padding=1, backend="cpu")
        assert sdf.shape == (22, 22, 22)

    def test_explicit_sizing_shapes(self, temp_obj_file):
        # test_sdfgen.py:636-643: nx=20, ny=30, nz=40, padding=1 -> (22, 32, 42)
        sdf, meta = sdfgen.generate_from_file(temp_obj_file, nx=20, ny=30, nz=40, padding=1, backend="cpu")
        assert sdf.shape == (22, 32, 42)

    def test_from_file_with_dx(self, temp_obj_file):
        sdf, meta = sdfgen.generate_from_file(temp_obj_file, dx=0.1, padding=2, backend="cpu")
        assert sdf.shape == (14, 14, 14) and meta["dx"] == 0.1


class TestSDFProperties:
    def test_zero_crossing_at_surface(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1.0, -1.0, -1.0), 0.1, 21, 21, 21, backend="cpu")
        # x = -0.5 is grid index 5 along i (origin -1, dx 0.1): |sdf| small on the face
        assert abs(sdf[5, 10, 10]) < 0.1

    def test_inside_negative_outside_positive(self, simple_cube):
        v, t = simple_cube
        sdf = sdfgen.generate_sdf(v, t, (-1.0, -1.0, -1.0), 0.1, 21, 21, 21, backend="cpu")
        assert sdf[10, 10, 10] < 0 and sdf[0, 0, 0] > 0 and sdf[20, 20, 20] > 0


def test_reference_stl_and_obj_resources_load():
    """The reference's own test meshes (tests/resources), copied into tests/golden as data."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "cases.npz"))
    v = z["x3y4z5_stl_32/vertices"]
    assert v.shape == (108, 3)   # binary STL: no de-duplication (mesh_io_stl.cpp:157-165)


def test_embedded_x3y4z5_mesh_matches_the_stl_file():
    """meshgen.x3y4z5() ships the reference's benchmark mesh as data (no test tree needed at run
    time); it must be exactly what the native loader reads from the STL file."""
    import os

    from sdfgenfast_amd import meshgen, meshio
    path = os.path.join(os.path.dirname(__file__), "golden", "resources", "test_x3y4z5_bin.stl")
    v, t = meshio.load_mesh(path)[:2]
    ev, et = meshgen.x3y4z5()
    assert ev.dtype == np.float32 and et.dtype == np.uint32
    assert np.array_equal(ev, np.asarray(v, np.float32)) and np.array_equal(et, np.asarray(t, np.uint32))


def test_sdfgen_ngpu_env_parsing(monkeypatch):
    """generate_sdf's GPU-count knob (SDFGEN_NGPU) parses like the C++ drop-in's ngpu_from_env."""
    import sdfgenfast_amd as S
    from sdfgenfast_amd import _lib
    for val, want in (("", _lib.NGPU_CURRENT), ("1", 1), ("all", _lib.NGPU_ALL), ("0", 0), ("8", 8)):
        monkeypatch.setenv("SDFGEN_NGPU", val)
        assert S._ngpu_from_env() == want, val
    monkeypatch.delenv("SDFGEN_NGPU")
    assert S._ngpu_from_env() == _lib.NGPU_CURRENT
    for bad in ("two", "-1", "2.5"):
        monkeypatch.setenv("SDFGEN_NGPU", bad)
        with pytest.raises(ValueError):
            S._ngpu_from_env()
