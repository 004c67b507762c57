"""The C++ drop-in boundary, exercised by a compiled C++ caller (tests/cxx/dropin_caller.cpp).

Reference interface: sdfgen::make_level_set3 / sdfgen::is_gpu_available
(/root/reference/common/sdfgen_unified.h:47-57, 68) over Array3f =
Array3<float, Array1<float>> (common/array3.h:330, common/array1.h:76-79) and Vec3f/Vec3ui
(common/vec.h:25-28).

* CPU, build container only: the caller is compiled against the REFERENCE's headers
  (/root/reference/common) and linked against libsdfgen_hip.so alone -- it links (same
  mangled symbol) and reproduces the reference fixture bit for bit (same Array3f layout).
* CPU: the same caller compiled against this repository's headers (include/sdfgen).
* GPU: that caller on HardwareBackend::GPU against the golden fixtures.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_CASES, ROOT, bits_equal
from sdfgenfast_amd import _lib

SRC = os.path.join(ROOT, "tests", "cxx", "dropin_caller.cpp")
BUILD = os.path.join(ROOT, "tests", "cxx", "build")
OWN_BIN = os.path.join(BUILD, "dropin_caller_own")
REF = "/root/reference"
REF_COMMON = REF + "/common"
REF_INCLUDES = [REF + "/common", REF + "/cpu_lib", REF + "/gpu_lib"]
SHIM = os.path.join(ROOT, "integration", "makelevelset3_gpu_shim.cpp")
LIBDIR = os.path.dirname(_lib.LIB_PATH)
CASES = {c.name: c for c in GOLDEN_CASES}


def compile_caller(include_dirs, out):
    """g++ the caller against `include_dirs`; link libsdfgen_hip.so only."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    inc = [a for d in ([include_dirs] if isinstance(include_dirs, str) else include_dirs) for a in ("-I", d)]
    cmd = ["g++", "-O2", "-std=c++11", *inc, SRC, "-o", out,
           "-L", LIBDIR, "-lsdfgen_hip", f"-Wl,-rpath,{LIBDIR}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, f"compile failed: {' '.join(cmd)}\n{r.stderr[-3000:]}"
    return out


def own_caller():
    """The caller built against include/sdfgen (build() prebuilds it; rebuilt if stale)."""
    if not os.path.exists(OWN_BIN) or os.path.getmtime(OWN_BIN) < max(
            os.path.getmtime(SRC), os.path.getmtime(_lib.LIB_PATH)):
        compile_caller(os.path.join(ROOT, "include", "sdfgen"), OWN_BIN)
    return OWN_BIN


def write_mesh(path, case):
    t = np.ascontiguousarray(case.triangles, np.uint32)
    v = np.ascontiguousarray(case.vertices, np.float32)
    ni, nj, nk = case.dims
    with open(path, "wb") as f:
        np.array([len(t), len(v), ni, nj, nk, case.exact_band], np.int32).tofile(f)
        np.array(list(np.asarray(case.origin, np.float32)) + [case.dx], np.float32).tofile(f)
        t.tofile(f)
        v.tofile(f)


def run_caller(binary, case, backend, tmp_path):
    mesh, out = str(tmp_path / f"{case.name}.mesh"), str(tmp_path / f"{case.name}.phi")
    write_mesh(mesh, case)
    r = subprocess.run([binary, mesh, backend, out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    ni, nj, nk = case.dims
    # Array3f storage is i fastest: a[i + ni*(j + nj*k)] -> phi[i, j, k]
    return np.fromfile(out, np.float32).reshape(nk, nj, ni).transpose(2, 1, 0)


CPU_CASES = ["x3y4z5_stl_32", "cube_tiny_2x3x1", "degenerate_tris", "sphere3600_band3"]


@pytest.mark.skipif(not os.path.isdir(REF_COMMON), reason="reference headers exist only in the build container")
def test_reference_header_caller_links_and_matches(tmp_path):
    """A caller compiled against the reference's own headers links to libsdfgen_hip.so (no
    reference library) and gets the reference fixture bit-exact on HardwareBackend::CPU."""
    binary = compile_caller(REF_INCLUDES, str(tmp_path / "dropin_caller_ref"))
    syms = subprocess.run(["nm", "-u", binary], capture_output=True, text=True).stdout
    for sym in ("_ZN6sdfgen15make_level_set3", "_ZN6sdfgen3cpu15make_level_set3", "_ZN6sdfgen3gpu15make_level_set3"):
        assert sym in syms, sym  # resolved from our library, not compiled in
    for name in CPU_CASES:
        case = CASES[name]
        for mode in ("cpu", "cpu-direct"):
            got = run_caller(binary, case, mode, tmp_path)
            assert bits_equal(got, case.phi), (name, mode)
    r = subprocess.run([binary, "--errors"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.isdir(REF_COMMON), reason="reference headers exist only in the build container")
def test_integration_shim_compiles_against_reference_headers(tmp_path):
    """INTEGRATION.md §1's shim (integration/makelevelset3_gpu_shim.cpp) compiles against the
    reference's gpu_lib/common headers and defines exactly the reference's gpu symbol."""
    obj = str(tmp_path / "shim.o")
    cmd = ["g++", "-O2", "-std=c++11", "-c", SHIM, "-o", obj, "-I", REF + "/gpu_lib", "-I", REF_COMMON,
           "-I", os.path.join(ROOT, "include")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    defined = subprocess.run(["nm", "--defined-only", obj], capture_output=True, text=True).stdout
    undefined = subprocess.run(["nm", "-u", obj], capture_output=True, text=True).stdout
    gpu_syms = [w for w in defined.split() if w.startswith("_ZN6sdfgen3gpu15make_level_set3") and "." not in w]
    assert len(gpu_syms) == 1, defined
    gpu_sym = gpu_syms[0]
    assert "sdfgen_hip_make_level_set3" in undefined
    lib_syms = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert gpu_sym in lib_syms  # the library exports the same symbol itself


def test_own_header_caller_matches_on_cpu(tmp_path):
    binary = own_caller()
    for name in CPU_CASES:
        case = CASES[name]
        for mode in ("cpu", "cpu-direct"):
            assert bits_equal(run_caller(binary, case, mode, tmp_path), case.phi), (name, mode)
    r = subprocess.run([binary, "--errors"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_own_and_reference_symbols_agree():
    """The symbol this repository's header makes a caller import is the one the library exports."""
    binary = own_caller()
    want = [s for s in subprocess.run(["nm", "-u", binary], capture_output=True, text=True).stdout.split()
            if s.startswith("_ZN6sdfgen")]
    have = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert want and all(s in have for s in want), want


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["x3y4z5_stl_32", "cube_64", "sphere3600_40x44x52", "cube_tiny_1x5x4",
                                  "degenerate_tris", "random_soup"])
def test_gpu_cxx_caller_matches_fixture(name, tmp_path):
    case = CASES[name]
    for mode in ("gpu", "gpu-direct", "auto"):
        assert bits_equal(run_caller(own_caller(), case, mode, tmp_path), case.phi), (name, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("ngpu", ["2", "all"])
def test_gpu_cxx_caller_sdfgen_ngpu_knob(ngpu, tmp_path):
    """SDFGEN_NGPU, the drop-in's GPU-count knob (the reference signature has no device argument,
    common/sdfgen_unified.h:47-57): the C++ caller, unchanged, splits the grid into Z-slabs -- here two
    slab sessions on this box's one GPU (SDFGEN_DEBUG_SLABS_ONE_DEVICE; 'all' is the one device, so one
    slab) -- bit-exact against the reference fixture."""
    case = CASES["sphere3600_40x44x52"]
    env = dict(os.environ, SDFGEN_NGPU=ngpu, SDFGEN_DEBUG_SLABS_ONE_DEVICE="1", GPU_MAX_HW_QUEUES="8")
    mesh, out = str(tmp_path / "m.mesh"), str(tmp_path / "m.phi")
    write_mesh(mesh, case)
    for mode in ("gpu", "gpu-direct"):
        r = subprocess.run([own_caller(), mesh, mode, out], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        ni, nj, nk = case.dims
        got = np.fromfile(out, np.float32).reshape(nk, nj, ni).transpose(2, 1, 0)
        assert bits_equal(got, case.phi), (ngpu, mode)


def test_cxx_sdfgen_ngpu_rejects_garbage(tmp_path):
    """A malformed SDFGEN_NGPU is std::invalid_argument from the GPU drop-in (checked before any
    device work; on a box without a GPU the 'no GPU' error comes first, which is also an error)."""
    case = CASES["cube_tiny_1x5x4"]
    mesh, out = str(tmp_path / "m.mesh"), str(tmp_path / "m.phi")
    write_mesh(mesh, case)
    env = dict(os.environ, SDFGEN_NGPU="two")
    r = subprocess.run([own_caller(), mesh, "gpu", out], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    # the CPU backend ignores the knob
    r = subprocess.run([own_caller(), mesh, "cpu", out], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
