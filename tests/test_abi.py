"""The C-ABI library loads and exports every symbol include/*.h declares.
No compute calls here (runs without a GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from sdfgenfast_amd import _lib


def declared_functions():
    names = set()
    for h in ("sdfgen_hip.h", "sdfgen_cpu.h", "sdfgen_meshio.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:int|void|const char \*)\s*(sdfgen_\w+)\s*\(", src, flags=re.M))
    return sorted(names)


def test_header_declares_expected_entry_points():
    names = declared_functions()
    assert "sdfgen_hip_make_level_set3" in names
    assert "sdfgen_hip_device_count" in names
    assert "sdfgen_cpu_make_level_set3" in names
    assert set(names) == set(_lib.EXPORTED)


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports_symbol(name):
    assert hasattr(_lib.lib, name), name


def test_cxx_dropin_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "_ZN6sdfgen15make_level_set3" in out
    assert "_ZN6sdfgen16is_gpu_availableEv" in out


def test_build_id_matches_sources():
    """The library's embedded identity is the Makefile's hash of the current sources: a stale
    library (sources edited, not rebuilt) is detectable, and PMC summaries are matched on it."""
    want = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sdfgenfast_amd"), "build-id"],
                          capture_output=True, text=True, check=True).stdout.strip()
    assert re.fullmatch(r"[0-9a-f]{16}", want)
    assert _lib.build_id() == want


def test_abi_version_and_device_count():
    assert _lib.lib.sdfgen_hip_abi_version() == 5
    assert _lib.device_count() >= 0


def test_topology_without_gpu_is_empty_not_an_error():
    t = _lib.topology()
    assert t["devices"] == _lib.device_count()
    assert len(t["pci_bus_ids"]) == min(t["devices"], 16) and len(t["peer_access"]) == len(t["pci_bus_ids"])
    assert all(t["peer_access"][i][i] == 1 for i in range(len(t["peer_access"])))


def test_argument_validation_without_gpu():
    # validation happens before any device work: dims, dx, layout
    v = np.zeros((3, 3), np.float32)
    t = np.array([[0, 1, 2]], np.uint32)
    with pytest.raises(ValueError):
        _lib.make_level_set3(v, t, (0, 0, 0), 0.1, 0, 4, 4)
    with pytest.raises(ValueError):
        _lib.make_level_set3(v, t, (0, 0, 0), -0.1, 4, 4, 4)
    with pytest.raises(ValueError):
        _lib.make_level_set3(v, t, (0, 0, 0), float("nan"), 4, 4, 4)


@pytest.mark.skipif(_lib.device_count() > 0, reason="checks the no-device contract")
def test_gpu_entry_without_device_reports_gpu():
    v, t = np.eye(3, dtype=np.float32), np.array([[0, 1, 2]], np.uint32)
    with pytest.raises(RuntimeError, match="(?i)gpu"):
        _lib.make_level_set3(v, t, (0, 0, 0), 0.1, 4, 4, 4)


def test_no_oracle_in_product_library():
    """The product .so must not contain or reference the oracle."""
    out = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    deps = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in deps and "sdfref" not in deps


def test_negative_ngpu_is_einval():
    v, t = np.eye(3, dtype=np.float32), np.array([[0, 1, 2]], np.uint32)
    with pytest.raises(ValueError, match="ngpu"):
        _lib.make_level_set3(v, t, (0, 0, 0), 0.1, 4, 4, 4, ngpu=-1)
