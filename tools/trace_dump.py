"""Dump per-task (start, first, mid, end) trace of one tile sweep to gpurun_out/trace_s<S>.npy (diagnostics)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _lib, meshgen
name = sys.argv[1]
v, t, o, dx, dims = meshgen.workload(name)
os.makedirs("gpurun_out", exist_ok=True)
for sw in map(int, sys.argv[2:]):
    os.environ["SDFGEN_TRACE_SWEEP"] = str(sw)
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
    _lib.make_level_set3(v, t, o, dx, *dims, 1)
    p = _lib.last_profile()
    tr = _lib.debug_sweep_trace().astype(np.int64)
    np.save(f"gpurun_out/trace_s{sw}.npy", tr)
    print(sw, p["sweep_launch_ms"][sw], tr.shape, flush=True)
