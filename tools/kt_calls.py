"""A few C3 calls for a rocprofv3 kernel trace (tools/kt_gaps.py reads the trace):
rocprofv3 --kernel-trace --output-format csv -d DIR -o kt -- python3 tools/kt_calls.py [workload] [calls]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sdfgenfast_amd import _lib, meshgen

wl = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
v, t, o, dx, dims = meshgen.workload(wl)
out = np.empty(dims[0] * dims[1] * dims[2], np.float32)
for _ in range(calls):
    _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out)
    print("total_ms", round(_lib.last_profile()["total_ms"], 3), flush=True)
