"""Time the reference's cpu_lib make_level_set3 (oracle/_ref, built from /root/reference) on ONE
thread of this host for a full workload -- the parity-valid CPU baseline (with more threads
its k-split sweep races).  Diagnostics / provenance for bench.py's cpu_baseline note.
    python tools/ref_1thread.py [WORKLOAD]"""
import json
import os
import platform
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from sdfgenfast_amd import meshgen  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
if not O.ref_available():
    sys.exit("oracle/_ref is not built (make -C oracle ref)")
v, t, o, dx, dims = meshgen.workload(name)
n = dims[0] * dims[1] * dims[2]
cpu = ""
try:
    cpu = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
except Exception:
    pass
print(f"timing the reference on 1 thread ({name}, {n} voxels) ...", flush=True)
t0 = time.perf_counter()
O.ref_make_level_set3(v, t, o, dx, *dims, 1, num_threads=1)
el = time.perf_counter() - t0
print(json.dumps({"workload": name, "seconds": round(el, 2), "mvoxels_per_s": round(n / el / 1e6, 4), "threads": 1,
                  "cpu": cpu, "machine": platform.machine()}), flush=True)
