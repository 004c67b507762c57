#!/bin/bash
# SQ instruction counters per kernel (one rocprofv3 --pmc pass; counters only, no tracing).
# Usage: bash tools/pmc_sq.sh [workload] ["COUNTERS"]   -> gpurun_out/pmc_sq/ + summary on stdout
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${1:-c3_sphere1m_256}
C=${2:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
rm -rf gpurun_out/pmc_sq
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-side --workload $W > gpurun_out/pmc_sq.log 2>&1
python3 - "$W" <<'PY'
import csv, glob, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float)); disp = defaultdict(set)
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
        per[n][r["Counter_Name"]] += float(r["Counter_Value"]); disp[n].add(r["Dispatch_Id"])
import json, os
out = {"workload": sys.argv[1], "units": "per launch (summed over the chip's counter instances)", "kernels": {}}
for n, c in per.items():
    d = len(disp[n])
    print(f"{n:42s} launches {d:3d} " + " ".join(f"{k}={v/d:.4g}" for k, v in sorted(c.items())))
    if n.strip():
        out["kernels"][n.strip()] = {"launches": d, **{k: v / d for k, v in sorted(c.items())}}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open("profiles/pmc_sq_summary.json", "w"), indent=1)
PY
