#!/bin/bash
# tools/pmc_pass.sh NAME WORKLOAD "COUNTERS" -- one rocprofv3 --pmc pass (counters only, no tracing domains) over a
# one-step bench run of WORKLOAD -> gpurun_out/pmcp_NAME/ (CSV) + gpurun_out/pmcp_NAME.log; reduce the passes
# here with tools/pmc_passes.py.  Keep each pass within the per-block limits (8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD,
# 2 GRBM): rocprofv3 does not split counters over passes (MI355X_MICROARCH.md).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
N=$1; W=$2; C=$3
rm -rf gpurun_out/pmcp_$N
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcp_$N -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-side --no-latency --workload $W > gpurun_out/pmcp_$N.log 2>&1
echo "pass $N ($W): $(ls gpurun_out/pmcp_$N/*/*counter_collection.csv gpurun_out/pmcp_$N/*counter_collection.csv 2>/dev/null | wc -l) csv"
