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
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-verify --no-side --no-latency --workload $W > gpurun_out/pmc_sq.log 2>&1
python3 tools/pmc_sq_summary.py "$W"
