#!/bin/bash
# quick GPU diagnostics session: tools/gpu_diag.sh [workload]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/sweep_diag.py "${1:-c3_sphere1m_256}" 2 2>&1 | tee gpurun_out/diag.log
