#!/bin/bash
# round-2 profile session: kernel trace of the C3 bench (no isolated-tile launches mixed in),
# HBM bytes (FETCH_SIZE, WRITE_SIZE passes) and SQ instruction counters per kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side --no-latency > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof rc=$?"; tail -5 gpurun_out/prof_bench.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/prof_by_grid.csv | head -12
bash tools/pmc.sh c3_sphere1m_256 > gpurun_out/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc.log; exit 1; }
grep -A4 k_sweep_tile profiles/pmc_summary.json | head -8
bash tools/pmc_sq.sh c3_sphere1m_256 2>&1 | tail -12
