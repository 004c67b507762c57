#!/bin/bash
# round 3 GPU session: -m gpu suite, default bench line, kernel-trace profile, PMC passes (HBM + SQ)
# usage: bash tools/r03_session.sh TAG [tests|bench|prof|pmc ...]   (default: all steps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03}; shift || true
STEPS=${*:-tests bench prof pmc}
for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread \
      > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
    tail -3 gpurun_out/${TAG}_gputest.log ;;
  bench)
    timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
    tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600 ;;
  prof)
    rm -rf gpurun_out/${TAG}_prof
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/${TAG}_prof_bench.log 2>&1 \
      || { echo "rocprof rc=$?"; tail -20 gpurun_out/${TAG}_prof_bench.log; exit 1; }
    find gpurun_out/${TAG}_prof -name "*kernel_stats*" ;;
  pmc)
    bash tools/pmc.sh c3_sphere1m_256 > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
    bash tools/pmc_sq.sh c3_sphere1m_256 > gpurun_out/${TAG}_pmc_sq.log 2>&1 || { echo "pmc_sq rc=$?"; tail -20 gpurun_out/${TAG}_pmc_sq.log; exit 1; }
    echo pmc done ;;
  esac
done
