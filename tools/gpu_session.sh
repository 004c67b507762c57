#!/bin/bash
# tools/gpu_session.sh -- one gpurun session: GPU parity tests, smoke, bench, rocprof.
# Each GPU step has its own time limit; any fault/abort/timeout (exit >= 124 or
# signal) stops the session.  Test FAILURES (pytest exit 1) do not stop it.
# Usage (on the box): bash tools/gpu_session.sh [tests|bench|prof|all] [extra pytest args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="${1:-all}"; shift || true
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "=== $name: $*" ; local t0=$(date +%s)
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)"; tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m1 -E "gfx950" || echo "no gfx950 in rocminfo"
if [ "$what" = tests ] || [ "$what" = all ]; then
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@"
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  step bench 900 python bench.py --steps 3 --warmup 1
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  rm -rf gpurun_out/prof
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-side --no-latency
  find gpurun_out/prof -name "*stats*" | head
fi
echo "=== session done"
