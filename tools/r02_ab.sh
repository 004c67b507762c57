#!/bin/bash
# A/B session: GPU parity tests, step profile of ab/prof.so, interleaved timing of ab/*.so variants vs the in-tree build
# usage: bash tools/r02_ab.sh "variant1 variant2 ..." [workload] [pytest-args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
VARS=${1:-}; WL=${2:-c3_sphere1m_256}; PT=${3:-tests/test_gpu_parity.py}
timeout -k 10 400 python3 -u -m pytest $PT -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
[ $rc -ne 0 ] && exit $rc
if [ -f ab/prof.so ]; then
  SDFGEN_LIB_OVERRIDE=ab/prof.so SDFGEN_COUNT_EVALS=1 timeout -k 10 200 python3 tools/step_prof.py $WL > gpurun_out/ab_prof.log 2>&1 || exit $?
  cat gpurun_out/ab_prof.log
fi
args="X=1"
for v in $VARS; do args="$args SDFGEN_LIB_OVERRIDE=ab/$v.so"; done
timeout -k 10 500 python3 tools/ab_env.py $WL $args 2>&1 | tee gpurun_out/ab_times.log
