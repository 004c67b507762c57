#!/bin/bash
# second-pass session: GPU parity (parity + slab tests), repair profile, A/B vs variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/sp_pytest.log
[ $rc -ne 0 ] && exit $rc
SDFGEN_LIB_OVERRIDE=ab/spprof.so timeout -k 10 100 python3 tools/sp_diag.py c3_sphere1m_256 c4_sphere1m_512 2>&1 || exit $?
args="X=1"
for v in ${1:-}; do args="$args SDFGEN_LIB_OVERRIDE=ab/$v.so"; done
timeout -k 10 500 python3 tools/ab_env.py c3_sphere1m_256 $args 2>&1
