#!/bin/bash
# tools/ab_band.sh TAG LIB [LIB ...] -- band A/B on the GPU box: the band + parity suites on each build in ab/,
# then interleaved C3 / C4 timings (diagnostics only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
cfgs=(); for v in "$@"; do cfgs+=("SDFGEN_LIB_OVERRIDE=ab/$v.so"); done
for v in "$@"; do
  SDFGEN_LIB_OVERRIDE=ab/$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_band.py tests/test_gpu_parity.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite_$v.log 2>&1
  rc=$?; echo "suite $v rc=$rc: $(tail -1 gpurun_out/${TAG}_suite_$v.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
for w in c3_sphere1m_256 c4_sphere1m_512; do
  timeout -k 10 400 python3 tools/ab_env.py $w "${cfgs[@]}" "${cfgs[@]}" > gpurun_out/${TAG}_ab_${w%%_*}.log 2>&1
  rc=$?; echo "ab $w rc=$rc"; cut -c1-200 gpurun_out/${TAG}_ab_${w%%_*}.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
