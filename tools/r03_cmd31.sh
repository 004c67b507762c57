set -u
export TMPDIR=/tmp
timeout -k 10 260 python3 -u tools/fuzz_parity.py 200 3033 > gpurun_out/r03_fuzz_default.log 2>&1; rc=$?; tail -1 gpurun_out/r03_fuzz_default.log; [ $rc -eq 0 ] || exit 1
SDFGEN_SPARSE_FROM=0 timeout -k 10 260 python3 -u tools/fuzz_parity.py 200 3034 > gpurun_out/r03_fuzz_sparse.log 2>&1; rc=$?; tail -1 gpurun_out/r03_fuzz_sparse.log; [ $rc -eq 0 ] || exit 1
SDFGEN_SPARSE_FROM=0 SDFGEN_SPARSE_BRICK=1 timeout -k 10 200 python3 -u tools/fuzz_parity.py 140 3035 > gpurun_out/r03_fuzz_brick.log 2>&1; rc=$?; tail -1 gpurun_out/r03_fuzz_brick.log; [ $rc -eq 0 ] || exit 1
