set -u
export TMPDIR=/tmp
SDFGEN_SPARSE_WORKERS=256 timeout -k 10 300 python3 -u tools/c5_time.py > gpurun_out/r03_c5_w256.log 2>&1; rc=$?; tail -3 gpurun_out/r03_c5_w256.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/c5_time.py > gpurun_out/r03k_c5_time.log 2>&1; rc=$?; tail -3 gpurun_out/r03k_c5_time.log
