set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/r03_brick_tests2.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_brick_tests2.log; exit 1; }
tail -2 gpurun_out/r03_brick_tests2.log
