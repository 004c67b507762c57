set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_hm_parity.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/r03_hm_parity.log | tail -25; exit $rc
