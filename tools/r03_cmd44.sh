set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "staged or full_size" > gpurun_out/r03_stage_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/r03_stage_new.log | tail -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/host_stage_diag.py c3_sphere1m_256 0 1 0 1 > gpurun_out/r03_stage_diag_c3.log 2>&1; rc=$?; cat gpurun_out/r03_stage_diag_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/r03_stage_gputests.log 2>&1; rc=$?; grep -E "FAIL|Error" gpurun_out/r03_stage_gputests.log | tail -20; tail -3 gpurun_out/r03_stage_gputests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03_stage_bench.json.log 2>&1; rc=$?; tail -c 1500 gpurun_out/r03_stage_bench.json.log; exit $rc
