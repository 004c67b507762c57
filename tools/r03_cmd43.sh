set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_map or full_size" > gpurun_out/r03_hm_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/r03_hm_new.log | tail -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/r03_hm_gputests.log 2>&1; rc=$?; grep -E "FAIL|Error" gpurun_out/r03_hm_gputests.log | tail -20; tail -3 gpurun_out/r03_hm_gputests.log; [ $rc -eq 0 ] || exit 1
for v in 0 3 0 3; do SDFGEN_HOST_MAP=$v timeout -k 10 120 python3 -u tools/host_rate.py c3_sphere1m_256 5 >> gpurun_out/r03_hm_rate.log 2>&1 || exit 1; echo "^ SDFGEN_HOST_MAP=$v" >> gpurun_out/r03_hm_rate.log; done; cat gpurun_out/r03_hm_rate.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03_hm_bench.json.log 2>&1; rc=$?; tail -c 1500 gpurun_out/r03_hm_bench.json.log; exit $rc
