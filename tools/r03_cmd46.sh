set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "staged or full_size or generate_sdf" > gpurun_out/r03_stage2_new.log 2>&1; rc=$?; grep -E "FAIL|Error" gpurun_out/r03_stage2_new.log | tail; tail -2 gpurun_out/r03_stage2_new.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/host_stage_diag.py c3_sphere1m_256 0 1 0 1 > gpurun_out/r03_stage2_diag_c3.log 2>&1; rc=$?; cat gpurun_out/r03_stage2_diag_c3.log; [ $rc -eq 0 ] || exit 1
SDFGEN_COPY_THREADS=4 timeout -k 10 300 python3 -u tools/host_stage_diag.py c3_sphere1m_256 1 > gpurun_out/r03_stage2_diag_c3_t4.log 2>&1; rc=$?; cat gpurun_out/r03_stage2_diag_c3_t4.log; [ $rc -eq 0 ] || exit 1
SDFGEN_COPY_THREADS=16 timeout -k 10 300 python3 -u tools/host_stage_diag.py c3_sphere1m_256 1 > gpurun_out/r03_stage2_diag_c3_t16.log 2>&1; rc=$?; cat gpurun_out/r03_stage2_diag_c3_t16.log; [ $rc -eq 0 ] || exit 1
SDFGEN_STAGE_CHUNK_KB=8192 timeout -k 10 300 python3 -u tools/host_stage_diag.py c3_sphere1m_256 1 > gpurun_out/r03_stage2_diag_c3_c8.log 2>&1; rc=$?; cat gpurun_out/r03_stage2_diag_c3_c8.log
