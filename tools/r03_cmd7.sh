set -u
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/trace_multi.py c3_sphere1m_256 > gpurun_out/r03_trace_c3.log 2>&1; rc=$?; cat gpurun_out/r03_trace_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/trace_multi.py c4_sphere1m_512 > gpurun_out/r03_trace_c4.log 2>&1; rc=$?; cat gpurun_out/r03_trace_c4.log; [ $rc -eq 0 ] || exit 1
SDFGEN_TILE_CFG=1 timeout -k 10 120 python3 tools/trace_multi.py c3_sphere1m_256 > gpurun_out/r03_trace_c3_thr.log 2>&1; rc=$?; cat gpurun_out/r03_trace_c3_thr.log
