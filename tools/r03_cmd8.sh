set -u
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/trace_multi.py c3_sphere1m_256 > gpurun_out/r03_trace2_c3.log 2>&1; rc=$?; cat gpurun_out/r03_trace2_c3.log; [ $rc -eq 0 ] || exit 1
