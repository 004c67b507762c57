set -u
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt37 -o kt -- python3 tools/kt_calls.py c3_sphere1m_256 4 > gpurun_out/r03_kt37.log 2>&1; rc=$?; tail -5 gpurun_out/r03_kt37.log; [ $rc -eq 0 ] || exit 1
f=$(find gpurun_out/kt37 -name "*kernel_trace.csv" | head -1); python3 tools/kt_gaps.py "$f" > gpurun_out/r03_kt_gaps_c3.log 2>&1; head -30 gpurun_out/r03_kt_gaps_c3.log
timeout -k 10 300 python3 -u tools/host_split.py c3_sphere1m_256 c4_sphere1m_512 > gpurun_out/r03_host_split2.log 2>&1; rc=$?; cat gpurun_out/r03_host_split2.log; exit $rc
