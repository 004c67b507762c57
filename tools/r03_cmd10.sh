set -u
export TMPDIR=/tmp
rm -rf gpurun_out/r03_prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_c4 -o run -- python3 tools/ab_run.py c4_sphere1m_512 3 > gpurun_out/r03_prof_c4.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/r03_prof_c4.log; exit 1; }
find gpurun_out/r03_prof_c4 -name "*kernel_stats*"
