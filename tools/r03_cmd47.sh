set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/c5_time.py > gpurun_out/r03j_c5_time.log 2>&1; rc=$?; tail -4 gpurun_out/r03j_c5_time.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/r02_nrank.sh 2; rc=$?; cp gpurun_out/bench_n2.log gpurun_out/r03j_n2_one_gpu_rehearsal.json.log; [ $rc -eq 0 ] || exit 1
