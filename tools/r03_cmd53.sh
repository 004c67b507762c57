set -u
export TMPDIR=/tmp
timeout -k 10 600 bash tools/r02_nrank.sh 2; rc=$?; cp gpurun_out/bench_n2.log gpurun_out/r03k_n2_one_gpu_rehearsal.json.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/r02_nrank.sh 4; rc=$?; cp gpurun_out/bench_n4.log gpurun_out/r03k_n4_one_gpu_rehearsal.json.log; exit $rc
