# tools/ab_multi.sh WORKLOAD A.so B.so ... : interleaved A/B of several library builds (tools/ab_times.py)
set -u
w=$1; shift
timeout -k 10 900 python3 tools/ab_times.py "$w" "$@" > "gpurun_out/abm_$w.log" 2>&1 || { echo "ab $w failed"; cat "gpurun_out/abm_$w.log"; exit 1; }
echo "== $w"; cat "gpurun_out/abm_$w.log"
