# tools/ab_pair.sh A.so B.so WORKLOAD... : interleaved A/B of two library builds (tools/ab_times.py) per workload
set -u
A=$1; B=$2; shift 2
for w in "$@"; do
  timeout -k 10 600 python3 tools/ab_times.py "$w" "$A" "$B" "$A" "$B" > "gpurun_out/ab_$w.log" 2>&1 || { echo "ab $w failed"; cat "gpurun_out/ab_$w.log"; exit 1; }
  echo "== $w"; cat "gpurun_out/ab_$w.log"
done
