# the failing sequence (stage-1 tests, in-process two-slab calls, then the first one-GPU call) with
# the comm-block pool: 3 fresh processes, then the whole file
set -u
T=tests/test_gpu_band.py
res=""
for r in 1 2 3; do
  timeout -k 10 120 python3 -u -m pytest $T -m gpu -q --timeout 100 --timeout-method thread -k "fixture_inputs or coarse_random or two_slabs or prop64" > gpurun_out/r04s.log 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "rc=$rc (stopping)"; tail -5 gpurun_out/r04s.log; exit $rc; }
  res="$res $rc"
done
echo "sequence rcs:$res"
timeout -k 10 300 python3 -u -m pytest $T -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/r04s_all.log 2>&1; rc=$?
echo "whole file rc=$rc"; tail -3 gpurun_out/r04s_all.log
exit $rc
