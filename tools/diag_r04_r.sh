# which earlier tests of tests/test_gpu_band.py make the first x3y4z5_prop64 call fail (3 fresh processes each)
set -u
T=tests/test_gpu_band.py
for sel in "fixture_inputs or coarse_random or c_abi or generate_sdf or two_slabs" "fixture_inputs" "coarse_random" "c_abi" "generate_sdf" "two_slabs" \
           "fixture_inputs or coarse_random or c_abi or generate_sdf" "fixture_inputs or coarse_random or two_slabs" "c_abi or generate_sdf or two_slabs"; do
  res=""
  for r in 1 2 3; do
    timeout -k 10 120 python3 -u -m pytest $T -m gpu -q -p no:randomly --timeout 100 --timeout-method thread -k "($sel) or prop64" > gpurun_out/r04r.log 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "[$sel] rc=$rc (stopping)"; tail -5 gpurun_out/r04r.log; exit $rc; }
    res="$res $rc"
  done
  echo "[$sel] rcs:$res"
done
exit 0
