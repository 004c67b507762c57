set -u
bash tools/diag_r04_quad.sh > gpurun_out/r04e_quad.log 2>&1; rc=$?; echo "quad rc=$rc"; cat gpurun_out/r04e_quad.log | tail -30; [ $rc -ge 124 ] && exit $rc
timeout -k 5 200 python3 tools/stress_mix.py 120 1 > gpurun_out/r04e_stress.log 2>&1; rc=$?; echo "stress rc=$rc"; tail -5 gpurun_out/r04e_stress.log
timeout -k 5 300 python3 tools/fetch_calib.py gpurun_out/r04e_fetch_calib.json > gpurun_out/r04e_fetch_calib.log 2>&1; rc=$?; echo "calib rc=$rc"; tail -12 gpurun_out/r04e_fetch_calib.log
exit 0
