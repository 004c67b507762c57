set -u
bash tools/diag_r04_i.sh; rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 5 300 python3 tools/fetch_calib.py gpurun_out/r04j_fetch_calib.json > gpurun_out/r04j_fetch_calib.log 2>&1; rc=$?; echo "calib rc=$rc"; grep -E "^k_" gpurun_out/r04j_fetch_calib.log
exit 0
