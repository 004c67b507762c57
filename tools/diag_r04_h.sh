set -u
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h_band.log 2>&1; rc=$?; echo "band file rc=$rc"; grep -E "tile watchdog|sweep slot|not done|passed|failed|Error" gpurun_out/r04h_band.log | head -40; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not batch_boxes_past" > gpurun_out/r04h_band2.log 2>&1; rc=$?; echo "band file without the 2^32 batch rc=$rc"; grep -E "tile watchdog|sweep slot|not done|passed|failed|Error" gpurun_out/r04h_band2.log | head -40
exit 0
