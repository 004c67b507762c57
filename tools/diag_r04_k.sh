set -u
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 300 --timeout-method thread -k "not batch_boxes_past" > gpurun_out/r04k_1.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "tile watchdog|gave up|slot 7|stream|task .* = tile|passed|failed" gpurun_out/r04k_1.log | head -30
exit 0
