set -u
i=0
for sel in "not batch_boxes_past" "not batch_boxes_past and not stage1" "not batch_boxes_past" "not batch_boxes_past and not stage1" "not batch_boxes_past"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/r04i_$i.log 2>&1; rc=$?
  echo "[$i: $sel] rc=$rc"; grep -E "tile watchdog|gave up|sweep slot 7|not done|passed|failed" gpurun_out/r04i_$i.log | head -12; [ $rc -ge 124 ] && exit $rc
done
exit 0
