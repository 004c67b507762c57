set -u
for v in "X=1" "SDFGEN_TILE_MULTI=0" "SDFGEN_SPARSE_FROM=16" "SDFGEN_SPARSE_INPLACE=0" "X=2"; do
  env $v timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 300 --timeout-method thread -k "not batch_boxes_past" > gpurun_out/r04n.log 2>&1; rc=$?
  echo "[$v] rc=$rc"; grep -E "^E  .*Error|tile watchdog|gave up|stream|= tile|passed|failed" gpurun_out/r04n.log | head -20; [ $rc -ge 124 ] && exit $rc
done
exit 0
