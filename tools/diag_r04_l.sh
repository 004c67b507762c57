set -u
SDFGEN_LIB_OVERRIDE=sdfgenfast_amd/libsdfgen_hip_bounds.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 300 --timeout-method thread -k "not batch_boxes_past" > gpurun_out/r04l_1.log 2>&1; rc=$?
echo "bounds rc=$rc"; grep -E "out-of-range|tile watchdog|gave up|stream|task .* = tile|passed|failed|Error" gpurun_out/r04l_1.log | head -30
exit 0
