set -u
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_band.py tools/diag_after_band.py -m gpu -q -s --timeout 300 --timeout-method thread -k "not batch_boxes_past" > gpurun_out/r04o.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "DIAG|^E  .*Error|tile watchdog|gave up|passed|failed" gpurun_out/r04o.log | head -30
bash tools/diag_r04_m.sh
SDFGEN_TILE_MULTI=0 SDFGEN_LIB_OVERRIDE=sdfgenfast_amd/libsdfgen_hip_bounds.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 200 --timeout-method thread -k "two_slabs" > gpurun_out/r04o_slab_bounds.log 2>&1; rc=$?
echo "slab multi=0 bounds rc=$rc"; grep -E "out-of-range|^E  .*Error|passed|failed" gpurun_out/r04o_slab_bounds.log | head -20
exit 0
