set -u
timeout -k 5 120 ./tools/hostreg_probe > gpurun_out/r04g_hostreg.log 2>&1; echo "hostreg rc=$?"; cat gpurun_out/r04g_hostreg.log
for v in full noslab slabonly; do
  timeout -k 5 200 python3 tools/repro_slab_then.py 4 $v > gpurun_out/r04g_repro_$v.log 2>&1; rc=$?; echo "repro $v rc=$rc"; cat gpurun_out/r04g_repro_$v.log | tail -30; [ $rc -ge 124 ] && exit $rc
done
exit 0
