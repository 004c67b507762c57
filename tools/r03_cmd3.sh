export SDFGEN_BUG=$PWD/sdfgenfast_amd/build_bug/libsdfgen_hip_bounds_bug.so
SDFGEN_LIB_OVERRIDE=$SDFGEN_BUG GPU_MAX_HW_QUEUES=8 SDFGEN_TILE_GRID=96 timeout -k 10 200 python3 tests/slab_inprocess_check.py 2 c2_sphere70k_128 1 > gpurun_out/r03_bugdemo_c2.log 2>&1; rc=$?; echo "bugdemo c2 rc=$rc"; tail -3 gpurun_out/r03_bugdemo_c2.log
if [ $rc -gt 1 ]; then exit 1; fi
SDFGEN_LIB_OVERRIDE=$SDFGEN_BUG GPU_MAX_HW_QUEUES=8 SDFGEN_TILE_GRID=96 timeout -k 10 200 python3 tests/slab_inprocess_check.py 2 c3_sphere1m_256 1 > gpurun_out/r03_bugdemo_c3.log 2>&1; rc=$?; echo "bugdemo c3 rc=$rc"; tail -3 gpurun_out/r03_bugdemo_c3.log
if [ $rc -gt 1 ]; then exit 1; fi
bash tools/r03_session.sh r03b && timeout -k 10 600 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/w1rr4.so SDFGEN_LIB_OVERRIDE=ab/w1rr4p3.so > gpurun_out/r03_ab_w1_c4.log 2>&1; cat gpurun_out/r03_ab_w1_c4.log
