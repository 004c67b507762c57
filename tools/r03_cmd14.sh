set -u
export TMPDIR=/tmp
SDFGEN_LIB_OVERRIDE=ab/pair2.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tile_cfg.py -x -q -k "thr" --timeout 300 --timeout-method thread > gpurun_out/r03_pair2_tests.log 2>&1 || { echo "pair2 tests failed"; tail -30 gpurun_out/r03_pair2_tests.log; exit 1; }
tail -2 gpurun_out/r03_pair2_tests.log
timeout -k 10 400 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/pair2.so > gpurun_out/r03_ab_pair2_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_pair2_c4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 tools/ab_env.py c5_sphere4m_1024 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/pair2.so > gpurun_out/r03_ab_pair2_c5.log 2>&1; rc=$?; cat gpurun_out/r03_ab_pair2_c5.log
