set -u
export TMPDIR=/tmp
SDFGEN_LIB_OVERRIDE=ab/twin4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tile_cfg.py -x -q -k "lat" --timeout 300 --timeout-method thread > gpurun_out/r03_twin4_tests.log 2>&1 || { echo "twin4 tests failed"; tail -30 gpurun_out/r03_twin4_tests.log; exit 1; }
tail -2 gpurun_out/r03_twin4_tests.log
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/twin4.so > gpurun_out/r03_ab_twin4_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_twin4_c3.log; [ $rc -eq 0 ] || exit 1
