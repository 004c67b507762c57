set -u
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/r03_any_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_any_tests.log; exit 1; }
tail -2 gpurun_out/r03_any_tests.log
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/A0.so SDFGEN_LIB_OVERRIDE=ab/A1.so > gpurun_out/r03_ab_any_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_any_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/A0.so SDFGEN_LIB_OVERRIDE=ab/A1.so > gpurun_out/r03_ab_any_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_any_c4.log
