set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_bounds.py > gpurun_out/r03_u2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03_u2_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/u1.so SDFGEN_LIB_OVERRIDE=ab/u2.so > gpurun_out/r03_ab_u2_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_u2_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/u1.so SDFGEN_LIB_OVERRIDE=ab/u2.so > gpurun_out/r03_ab_u2_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_u2_c4.log
