set -u
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py tests/test_gpu_bounds.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/r03_inplace_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_inplace_tests.log; exit 1; }
tail -2 gpurun_out/r03_inplace_tests.log
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_SPARSE_INPLACE=0 SDFGEN_SPARSE_INPLACE=1 > gpurun_out/r03_ab_inplace_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_inplace_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_SPARSE_INPLACE=0 SDFGEN_SPARSE_INPLACE=1 > gpurun_out/r03_ab_inplace_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_inplace_c4.log
