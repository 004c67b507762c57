set -u
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/r03_brick_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_brick_tests.log; exit 1; }
tail -2 gpurun_out/r03_brick_tests.log
SDFGEN_LIB_OVERRIDE=ab/bp.so timeout -k 10 120 python3 tools/ab_run.py c3_sphere1m_256 2 > gpurun_out/r03_bp.log 2>&1 || { tail -5 gpurun_out/r03_bp.log; exit 1; }
tail -2 gpurun_out/r03_bp.log
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_SPARSE_BRICK=0 SDFGEN_SPARSE_BRICK=1 > gpurun_out/r03_ab_brick_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_brick_c3.log; [ $rc -eq 0 ] || exit 1
