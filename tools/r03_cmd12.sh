set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_quick.log 2>&1 || { echo "quick tests failed"; tail -30 gpurun_out/r03e_quick.log; exit 1; }
tail -2 gpurun_out/r03e_quick.log
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_JACOBI_TILED=0 SDFGEN_JACOBI_TILED=1 > gpurun_out/r03_ab_jac_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jac_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_JACOBI_TILED=0 SDFGEN_JACOBI_TILED=1 > gpurun_out/r03_ab_jac_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jac_c4.log; [ $rc -eq 0 ] || exit 1
bash tools/r03_session.sh r03e tests
