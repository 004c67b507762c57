set -u
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tile_cfg.py > gpurun_out/r03_pk_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03_pk_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/pk.so > gpurun_out/r03_ab_pk_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_pk_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/pk.so > gpurun_out/r03_ab_pk_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_pk_c4.log
