set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/hs4.so SDFGEN_LIB_OVERRIDE=ab/cs4.so SDFGEN_LIB_OVERRIDE=ab/cs16.so > gpurun_out/r03_ab_sleep_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_sleep_c4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/cs4.so SDFGEN_LIB_OVERRIDE=ab/cs16.so > gpurun_out/r03_ab_sleep_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_sleep_c3.log
