set -u
L="SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/w1rr4.so SDFGEN_LIB_OVERRIDE=ab/w1rr4p3.so SDFGEN_LIB_OVERRIDE=ab/w1ro2p3.so"
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 $L > gpurun_out/r03_ab_w1_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_w1_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/w1ro2p3.so > gpurun_out/r03_ab_w1_c4b.log 2>&1; rc=$?; cat gpurun_out/r03_ab_w1_c4b.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 tools/ab_env.py c5_sphere4m_1024 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/w1rr4.so SDFGEN_LIB_OVERRIDE=ab/w1ro2p3.so > gpurun_out/r03_ab_w1_c5.log 2>&1; rc=$?; cat gpurun_out/r03_ab_w1_c5.log; [ $rc -eq 0 ] || exit 1
