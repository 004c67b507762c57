set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/host_split.py > gpurun_out/r03_host_split.log 2>&1; rc=$?; cat gpurun_out/r03_host_split.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/pk.so > gpurun_out/r03_ab_pk2_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_pk2_c4.log
