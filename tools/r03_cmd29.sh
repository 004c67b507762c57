set -u
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_JLIST_MULT=32 SDFGEN_JLIST_MULT=16 SDFGEN_JLIST_MULT=8 SDFGEN_JLIST_MULT=4 > gpurun_out/r03_ab_jlist_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jlist_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_JLIST_MULT=32 SDFGEN_JLIST_MULT=16 SDFGEN_JLIST_MULT=8 > gpurun_out/r03_ab_jlist_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jlist_c4.log
