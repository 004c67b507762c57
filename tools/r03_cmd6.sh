set -u
export TMPDIR=/tmp
SDFGEN_OCC=1 SDFGEN_LIB_OVERRIDE=ab/cur.so timeout -k 10 120 python3 tools/ab_run.py c4_sphere1m_512 1 2>&1 | grep -E "occupancy|calls" | sort | uniq
SDFGEN_OCC=1 SDFGEN_LIB_OVERRIDE=ab/rh4p3.so timeout -k 10 120 python3 tools/ab_run.py c4_sphere1m_512 1 2>&1 | grep -E "occupancy|calls" | sort | uniq
SDFGEN_OCC=1 SDFGEN_LIB_OVERRIDE=ab/g4.so timeout -k 10 120 python3 tools/ab_run.py c4_sphere1m_512 1 2>&1 | grep -E "occupancy|calls" | sort | uniq
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/cur.so SDFGEN_LIB_OVERRIDE=ab/rh4p3.so SDFGEN_LIB_OVERRIDE=ab/g4.so > gpurun_out/r03_ab_thr_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_thr_c4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 tools/ab_env.py c5_sphere4m_1024 SDFGEN_LIB_OVERRIDE=ab/cur.so SDFGEN_LIB_OVERRIDE=ab/rh4p3.so SDFGEN_LIB_OVERRIDE=ab/g4.so > gpurun_out/r03_ab_thr_c5.log 2>&1; rc=$?; cat gpurun_out/r03_ab_thr_c5.log
