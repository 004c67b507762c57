set -u
export TMPDIR=/tmp
SDFGEN_LIB_OVERRIDE=ab/prof.so SDFGEN_COUNT_EVALS=1 timeout -k 10 200 python3 tools/step_prof.py c3_sphere1m_256 c4_sphere1m_512 > gpurun_out/r03_stepprof.log 2>&1; rc=$?; cat gpurun_out/r03_stepprof.log; [ $rc -eq 0 ] || exit 1
SDFGEN_TILE_CFG=1 SDFGEN_LIB_OVERRIDE=ab/prof.so SDFGEN_COUNT_EVALS=1 timeout -k 10 200 python3 tools/step_prof.py c3_sphere1m_256 > gpurun_out/r03_stepprof_thr.log 2>&1; rc=$?; cat gpurun_out/r03_stepprof_thr.log
