set -u
export TMPDIR=/tmp
SDFGEN_LIB_OVERRIDE=ab/J1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/r03_jc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03_jc_tests.log; exit 1; }
tail -2 gpurun_out/r03_jc_tests.log
timeout -k 10 500 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/J0.so SDFGEN_LIB_OVERRIDE=ab/J1.so > gpurun_out/r03_ab_jchunk_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jchunk_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_LIB_OVERRIDE=ab/J0.so SDFGEN_LIB_OVERRIDE=ab/J1.so > gpurun_out/r03_ab_jchunk_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_jchunk_c4.log; [ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/jc_prof
SDFGEN_LIB_OVERRIDE=ab/J1.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jc_prof -o run -- python3 tools/ab_run.py c3_sphere1m_256 4 > gpurun_out/jc_prof.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/jc_pmc_$c
  SDFGEN_LIB_OVERRIDE=ab/J1.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/jc_pmc_$c -o run -- python3 tools/ab_run.py c3_sphere1m_256 2 > gpurun_out/jc_pmc_$c.log 2>&1 || exit 1
done
echo done
