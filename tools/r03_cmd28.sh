set -u
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/base.so SDFGEN_LIB_OVERRIDE=ab/hs4.so SDFGEN_LIB_OVERRIDE=ab/hs64.so > gpurun_out/r03_ab_hsleep_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_hsleep_c3.log; [ $rc -eq 0 ] || exit 1
for L in base hs4 hs64; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/hs_${L}_$c
    SDFGEN_LIB_OVERRIDE=ab/$L.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/hs_${L}_$c -o run -- python3 tools/ab_run.py c3_sphere1m_256 2 > gpurun_out/hs_${L}_$c.log 2>&1 || { echo "pmc $L $c failed"; exit 1; }
  done
done
echo done
