set -u
export TMPDIR=/tmp
for L in ip; do
  echo "== $L"; SDFGEN_LIB_OVERRIDE=ab/$L.so timeout -k 10 120 python3 tools/ab_run.py c3_sphere1m_256 3 > gpurun_out/r03_ip_$L.log 2>&1 || { tail -5 gpurun_out/r03_ip_$L.log; exit 1; }
  tail -2 gpurun_out/r03_ip_$L.log
  SDFGEN_LIB_OVERRIDE=ab/$L.so timeout -k 10 200 python3 tools/ab_run.py c4_sphere1m_512 2 > gpurun_out/r03_ip_${L}_c4.log 2>&1 || { tail -5 gpurun_out/r03_ip_${L}_c4.log; exit 1; }
  tail -2 gpurun_out/r03_ip_${L}_c4.log
done
