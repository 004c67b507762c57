set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in js0 js3; do
  SDFGEN_LIB_OVERRIDE=ab/$v.so bash tools/pmc_sq.sh c4_sphere1m_512 > gpurun_out/sqab_${v}_a.log 2>&1 || exit $?
  SDFGEN_LIB_OVERRIDE=ab/$v.so bash tools/pmc_sq.sh c4_sphere1m_512 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" > gpurun_out/sqab_${v}_b.log 2>&1 || exit $?
  echo "== $v"; grep -i "jacobi" gpurun_out/sqab_${v}_a.log gpurun_out/sqab_${v}_b.log | cut -c1-400
done
