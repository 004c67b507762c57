set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in wnohwb wideb; do
SDFGEN_LIB_OVERRIDE=ab/$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tile_cfg.py -m gpu -q --timeout 120 --timeout-method thread -k "quad" > gpurun_out/r05t_parity_$v.log 2>&1
rc=$?; echo "parity $v rc=$rc"; tail -1 gpurun_out/r05t_parity_$v.log
if [ $rc -ge 124 ]; then exit $rc; fi
done
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 X=1 SDFGEN_LIB_OVERRIDE=ab/basenr.so SDFGEN_LIB_OVERRIDE=ab/wnohwb.so SDFGEN_LIB_OVERRIDE=ab/wideb.so > gpurun_out/r05t_ab_c3.log 2>&1
echo "ab rc=$?"; cut -c1-200 gpurun_out/r05t_ab_c3.log
