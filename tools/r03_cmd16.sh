set -u
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_LIB_OVERRIDE=ab/ov0.so SDFGEN_LIB_OVERRIDE=ab/ov1c0.so SDFGEN_LIB_OVERRIDE=ab/ov0.so,SDFGEN_SPARSE_WORKERS=64 SDFGEN_LIB_OVERRIDE=ab/ov1c0.so,SDFGEN_SPARSE_WORKERS=64 > gpurun_out/r03_ab_ov2_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_ov2_c3.log
