set -u
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_SPARSE_WORKERS=256 SDFGEN_SPARSE_WORKERS=512 SDFGEN_SPARSE_WORKERS=384 > gpurun_out/r03_ab_workers_c4.log 2>&1; rc=$?; cat gpurun_out/r03_ab_workers_c4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_SPARSE_WORKERS=256 SDFGEN_SPARSE_WORKERS=512 > gpurun_out/r03_ab_workers_c3.log 2>&1; rc=$?; cat gpurun_out/r03_ab_workers_c3.log
