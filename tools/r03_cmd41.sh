set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/hostmap_diag.py c3_sphere1m_256 0 1 2 3 > gpurun_out/r03_hm_diag_c3.log 2>&1; rc=$?; cat gpurun_out/r03_hm_diag_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u tools/hostmap_diag.py c4_sphere1m_512 0 1 2 3 > gpurun_out/r03_hm_diag_c4.log 2>&1; rc=$?; cat gpurun_out/r03_hm_diag_c4.log; exit $rc
