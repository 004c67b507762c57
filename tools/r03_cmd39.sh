set -u
export TMPDIR=/tmp
timeout -k 10 120 ./tools/pcie_write 67.108864 0 > gpurun_out/r03_pcie_write.log 2>&1; rc=$?; cat gpurun_out/r03_pcie_write.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/pcie_write 67.108864 4 > gpurun_out/r03_pcie_write_off4.log 2>&1; rc=$?; cat gpurun_out/r03_pcie_write_off4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -u tools/d2h_probe.py 67.1 > gpurun_out/r03_d2h_b.log 2>&1; rc=$?; head -3 gpurun_out/r03_d2h_b.log; [ $rc -eq 0 ] || exit 1
HSA_ENABLE_SDMA=0 timeout -k 10 120 python3 -u tools/d2h_probe.py 67.1 > gpurun_out/r03_d2h_nosdma.log 2>&1; rc=$?; cat gpurun_out/r03_d2h_nosdma.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/host_split.py c3_sphere1m_256 > gpurun_out/r03_host_split3.log 2>&1; rc=$?; cat gpurun_out/r03_host_split3.log; exit $rc
