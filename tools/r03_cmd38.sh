set -u
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/d2h_probe.py 67.1 > gpurun_out/r03_d2h.log 2>&1; rc=$?; cat gpurun_out/r03_d2h.log; [ $rc -eq 0 ] || exit 1
GPU_PINNED_MIN_XFER_SIZE=1 timeout -k 10 120 python3 -u tools/d2h_probe.py 67.1 > gpurun_out/r03_d2h_pin1.log 2>&1; rc=$?; cat gpurun_out/r03_d2h_pin1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -u tools/host_rate.py c3_sphere1m_256 5 > gpurun_out/r03_host_rate.log 2>&1; rc=$?; cat gpurun_out/r03_host_rate.log; [ $rc -eq 0 ] || exit 1
GPU_PINNED_MIN_XFER_SIZE=1 timeout -k 10 120 python3 -u tools/host_rate.py c3_sphere1m_256 5 > gpurun_out/r03_host_rate_pin1.log 2>&1; rc=$?; cat gpurun_out/r03_host_rate_pin1.log
