set -u
timeout -k 5 200 python3 tools/stress_mix.py 150 1; rc=$?; echo "rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 5 200 python3 -u -m pytest tests/test_gpu_band.py -m gpu -q --timeout 300 --timeout-method thread -x 2>&1 | tail -15
exit 0
