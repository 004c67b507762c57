set -u
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r03k_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r03k_gputest.log; [ $rc -eq 0 ] || exit 1
bash tools/r03_session.sh r03k bench prof pmc
