set -e
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_sp.log 2>&1 || (tail -40 gpurun_out/pytest_sp.log; exit 1)
tail -2 gpurun_out/pytest_sp.log
timeout -k 10 120 python tools/sweep_times.py
SDFGEN_NO_SEEN_SKIP=1 timeout -k 10 120 python tools/sweep_times.py
