set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -2
timeout -k 10 120 python tools/sweep_times.py
SDFGEN_COUNT_EVALS=1 SDFGEN_SPARSE_FROM=16 timeout -k 10 120 python tools/sweep_times.py | tail -1
