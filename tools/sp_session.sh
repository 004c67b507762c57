set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -2
timeout -k 10 120 python tools/sweep_times.py
timeout -k 10 300 python bench.py --workload c4_sphere1m_512 --steps 1 --warmup 1 --no-cpu-baseline | cut -c1-200
