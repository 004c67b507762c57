set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -x -q 2>&1 | tail -2
timeout -k 10 120 python tools/sweep_times.py
timeout -k 10 120 python tools/sweep_times.py c4_sphere1m_512 | tail -1
