set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "sweep_impls or golden" 2>&1 | tail -2
timeout -k 10 120 python tools/sweep_times.py
timeout -k 10 200 python tools/trace_diag.py c3_sphere1m_256 1 | tail -2
