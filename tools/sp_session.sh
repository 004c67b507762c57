set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -x -q 2>&1 | tail -2
for L in 0 1; do
echo "SDFGEN_SPARSE_LOCAL=$L"
SDFGEN_SPARSE_LOCAL=$L timeout -k 10 120 python tools/sweep_times.py
SDFGEN_SPARSE_LOCAL=$L timeout -k 10 120 python tools/sweep_times.py c4_sphere1m_512 | tail -1
done
