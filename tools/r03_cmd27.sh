set -u
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_slab.py tests/test_gpu_distributed.py tests/test_gpu_bounds.py tests/test_gpu_tile_cfg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_slabip_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_slabip_tests.log; exit 1; }
tail -2 gpurun_out/r03_slabip_tests.log
for IP in 0 1; do
  SDFGEN_SPARSE_INPLACE=$IP timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$IP bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r03_slabip_n2_$IP.log 2>&1 || { echo "n2 failed"; tail -20 gpurun_out/r03_slabip_n2_$IP.log; exit 1; }
  tail -1 gpurun_out/r03_slabip_n2_$IP.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('inplace $IP', d['value'], d['ms_per_step'], d.get('phases_ms'), (d.get('zslab_c4') or {}).get('ms_per_step'), (d.get('zslab_c4') or {}).get('phases_ms'))"
done
