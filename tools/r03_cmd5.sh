set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tile_cfg.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c_tilecfg.log 2>&1 || { echo "tile cfg tests failed"; tail -30 gpurun_out/r03c_tilecfg.log; exit 1; }
tail -2 gpurun_out/r03c_tilecfg.log
bash tools/r03_session.sh r03c tests bench || exit 1
timeout -k 10 60 ./tools/uc_lat > gpurun_out/r03c_uc_lat.log 2>&1 || { echo uc_lat failed; cat gpurun_out/r03c_uc_lat.log; exit 1; }
cat gpurun_out/r03c_uc_lat.log
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r03c_n2.log 2>&1 || { echo "n2 failed"; tail -20 gpurun_out/r03c_n2.log; exit 1; }
tail -1 gpurun_out/r03c_n2.log | cut -c1-400
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/r03c_n4.log 2>&1 || { echo "n4 failed"; tail -20 gpurun_out/r03c_n4.log; exit 1; }
tail -1 gpurun_out/r03c_n4.log | cut -c1-400
