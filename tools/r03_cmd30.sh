set -u
export TMPDIR=/tmp
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/r03h_n4.log 2>&1 || { echo "n4 failed"; tail -30 gpurun_out/r03h_n4.log; exit 1; }
tail -1 gpurun_out/r03h_n4.log | cut -c1-1500
