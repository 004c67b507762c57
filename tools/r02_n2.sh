#!/bin/bash
# the N=2 Z-slab bench path with both ranks on the one GPU (persistent grids capped by bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2.log 2>&1; echo "n2 rc=$?"; tail -3 gpurun_out/bench_n2.log
