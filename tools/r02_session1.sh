#!/bin/bash
# round 2: kernel-trace profile of the C3 bench + the N=2 Z-slab bench path (both ranks on the one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof rc=$?"; tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats*"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2.log 2>&1; echo "n2 rc=$?"; tail -5 gpurun_out/bench_n2.log
