#!/bin/bash
# Z-slab bench path with N ranks on the one GPU (persistent grids capped by bench.py): correctness
# rehearsal of the multi-slab schedule, not a scaling measurement.  usage: bash tools/r02_nrank.sh N
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
N=${1:-4}
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus $N --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n$N.log 2>&1; rc=$?
echo "n$N rc=$rc"; grep -v "amdgpu.ids" gpurun_out/bench_n$N.log | tail -4
exit $rc
