#!/bin/bash
# tools/pmc_split.sh -- the per-buffer traffic split of the C3 first-pass launch:
# FETCH_SIZE and WRITE_SIZE passes (one counter per run) over the diagnostic builds
# ab/split{0..4}.so (tools/ab_build.sh splitV -DST_DIAG_SPLIT=V, built in the container), each
# stopping after the first pass (SDFGEN_DEBUG_NSWEEPS=8).  V = 0 is the unmodified kernel; the
# others take one buffer's accesses off the fabric (sweep_tile.hpp ST_DIAG_SPLIT).  Raw CSVs under
# gpurun_out/split_V_COUNTER/; reduce with tools/pmc_split.py.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${1:-c3_sphere1m_256}
for v in 0 1 2 3 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/split_${v}_$c
    echo "=== $(date +%T) split$v $c"
    SDFGEN_LIB_OVERRIDE=ab/split$v.so SDFGEN_DEBUG_NSWEEPS=8 \
      timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/split_${v}_$c -o run -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-side --no-latency --workload $W \
      > gpurun_out/split_${v}_$c.log 2>&1
  done
done
echo "=== split passes done"
