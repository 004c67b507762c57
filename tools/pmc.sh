#!/bin/bash
# HBM traffic per kernel launch from rocprofv3 PMC counters (MI355X_MICROARCH.md "HBM"):
# FETCH_SIZE and WRITE_SIZE need separate passes; counters only, no tracing domains.
# Writes profiles/pmc_summary.json (+ the raw per-dispatch CSVs under gpurun_out/pmc_*).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${1:-c3_sphere1m_256}
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$c
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-side --no-latency --workload $W > gpurun_out/pmc_$c.log 2>&1
done
python3 tools/pmc_summary.py "$W"   # (writes profiles/ on the box; gpurun merges only gpurun_out/: rerun it here)
