#!/bin/bash
# tools/kprof_env.sh TAG WORKLOAD [VAR=VALUE ...] -- per-kernel times (rocprofv3 --kernel-trace --stats) of a short
# bench run of WORKLOAD with the given environment -> gpurun_out/TAG_kprof/ (+ the stats table on stdout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; W=$2; shift 2
rm -rf "gpurun_out/${T}_kprof"
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${T}_kprof" -o run -- \
  python3 bench.py --workload "$W" --steps 5 --warmup 1 --no-cpu-baseline --no-side --no-latency > "gpurun_out/${T}_kprof.log" 2>&1
rc=$?
f=$(find "gpurun_out/${T}_kprof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv
for x in list(csv.DictReader(open('$f')))[:8]: print('%-60s %4s %10.1f us' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e3))"
exit $rc
