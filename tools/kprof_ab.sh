#!/bin/bash
# tools/kprof_ab.sh LIB [LIB ...] -- per-kernel averages (rocprofv3 --kernel-trace --stats) of A/B builds in ab/ at C3
# and C4 through bench.py (diagnostics only; "cur" = the in-tree library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do for w in c3_sphere1m_256 c4_sphere1m_512; do
  d=gpurun_out/kp_${v}_${w%%_*}; rm -rf $d
  lib=ab/$v.so; [ "$v" = cur ] && lib=
  SDFGEN_LIB_OVERRIDE=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-side --no-latency > $d.log 2>&1 || exit $?
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $v $w"; python3 - "$f" <<'P'
import csv,sys
for x in list(csv.DictReader(open(sys.argv[1])))[:6]: print(f"  {x['Name'][:45]:45s} {x['Calls']:>5s} {float(x['AverageNs'])/1000:9.1f} us")
P
done; done
