#!/bin/bash
# tools/session.sh -- one parameterized gpurun session (replaces round 3's one-off tools/r03_cmdNN.sh).
# usage (on the box, from the repo root):
#   bash tools/session.sh TAG STEP [STEP ...]
# STEP is one of
#   tests            the whole -m gpu suite                          -> gpurun_out/TAG_gputest.log
#   t=SEL            a part of it: a test file / node id / -k expr  -> gpurun_out/TAG_t<n>.log
#                    (t=tests/test_gpu_band.py, t=-k:band_stage1, t=tests/test_gpu_parity.py::test_gpu_repeatable)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line                          -> gpurun_out/TAG_bench.log
#   bench=ARGS       bench.py with ARGS (commas for spaces: bench=--workload,x3y4z5_prop256,--no-side)
#   prof             rocprofv3 --kernel-trace --stats of bench C3    -> gpurun_out/TAG_prof/
#   prof=WORKLOAD    the same on another workload
#   pmc              HBM + SQ counter passes on C3 (tools/pmc.sh, tools/pmc_sq.sh)
#   py=SCRIPT,ARGS   python3 SCRIPT ARGS (a tools/ script)           -> gpurun_out/TAG_py<n>.log
#   exe=PROG,ARGS    a probe built here (tools/uc_free_probe,3)      -> gpurun_out/TAG_exe<n>.log
#                    (py=tools/fuzz_parity.py,200,3033  py=tools/c5_time.py  py=tools/wl_check.py,x3y4z5_prop256)
#   nrank=N          bench.py --gpus N under torch.distributed.run with all N ranks on this box's ONE GPU:
#                    a rehearsal of the Z-slab path (bit-exact check), not a scaling figure
#                                                                    -> gpurun_out/TAG_nN_one_gpu_rehearsal.json.log
# Every GPU step runs under its own time limit; a fault, abort or time-out (exit >= 124) ends the
# session at once, a failing test (pytest exit 1) is reported and the session goes on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:?usage: session.sh TAG STEP...}
shift
n=0
run() {  # logname timeout cmd...
  local log=gpurun_out/$1 tmo=$2
  shift 2
  echo "=== $(date +%T) $log: $*"
  local t0=$(date +%s)
  timeout -k 10 "$tmo" "$@" > "$log" 2>&1
  local rc=$?
  echo "=== rc=$rc ($(( $(date +%s) - t0 )) s)"
  tail -n 6 "$log" | cut -c1-400
  if [ "$rc" -ge 124 ]; then echo "FATAL rc=$rc in $log: session stops"; exit "$rc"; fi
  return 0
}
for s in "$@"; do
  n=$((n + 1))
  case $s in
  tests) run "${TAG}_gputest.log" 1000 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread ;;
  t=*)
    sel=${s#t=}
    if [[ $sel == -k:* ]]; then
      run "${TAG}_t$n.log" 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "${sel#-k:}"
    else
      run "${TAG}_t$n.log" 900 python3 -u -m pytest "$sel" -m gpu -v --timeout 600 --timeout-method thread
    fi ;;
  smoke) run "${TAG}_smoke.log" 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
  bench) run "${TAG}_bench.log" 600 python3 bench.py ;;
  bench=*)
    a=${s#bench=}
    run "${TAG}_bench$n.log" 600 python3 bench.py ${a//,/ } ;;
  prof|prof=*)
    w=c3_sphere1m_256
    [[ $s == prof=* ]] && w=${s#prof=}
    rm -rf "gpurun_out/${TAG}_prof_$w"
    run "${TAG}_prof_$w.log" 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof_$w" -o run -- \
      python3 bench.py --workload "$w" --steps 5 --warmup 1 --no-cpu-baseline --no-side --no-latency
    find "gpurun_out/${TAG}_prof_$w" -name "*kernel_stats*" ;;
  pmc)
    run "${TAG}_pmc.log" 600 bash tools/pmc.sh c3_sphere1m_256
    run "${TAG}_pmc_sq.log" 600 bash tools/pmc_sq.sh c3_sphere1m_256 ;;
  nrank=*)
    N=${s#nrank=}
    run "${TAG}_n${N}_one_gpu_rehearsal.json.log" 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $((29541 + n)) bench.py --gpus "$N" --steps 2 --warmup 1 --no-cpu-baseline ;;
  py=*)
    a=${s#py=}
    run "${TAG}_py$n.log" 900 python3 ${a//,/ } ;;
  exe=*)
    a=${s#exe=}
    run "${TAG}_exe$n.log" 300 ${a//,/ } ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session $TAG done"
