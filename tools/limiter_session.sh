#!/bin/bash
# tools/limiter_session.sh TAG WORKLOAD -- the counter passes that name a kernel's limiter (the
# Jacobi scan's rate): L2 hits / misses, TA and TD busy, L1 (TCP) accesses, requests to L2 and stalls, SQ memory
# instruction counts and waits.  One pass per counter block group; a pass that times out or is killed ends the
# session (rc >= 124).  Reduce here: python tools/pmc_passes.py profiles/<out>.json TAG_tcc TAG_ta ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; W=$2
run() {
  bash tools/pmc_pass.sh "${T_}_$1" "$W" "$2"
  local rc=$?
  echo "pass $1 rc=$rc"
  if [ $rc -ge 124 ]; then echo "FATAL: pass $1 rc=$rc, session stops"; exit $rc; fi
}
T_=$T
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
run ta "TA_BUSY_avr TA_BUSY_max"
run td "TD_BUSY_avr TD_BUSY_max"
run tcp "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
run sqm "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_ANY"
run grbm "GRBM_GUI_ACTIVE GRBM_COUNT"
