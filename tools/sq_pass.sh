#!/bin/bash
# tools/sq_pass.sh TAG WORKLOAD -- one SQ counter pass (occupancy / stall split) over a bench run of WORKLOAD
# with the library in use (SDFGEN_LIB_OVERRIDE honoured); per-kernel values -> gpurun_out/TAG_sq.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_sq.sh "$2" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" > gpurun_out/$1_sq.log 2>&1
rc=$?
cp profiles/pmc_sq_summary.json gpurun_out/$1_sq_summary.json 2>/dev/null
exit $rc
