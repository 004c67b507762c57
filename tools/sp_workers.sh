#!/bin/bash
# Repair-kernel duration vs worker count (diagnostics): per-dispatch k_sp_* times from a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for wk in ${@:-16 64 128 512}; do
  rm -rf gpurun_out/spw
  SDFGEN_SPARSE_WORKERS=$wk timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/spw -o run -- \
    python3 tools/sweep_times.py > /dev/null 2>&1 || exit $?
  python3 - $wk <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob("gpurun_out/spw/**/*kernel_trace.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "k_sp_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-16:]
d = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"workers {sys.argv[1]:>4}: jacobi", " ".join(f"{d(r):6.0f}" for r in rows if "jacobi" in r["Kernel_Name"]),
      "| recheck", " ".join(f"{d(r):6.0f}" for r in rows if "recheck" in r["Kernel_Name"]), flush=True)
PY
done
