#!/bin/bash
# Per-sweep times with the sparse (Jacobi + repair) path starting at sweep N (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in 8 6 4 3 2; do
  echo "== SDFGEN_SPARSE_FROM=$n"
  SDFGEN_SPARSE_FROM=$n timeout -k 10 120 python tools/sweep_times.py ${1:-c3_sphere1m_256} || exit $?
done
