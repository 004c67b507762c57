set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03j_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r03j_smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u tools/fuzz_parity.py 240 4044 > gpurun_out/r03j_fuzz.log 2>&1; rc=$?; tail -2 gpurun_out/r03j_fuzz.log; exit $rc
