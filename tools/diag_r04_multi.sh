set -u
timeout -k 5 120 python3 tools/trace_multi.py x3y4z5_prop64; rc=$?; echo "rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 5 120 python3 tools/wl_check.py x3y4z5_prop64 6; rc=$?; echo "rc=$rc"; [ $rc -ge 124 ] && exit $rc
SDFGEN_TILE_GRID=143 timeout -k 5 120 python3 tools/wl_check.py x3y4z5_prop64 3; rc=$?; echo "rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 5 120 python3 tools/trace_multi.py c2_sphere70k_128; rc=$?; echo "rc=$rc"
exit 0
