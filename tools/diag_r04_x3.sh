set -u
W=x3y4z5_prop64
for v in "" "SDFGEN_LIB_OVERRIDE=ab/old.so" "SDFGEN_TILE_MULTI=0" "SDFGEN_TILE_CFG=1" "SDFGEN_SWEEP=plane" "SDFGEN_SPARSE_FROM=16"; do
  env $v timeout -k 5 90 python3 tools/wl_check.py $W; rc=$?; echo "[$v] rc=$rc"; [ $rc -ge 124 ] && exit $rc
done
for W in x3y4z5_prop128 x3y4z5_prop256 tetra_512; do
  timeout -k 5 120 python3 tools/wl_check.py $W; rc=$?; echo "[$W] rc=$rc"; [ $rc -ge 124 ] && exit $rc
done
exit 0
