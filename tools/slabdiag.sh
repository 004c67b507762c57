export SDFGEN_TILE_GRID=64
for c in "3 33 41 29" "3 33 40 29" "3 32 41 29" "3 33 41 30"; do
  echo "== $c"; timeout -k 5 90 python tests/slab_inprocess_check.py $c 2>&1 | tail -1
done
