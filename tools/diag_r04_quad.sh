set -u
# quad-lane tiles: parity first (stop on failure), then A/B timing at C3 / C2 / C4
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tile_cfg.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -8; rc=${PIPESTATUS[0]}
echo "tile_cfg tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_env.py c3_sphere1m_256 SDFGEN_TILE_CFG=0 SDFGEN_TILE_CFG=2; rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 tools/ab_env.py c2_sphere70k_128 SDFGEN_TILE_CFG=0 SDFGEN_TILE_CFG=2; rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 tools/ab_env.py c4_sphere1m_512 SDFGEN_TILE_CFG=1 SDFGEN_TILE_CFG=2; rc=$?; [ $rc -ge 124 ] && exit $rc
exit 0
