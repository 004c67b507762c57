set -u
for v in dband_coarse whole_coarse dband_coarse; do
  timeout -k 5 120 python3 tools/repro_band_then.py $v 2>&1 | grep -E "ok|MISMATCH|ERROR|tile watchdog|gave up|stream|= tile"; rc=${PIPESTATUS[0]}; [ $rc -ge 124 ] && exit $rc
done
exit 0
