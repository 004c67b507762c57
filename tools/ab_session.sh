#!/bin/bash
# tools/ab_session.sh TAG LIB [LIB ...] -- one A/B session on the GPU box for builds in ab/ (tools/ab_build.sh):
# the quad tile-configuration + parity suites on each, then interleaved C3 and C4 timings and the isolated
# tile step (ab/NAME.so; "cur" = the in-tree library).  Diagnostics only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
lib() { [ "$1" = cur ] && echo "" || echo "ab/$1.so"; }   # "cur": the in-tree library
# every library of the session must exist before anything runs (round 5 lost sessions to "ab/cur.so is
# missing": a build that was never made, or "cur" spelled as a file)
for v in "$@"; do
  f=$([ "$v" = cur ] && echo sdfgenfast_amd/libsdfgen_hip.so || echo "ab/$v.so")
  [ -f "$f" ] || { echo "ab_session: $f is missing -- build it first (tools/ab_build.sh); nothing run"; exit 2; }
done
cfgs=(); for v in "$@"; do cfgs+=("SDFGEN_LIB_OVERRIDE=$(lib $v)"); done
for v in "$@"; do
  [ "$v" = cur ] && continue
  SDFGEN_LIB_OVERRIDE=ab/$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tile_cfg.py tests/test_gpu_parity.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc: $(tail -1 gpurun_out/${TAG}_parity_$v.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
for w in c3_sphere1m_256 c4_sphere1m_512; do
  timeout -k 10 400 python3 tools/ab_env.py $w "${cfgs[@]}" > gpurun_out/${TAG}_ab_${w%%_*}.log 2>&1
  rc=$?; echo "ab $w rc=$rc"; cut -c1-200 gpurun_out/${TAG}_ab_${w%%_*}.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
for v in "$@"; do
  SDFGEN_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python3 tools/step_lat.py 2 > gpurun_out/${TAG}_steplat_$v.log 2>&1
  echo "step $v: $(tr '\n' ' ' < gpurun_out/${TAG}_steplat_$v.log)"
done
