set -u
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/sign_rate.py c3_sphere1m_256 c4_sphere1m_512 > gpurun_out/r03_sign_rate.log 2>&1; rc=$?; cat gpurun_out/r03_sign_rate.log; [ $rc -eq 0 ] || exit 1
bash tools/r03_session.sh r03d tests
