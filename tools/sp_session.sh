set -e
export TMPDIR=/tmp
rm -rf gpurun_out/prof_sp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o run -- python tools/sweep_times.py > /dev/null 2>&1
cut -c1-120 gpurun_out/prof_sp/run_kernel_stats.csv | head -8
