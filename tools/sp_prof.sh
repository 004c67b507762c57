set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for J in 0 1; do
rm -rf gpurun_out/spprof$J
SDFGEN_JACOBI=$J timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/spprof$J -o run -- python3 tools/sweep_times.py > gpurun_out/spprof$J.log 2>&1
grep total_ms gpurun_out/spprof$J.log
python3 - $J <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/spprof{sys.argv[1]}/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
seq=[(r['Kernel_Name'].split('(')[0][-14:],(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3) for r in rows]
seq=[s for s in seq if 'sp_' in s[0]][-16:]
print(' '.join(f"{n}:{t:.0f}" for n,t in seq))
PY
done
