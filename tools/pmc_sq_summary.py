"""Reduce gpurun_out/pmc_sq (rocprofv3 --pmc SQ_* counters) to per-launch values per kernel
-> profiles/pmc_sq_summary.json.  Usage: python tools/pmc_sq_summary.py WORKLOAD (run where the CSVs are:
gpurun merges gpurun_out/ back, so run it here after the GPU pass)."""
import csv, glob, re, sys
from collections import defaultdict


def kernel_key(full):
    """'void sdfhip::k_sweep_tile<sdfhip::StCfg<2, 8, true, 3>, false>(sdfhip::StParams)' ->
    'k_sweep_tile<StCfg<2, 8, true, 3>, false>': the name after its namespaces, then its template
    arguments (a namespace split inside them gave 'StCfg<...' and bench.py found no sweep kernel)."""
    head = re.sub(r"^void ", "", full.replace("(anonymous namespace)::", "")).split("(")[0]
    lt = head.find("<")
    base, targs = (head, "") if lt < 0 else (head[:lt], head[lt:])
    return (base.split("::")[-1] + targs.replace("sdfhip::", ""))[:60]


per = defaultdict(lambda: defaultdict(float)); disp = defaultdict(set)
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = kernel_key(r["Kernel_Name"])
        per[n][r["Counter_Name"]] += float(r["Counter_Value"]); disp[n].add(r["Dispatch_Id"])
import json, os
bid = None
for line in reversed(open("gpurun_out/pmc_sq.log").read().splitlines()):
    if line.startswith("{"):
        bid = json.loads(line).get("build_id")
        break
if not bid:
    sys.exit("gpurun_out/pmc_sq.log has no bench line with a build_id")
out = {"workload": sys.argv[1], "build_id": bid, "units": "per launch (summed over the chip's counter instances)", "kernels": {}}
for n, c in per.items():
    d = len(disp[n])
    print(f"{n:62s} launches {d:3d} " + " ".join(f"{k}={v/d:.4g}" for k, v in sorted(c.items())))
    if n.strip():
        out["kernels"][n.strip()] = {"launches": d, **{k: v / d for k, v in sorted(c.items())}}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open("profiles/pmc_sq_summary.json", "w"), indent=1)
