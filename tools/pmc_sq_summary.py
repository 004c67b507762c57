"""Reduce gpurun_out/pmc_sq (rocprofv3 --pmc SQ_* counters) to per-launch values per kernel
-> profiles/pmc_sq_summary.json.  Usage: python tools/pmc_sq_summary.py WORKLOAD (run where the CSVs are:
gpurun merges gpurun_out/ back, so run it here after the GPU pass)."""
import csv, glob, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float)); disp = defaultdict(set)
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
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
    print(f"{n:42s} launches {d:3d} " + " ".join(f"{k}={v/d:.4g}" for k, v in sorted(c.items())))
    if n.strip():
        out["kernels"][n.strip()] = {"launches": d, **{k: v / d for k, v in sorted(c.items())}}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open("profiles/pmc_sq_summary.json", "w"), indent=1)
