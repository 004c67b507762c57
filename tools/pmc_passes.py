"""Reduce tools/pmc_pass.sh passes to per-launch values per kernel:
    python tools/pmc_passes.py OUT.json NAME [NAME ...]   (reads gpurun_out/pmcp_NAME/; run here after the GPU call)
Every counter is summed over the chip's instances (rocprofv3 *_sum / per-XCD rows) and divided by the kernel's
dispatch count; the bench line of the first pass stamps the build id."""
import csv, glob, json, os, sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_sq_summary_lib import kernel_key  # noqa: E402

out_path, names = sys.argv[1], sys.argv[2:]
per = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
bid = None
for n in names:
    for f in glob.glob(f"gpurun_out/pmcp_{n}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    if bid is None and os.path.exists(f"gpurun_out/pmcp_{n}.log"):
        for line in reversed(open(f"gpurun_out/pmcp_{n}.log").read().splitlines()):
            if line.startswith("{"):
                bid = json.loads(line).get("build_id")
                break
res = {"build_id": bid, "passes": names, "units": "per launch, summed over the chip's counter instances", "kernels": {}}
for k, c in sorted(per.items()):
    vals = {cn: v / max(len(disp[k][cn]), 1) for cn, v in sorted(c.items())}
    res["kernels"][k] = {"launches": max(len(s) for s in disp[k].values()), **vals}
    print(f"{k:62s} " + " ".join(f"{cn}={v:.4g}" for cn, v in vals.items()))
json.dump(res, open(out_path, "w"), indent=1)
