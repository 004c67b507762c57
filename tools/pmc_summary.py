"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs to HBM bytes per kernel launch.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reports half the bytes of wide coalesced reads -> doubled here; WRITE_SIZE
is taken as is.  Round 4 calibrated the widths the tile sweep uses (tools/fetch_calib.hip,
profiles/r04_fetch_calib.json): FETCH_SIZE counts 64 B per 128-B line for 8- and 16-byte, plain
and agent-scope loads alike, so the doubling holds for them; WRITE_SIZE counts 32-B granules (an
8-byte store alone in its line counts 32 B).
"""
import csv, glob, json, os, sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
work = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"
SHORT = {"k_sweep_tile": "k_sweep_tile", "k_sp_jacobi": "k_sp_jacobi", "k_sp_recheck": "k_sp_recheck",
         "k_band": "k_band", "k_sign": "k_sign", "k_init": "k_init", "k_prep_soup": "k_prep_soup"}


def load(counter):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{counter}", "**", "*counter_collection.csv"),
                      recursive=True)
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            key = next((v for k, v in SHORT.items() if k in name), None)
            if key:
                per[(key, row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    out = defaultdict(list)
    for (k, _), vals in per.items():
        out[k].append(sum(vals))   # sum over XCD / instance rows of one dispatch
    return out


def build_id_of(log):
    """The library build id the pass ran with: bench.py's JSON line in the pass's log."""
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line).get("build_id")
    return None


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
ids = {build_id_of(os.path.join(ROOT, "gpurun_out", f"pmc_{c}.log")) for c in ("FETCH_SIZE", "WRITE_SIZE")}
if len(ids) != 1 or None in ids:
    sys.exit(f"pmc passes ran with different or unknown library builds: {ids}")
kern = {}
for k in sorted(set(fetch) | set(write)):
    f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1) * 1024.0
    w = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1) * 1024.0
    kern[k] = {"launches_fetch": len(fetch.get(k, [])), "launches_write": len(write.get(k, [])),
               "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_per_launch": int(2 * f + w)}
res = {"workload": work, "build_id": ids.pop(), "units": "bytes per launch; FETCH_SIZE doubled (gfx950 wide-read correction)",
       "note": "FETCH doubling calibrated for 8- and 16-byte loads (profiles/r04_fetch_calib.json); WRITE_SIZE counts 32-B granules; byte-sized accesses uncalibrated; Infinity-Cache hits are counted",
       "kernels": kern}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
