"""Reduce tools/pmc_split.sh's counter passes to the per-buffer traffic of one first-pass launch.

Each diagnostic build (sweep_tile.hpp ST_DIAG_SPLIT) takes one buffer's accesses off the fabric;
its difference to the unmodified kernel (V = 0) is that buffer's traffic.  FETCH_SIZE counts 64 B
per 128-B line fetched (profiles/r04_fetch_calib.json), so fetched line traffic = 2 x FETCH_SIZE;
WRITE_SIZE counts 32-B granules.  Writes profiles/r04_pmc_split.json.
usage: python3 tools/pmc_split.py [workload]
"""
import csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
work = sys.argv[1] if len(sys.argv) > 1 else "c3_sphere1m_256"


def per_launch(v, counter):
    """Mean bytes per k_sweep_tile launch (the counter's KiB summed over the dispatch's rows)."""
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"split_{v}_{counter}", "**", "*counter_collection.csv"),
                      recursive=True)
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter and "k_sweep_tile" in row["Kernel_Name"]:
                per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    if not per:
        sys.exit(f"no k_sweep_tile rows for split{v} {counter}")
    return sum(per.values()) / len(per) * 1024.0, len(per)


F, Wr, n = {}, {}, {}
for v in range(5):
    F[v], nf = per_launch(v, "FETCH_SIZE")
    Wr[v], nw = per_launch(v, "WRITE_SIZE")
    n[v] = (nf, nw)
line = {v: 2.0 * F[v] for v in F}   # fetched line traffic
split = {
    "cell stores (written)": Wr[0] - Wr[1],
    "halo granule stores and the rest of the writes": Wr[1],
    "own-label vertex gathers (fetched)": line[0] - line[2],
    "own cells (fetched)": line[2] - line[4],
    "halo vertex gathers (fetched)": line[0] - line[3],
}
split["halo granule polls and the rest of the fetches"] = line[0] - (split["own-label vertex gathers (fetched)"] +
                                                                     split["own cells (fetched)"] +
                                                                     split["halo vertex gathers (fetched)"])
res = {
    "workload": work,
    "what": "bytes per k_sweep_tile launch (the 8-sweep first pass), differential over ST_DIAG_SPLIT builds",
    "variants": {str(v): {"fetch_size_bytes_raw": F[v], "fetch_line_bytes": line[v], "write_bytes": Wr[v],
                          "launches_fetch_write": n[v]} for v in F},
    "split_bytes": split,
    "totals": {"fetched_line_bytes": line[0], "written_bytes": Wr[0], "hbm_bytes": line[0] + Wr[0]},
}
json.dump(res, open(os.path.join(ROOT, "profiles", "r04_pmc_split.json"), "w"), indent=1)
for k, b in split.items():
    print(f"{k:52s} {b / 1e9:7.3f} GB")
print(f"{'total fetched (lines) / written':52s} {line[0] / 1e9:7.3f} / {Wr[0] / 1e9:.3f} GB")
