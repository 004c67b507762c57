"""Per-kernel summary of a rocprofv3 --kernel-trace CSV, split by launch grid size.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [out.csv]

bench.py also launches the tile sweep on a 1024x9x9 grid (the isolated step time of
roofline.latency); rocprof's own kernel_stats.csv averages those launches with the workload's.
Grouping by (kernel, grid) keeps the workload's launches apart.
"""
import csv
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    d = defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0]
        d[(name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    total = sum(sum(v) for _, v in rows)
    out = [["kernel", "grid", "block", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "pct"]]
    for (name, grid, block), v in rows:
        out.append([name, grid, block, len(v), round(sum(v), 4), round(sum(v) / len(v), 4), round(min(v), 4),
                    round(max(v), 4), round(100 * sum(v) / total, 2)])
    if dst:
        with open(dst, "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out:
        print(",".join(str(x) for x in r))


if __name__ == "__main__":
    main()
