"""Idle gaps between consecutive kernels of the LAST call in a rocprofv3 kernel trace CSV.
python tools/kt_gaps.py path/to/kt_kernel_trace.csv"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
# the last call starts at its last k_prep_soup
i0 = max(i for i, k in enumerate(ks) if "k_prep_soup" in k[2])
last = ks[i0:]
short = lambda n: n.split("(")[0].split("<")[0].replace("void ", "").replace("sdfhip::", "").replace("(anonymous namespace)::", "")
busy = sum(e - s for s, e, _ in last)
span = last[-1][1] - last[0][0]
print(f"last call: {len(last)} kernels, span {span / 1e6:.3f} ms, kernel time {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms")
gaps = {}
for (s0, e0, n0), (s1, e1, n1) in zip(last, last[1:]):
    g = s1 - e0
    key = f"{short(n0)} -> {short(n1)}"
    gaps.setdefault(key, []).append(g)
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:40s} n={len(v):3d} gap avg {sum(v) / len(v) / 1e3:8.2f} us  sum {sum(v) / 1e3:8.1f} us")
for s, e, n in last:
    print(f"  {short(n):24s} start {(s - last[0][0]) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us")
