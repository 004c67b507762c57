"""Calibrate FETCH_SIZE / WRITE_SIZE on gfx950 for 8-byte, agent-scope and per-line accesses
(tools/fetch_calib.hip; MI355X_MICROARCH.md "HBM": only 16-B coalesced reads / stores are calibrated).
Runs two rocprofv3 --pmc passes over the probe, takes each kernel's second launch, and prints the
counter's bytes over the kernel's known bytes.   python tools/fetch_calib.py [OUT.json]"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "fetch_calib")
GIB, LINES = 1 << 30, (1 << 30) // 128
# kernel -> (what, requested bytes, 128-B lines touched)
KNOWN = {"k_read16": ("16-B coalesced plain loads", GIB, LINES),
         "k_read8": ("8-B coalesced plain loads", GIB, LINES),
         "k_read8_agent": ("8-B coalesced agent-scope atomic loads (sc1)", GIB, LINES),
         "k_read8_agent_line": ("one 8-B agent-scope load per 128-B line", 8 * LINES, LINES),
         "k_gather16_line": ("one 16-B plain load per 128-B line, scattered", 16 * LINES, LINES),
         "k_write8": ("8-B coalesced plain stores", GIB, LINES),
         "k_write8_agent": ("8-B coalesced agent-scope atomic stores", GIB, LINES),
         "k_write8_agent_line": ("one 8-B agent-scope store per 128-B line", 8 * LINES, LINES),
         # 16 passes over 1 MiB (8,192 lines): FETCH/line ~64 B = one fetch per line, ~16 x 64 B = every pass
         "k_reread8_agent": ("16 passes of 8-B agent-scope loads over 1 MiB", 16 << 20, 8192),
         "k_reread8": ("16 passes of 8-B plain loads over 1 MiB", 16 << 20, 8192)}


def run(counter):
    d = os.path.join(ROOT, "gpurun_out", f"calib_{counter}")
    subprocess.run(["rm", "-rf", d], check=True)
    subprocess.run(["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--", EXE],
                   check=True, timeout=120)
    per = defaultdict(float)
    order = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = next((k for k in KNOWN if row["Kernel_Name"].startswith(k + "(") or row["Kernel_Name"] == k), None)
            if k:
                did = int(row["Dispatch_Id"])
                per[(k, did)] += float(row["Counter_Value"]) * 1024.0   # KiB
    last = {}
    for (k, did), v in per.items():
        if k not in last or did > last[k][0]:
            last[k] = (did, v)
    return {k: v for k, (_, v) in last.items()}


fetch, write = run("FETCH_SIZE"), run("WRITE_SIZE")
out = {}
for k, (what, req, lines) in KNOWN.items():
    out[k] = {"what": what, "requested_bytes": req, "lines_128B": lines, "fetch_bytes_raw": fetch.get(k),
              "write_bytes_raw": write.get(k),
              "fetch_per_requested": round(fetch[k] / req, 4) if fetch.get(k) is not None else None,
              "fetch_per_line": round(fetch[k] / lines, 2) if fetch.get(k) is not None else None,
              "write_per_requested": round(write[k] / req, 4) if write.get(k) is not None else None,
              "write_per_line": round(write[k] / lines, 2) if write.get(k) is not None else None}
    print(f"{k:22s} {what:48s} FETCH/req {out[k]['fetch_per_requested']}  FETCH/line {out[k]['fetch_per_line']} B  "
          f"WRITE/req {out[k]['write_per_requested']}  WRITE/line {out[k]['write_per_line']} B", flush=True)
if len(sys.argv) > 1:
    json.dump({"probe": "tools/fetch_calib.hip", "buffer_bytes": GIB, "kernels": out}, open(sys.argv[1], "w"), indent=1)
