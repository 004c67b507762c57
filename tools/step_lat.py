"""Isolated tile-step latency (bench.py's probe: a 1024 x 9 x 9 grid, one tile per sweep in series) per
tile configuration, interleaved over two rounds:  python tools/step_lat.py [CFG ...]   (SDFGEN_TILE_CFG
values; default 2 3)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfgs = sys.argv[1:] or ["2", "3"]
code = ("import sys; sys.path.insert(0, %r); import bench; from sdfgenfast_amd import _lib; "
        "us = bench.step_latency(0); print('%%s %%.4f' %% (_lib.last_profile()['tile_cfg'], us))") % ROOT
for rnd in range(2):
    for c in cfgs:
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SDFGEN_TILE_CFG=c), capture_output=True,
                           text=True, timeout=300)
        print(f"SDFGEN_TILE_CFG={c}: " + (r.stdout.strip() if r.returncode == 0 else "FAILED " + r.stderr[-500:]),
              flush=True)
