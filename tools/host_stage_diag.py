"""Host entry point with each SDFGEN_HOST_STAGE setting (staged copy-out on/off), one subprocess each: time, digest, or the error.
python tools/hostmap_diag.py WORKLOAD [settings...]"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
wl = sys.argv[1]
code = r'''
import sys, json, os, hashlib, time; sys.path.insert(0, %r)
import numpy as np
from sdfgenfast_amd import _lib, meshgen
wl = %r
v, t, o, dx, dims = meshgen.workload(wl)
ref = json.load(open(os.path.join(sys.path[0], "tests", "golden", "hashes.json"))).get(wl, {}).get("sha256_phi")
out = np.empty(dims[0] * dims[1] * dims[2], np.float32)
ts = []
for rep in range(4):
    t0 = time.perf_counter()
    try:
        phi = _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out)
    except Exception as e:
        print("ERROR", type(e).__name__, e); sys.exit(0)
    ts.append(time.perf_counter() - t0)
    if rep == 0:
        got = hashlib.sha256(np.asfortranarray(phi).ravel(order="F").astype("<f4").tobytes()).hexdigest()
print("first %%.2f ms, then %%s ms, device %%.2f ms, digest %%s" %% (ts[0] * 1e3, [round(x * 1e3, 2) for x in ts[1:]],
      _lib.last_profile()["total_ms"], "ok" if got == ref else ("MISMATCH" if ref else "-")))
''' % (ROOT, wl)
for s in sys.argv[2:] or ["0", "1", "2", "3"]:
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SDFGEN_HOST_STAGE=s), capture_output=True,
                       text=True, timeout=300)
    print(f"SDFGEN_HOST_STAGE={s}: rc {r.returncode} {r.stdout.strip()[-400:]} {r.stderr.strip()[-300:] if r.returncode else ''}",
          flush=True)
