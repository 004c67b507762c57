"""A/B by environment: python tools/ab_env.py WORKLOAD 'VAR=a' 'VAR=b' ... (each in a subprocess, interleaved;
several variables in one configuration joined by ',' or '+', the latter for tools/session.sh's comma lists)."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
wl, cfgs = sys.argv[1], sys.argv[2:]
code = r'''
import sys, json, os, hashlib; sys.path.insert(0, %r)
import numpy as np
from sdfgenfast_amd import _lib, meshgen
wl = %r
v, t, o, dx, dims = meshgen.workload(wl)
ref = json.load(open(os.path.join(sys.path[0], "tests", "golden", "hashes.json"))).get(wl, {}).get("sha256_phi")
best = None
for rep in range(6):
    phi = _lib.make_level_set3(v, t, o, dx, *dims, 1)
    if rep == 0 and ref:
        got = hashlib.sha256(np.asfortranarray(phi).ravel(order="F").astype("<f4").tobytes()).hexdigest()
        digest = "ok" if got == ref else "MISMATCH"
    p = _lib.last_profile()
    if rep and (best is None or p["total_ms"] < best["total_ms"]): best = p
print(json.dumps({k: best[k] for k in ("total_ms", "band_ms", "sweep_ms", "sparse_rechecks", "sparse_claims")} | {"sw": [round(x, 3) for x in best["sweep_launch_ms"]], "digest": digest if ref else "-"}))
''' % (ROOT, wl)
for rnd in range(2):
    for cfg in cfgs:
        env = dict(os.environ)
        for kv in cfg.replace("+", ",").split(","):
            if "=" in kv:
                k, v = kv.split("=", 1)
                env[k] = v
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(cfg, "FAILED", r.stderr[-800:]); sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        print(f"{cfg:28s} total {d['total_ms']:7.3f} band {d['band_ms']:6.3f} sweep {d['sweep_ms']:7.3f} | tile {sum(d['sw'][:8]):6.3f} sparse {sum(d['sw'][8:]):6.3f} rechecks {d['sparse_rechecks']} claims {d['sparse_claims']} digest {d['digest']}", flush=True)
