"""Benchmark: make_level_set3 on MI355X (BASELINE.json metric: Mvoxels/s at 256^3, 1M-tri mesh).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--mode MODE]

One step = one complete make_level_set3 (prep, band + ray parity, 16 sweeps, sign) on the
deterministic 1M-triangle bumpy sphere with inputs already resident in HBM and phi written to
HBM (sdfgen_hip_make_level_set3_device, or the Z-slab sessions).

The headline `value`:
  N = 1  (`single`)  the C3 grid (256^3, the metric's configuration) on one GPU.
  N > 1  (`zslab`)   the SAME C3 grid split into N Z-slabs, one per GPU, the wavefront running
                     across the GPUs (north_star's decomposition) -- strong scaling; rank 0 first
                     times the single-GPU run so the line carries `efficiency` = T1 / (N * TN).
Side objects on the same line:
  zslab_c4   the C4 grid (512^3, north_star's Z-slab configuration) over the same N GPUs, with its
             own efficiency against rank 0's single-GPU C4 run (at N = 1: the single-GPU run).
  replicas   (N > 1) every rank computes the whole C3 grid on its own GPU at once: the node's
             throughput on a batch of independent jobs (weak scaling, no data-path exchange).
  host       (N = 1) host arrays in, host Array3f out through sdfgen_hip_make_level_set3 (the
             C++/Python drop-in's path; SURVEY 8.d's definition of t), PCIe included.
  roofline   the first-pass tile sweep (the dominant kernel): HBM bytes vs 8 TB/s, plus `latency`:
             the launch's modelled critical path (steps) x the isolated per-step time.
  ref_benchmark (N = 1) the reference's own published benchmark (test_x3y4z5_bin.stl on its 64/128/256
             proportional grids): device-resident and host-array times, phases, parity, the published times.
  cpu_baseline  (N = 1) the reference's own cpu_lib on this host's cores (oracle/_ref, built from
             /root/reference) or, when that build is absent, the repository's deterministic native
             CPU backend -- both on the FULL C3 workload; `kind` says which.
If the Z-slab run fails on N > 1 (reported in `zslab_error`), `value` falls back to the replicas
measurement and `config.parallelism` says so.
"""
import argparse
import hashlib
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mvoxels/sec at 256³ (1M-tri mesh); achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions/s: 256 CUs x 4 SIMDs, 2 cycles each
SWEEP_BYTES_PER_CELL = 16   # read phi+ct (8 B) + write phi+ct (8 B) per cell per sweep
PARITY_OK = "bit-exact vs reference (sha256 of phi)"
C3, C4 = "c3_sphere1m_256", "c4_sphere1m_512"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _host_threads() -> int:
    """Host cores this job may use: the box's CPU share (OMP_NUM_THREADS is set to it on the
    GPU boxes; os.cpu_count() there shows the whole machine), else the affinity set."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, min(len(os.sched_getaffinity(0)), 16))
    except AttributeError:
        return max(1, min(os.cpu_count() or 1, 16))


def cpu_baseline(workload: str):
    """The CPU path timed on this host's cores on the FULL workload (~5-10 s).
    kind "reference": the reference's own cpu_lib/makelevelset3.cpp (oracle/_ref/libsdfref.so,
    compiled from /root/reference by `make -C oracle ref`, travels with the tree; its k-split sweep
    races, SURVEY K1, so it is a timing baseline only).  kind "port": without that build, the
    repository's native CPU backend (sdfgen_cpu_make_level_set3, csrc/cpu_backend.cpp), a
    deterministic multi-threaded restatement of the same algorithm -- never a smaller sample."""
    from oracle import oracle as O
    from sdfgenfast_amd import _lib, meshgen

    v, t, o, dx, dims = meshgen.workload(workload)
    n = dims[0] * dims[1] * dims[2]
    th = _host_threads()
    if O.ref_available():
        t0 = time.perf_counter()
        O.ref_make_level_set3(v, t, o, dx, *dims, 1, num_threads=th)
        el = time.perf_counter() - t0
        return {"value": round(n / el / 1e6, 4), "unit": "Mvoxels/s", "cores": th, "kind": "reference",
                "sample": f"reference cpu_lib make_level_set3 (oracle/_ref, built from /root/reference), "
                          f"num_threads={th}, the full {workload} workload ({n} voxels, {t.shape[0]} triangles), "
                          f"{el:.2f} s; 1 thread on an MI355X box host (EPYC 9575F): 42.3 s, 0.397 Mvoxels/s "
                          f"(profiles/r03_ref_1thread_box.log; 89.3 s in the build container: tests/golden/hashes.json "
                          f"ref_seconds_1thread). Timing only: with "
                          f"{th} threads the reference's k-split sweep races (SURVEY K1), so its output is not "
                          f"parity-valid (the parity target is its 1-thread result)"}
    log("bench: oracle/_ref (the reference build) is absent -- timing the native CPU backend instead")
    t0 = time.perf_counter()
    _lib.cpu_make_level_set3(v, t, o, dx, *dims, 1, th, _lib.LAYOUT_ARRAY3)
    el = time.perf_counter() - t0
    return {"value": round(n / el / 1e6, 4), "unit": "Mvoxels/s", "cores": th, "kind": "port",
            "sample": f"native CPU backend sdfgen_cpu_make_level_set3 (deterministic restatement of cpu_lib), "
                      f"num_threads={th}, the full {workload} workload ({n} voxels), {el:.2f} s "
                      f"(oracle/_ref absent on this host)"}


def _golden(workload):
    hp = os.path.join(ROOT, "tests", "golden", "hashes.json")
    return json.load(open(hp)).get(workload) if os.path.exists(hp) else None


def _phases(profs):
    ph = {k: round(sum(p[k] for p in profs) / len(profs), 4)
          for k in ("prep_ms", "band_ms", "sweep_ms", "sign_ms", "total_ms")}
    last = profs[-1]
    n_tile = last["sparse_first"] if last["sparse_sweeps"] else 16
    tile = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile)]
    sparse = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile, 16)]
    ph["tile_sweeps_ms"] = round(sum(tile), 4)
    ph["sparse_sweeps_ms"] = round(sum(sparse), 4)
    multi = last.get("tile_multi", 0)   # the first pass as one overlapped launch of `multi` sweeps
    launches = 1 if multi > 1 else max(len(tile), 1)
    return ph, sum(tile) / launches, (multi if multi > 1 else 1), launches


def _time(step, steps, warmup, dist):
    """Warm up, then time exactly `steps` calls between barriers; max over ranks."""
    from sdfgenfast_amd import _hiprt

    for _ in range(warmup):
        step()
    _hiprt.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    profs = [step() for _ in range(steps)]
    _hiprt.synchronize()
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        import torch
        x = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
    return el, profs


def measure_single(workload, steps, warmup, dev, verify=True, dist=None):
    """One GPU, the whole grid.  With `dist`, every rank does this at once (replicas)."""
    from sdfgenfast_amd import _hiprt, _lib, meshgen

    v, t, o, dx, dims = meshgen.workload(workload)
    ni, nj, nk = dims
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    out = _hiprt.DeviceBuffer(ni * nj * nk * 4)

    def step():
        _lib.make_level_set3_device(dev, dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, ni, nj, nk, 1,
                                    _lib.LAYOUT_ARRAY3, out.ptr, 0)
        return _lib.last_profile()

    el, profs = _time(step, steps, warmup, dist)
    ph, launch_ms, spl, launches = _phases(profs)
    A, B, C = ni - 1, nj - 1, nk - 1
    r = {"workload": workload, "dims": dims, "triangles": int(t.shape[0]), "ms_per_step": el / steps * 1e3,
         "value": ni * nj * nk * steps / el / 1e6, "phases": ph, "launch_ms": launch_ms,
         "sweeps_per_launch": spl, "launches": launches, "sweep_impl": profs[-1]["sweep_impl"],
         "chain_steps": profs[-1]["chain_steps"], "tile_cfg": profs[-1]["tile_cfg"],
         "bytes_per_launch": SWEEP_BYTES_PER_CELL * A * B * C * spl, "parity": None}
    if verify:
        rec = _golden(workload)
        if rec:
            got = out.download(np.float32, ni * nj * nk)
            ok = hashlib.sha256(got.astype("<f4").tobytes()).hexdigest() == rec["sha256_phi"]
            if dist is not None:   # every replica must match
                oks = [None] * dist.get_world_size()
                dist.all_gather_object(oks, ok)
                ok = all(oks)
            r["parity"] = PARITY_OK if ok else "MISMATCH vs reference sha256"
    for b in (dv, dt, out):
        b.close()
    return r


def _slab_phases(p):
    """Where one slab's time went in its last timed call (device wall-clock phase timers,
    include/sdfgen_hip.h slab_*): the first pass's tile launch, the boundary tiles' waits on the
    upstream GPU, and per second-pass sweep the DONE / READY handshakes, the repair kernel and its
    inbound-ring draining."""
    r3 = lambda xs: [round(x, 4) for x in xs]
    it, ot = p["slab_inbox_tasks"], p["slab_other_tasks"]
    return {"first_pass_ms": round(p["sweep_launch_ms"][0], 4),
            "second_pass_ms": round(sum(p["sweep_launch_ms"][8:]), 4),
            "inbox_tasks": it, "inbox_idle_ms_per_task": round(p["slab_inbox_idle_ms"] / it, 4) if it else None,
            "other_tasks": ot, "other_idle_ms_per_task": round(p["slab_other_idle_ms"] / ot, 4) if ot else None,
            "wait_done_ms": r3(p["slab_wait_done_ms"]), "wait_ready_ms": r3(p["slab_wait_ready_ms"]),
            "repair_ms": r3(p["slab_repair_ms"]), "inbound_ms": r3(p["slab_inbound_ms"]),
            "inbound_entries": list(p["slab_inbound_entries"])}


def measure_zslab(workload, steps, warmup, dev, dist, world, rank, verify=True):
    """One grid split into `world` Z-slabs, one per rank/GPU (sdfgenfast_amd.distributed)."""
    from sdfgenfast_amd import _hiprt, _lib, meshgen
    from sdfgenfast_amd import distributed as D

    v, t, o, dx, dims = meshgen.workload(workload)
    ni, nj, nk = dims
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    sess = D._gpu_session(dist, None, dev, dims, world, rank)
    out = _hiprt.DeviceBuffer(ni * nj * (sess.k_end - sess.k_begin) * 4)
    sess.prepare(t.shape[0])
    dist.barrier()   # every slab's buffers and tables are in place before any slab's kernels wait on it

    def step():
        sess.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_ARRAY3, out.ptr)
        return sess.finish(v.shape[0])

    el, profs = _time(step, steps, warmup, dist)
    ph, launch_ms, spl, launches = _phases(profs)
    A, B = ni - 1, nj - 1
    r = {"workload": workload, "dims": dims, "triangles": int(t.shape[0]), "ms_per_step": el / steps * 1e3,
         "value": ni * nj * nk * steps / el / 1e6, "phases": ph, "launch_ms": launch_ms,
         "sweeps_per_launch": spl, "launches": launches, "sweep_impl": profs[-1]["sweep_impl"],
         "chain_steps": profs[-1]["chain_steps"],
         "bytes_per_launch": SWEEP_BYTES_PER_CELL * A * B * (sess.k_end - sess.k_begin) * spl, "parity": None}
    phases = [None] * world
    dist.all_gather_object(phases, dict(_slab_phases(profs[-1]), rank=rank, k_range=[sess.k_begin, sess.k_end]))
    r["slab_phases"] = phases
    if verify:
        rec = _golden(workload)
        got = out.download(np.float32, out.nbytes // 4)
        parts = [None] * world if rank == 0 else None
        dist.gather_object(got, parts, dst=0)   # outside the timed region
        if rank == 0 and rec:
            full = np.concatenate(parts)
            ok = hashlib.sha256(full.astype("<f4").tobytes()).hexdigest() == rec["sha256_phi"]
            r["parity"] = PARITY_OK if ok else "MISMATCH vs reference sha256"
    for b in (dv, dt, out):
        b.close()
    return r


def measure_host(workload, reps=3):
    """Host arrays in, host Array3f out (sdfgen_hip_make_level_set3, one GPU): steady state with
    a reused output array, and the first call into a fresh one (first-touch page faults)."""
    from sdfgenfast_amd import _lib, meshgen

    v, t, o, dx, dims = meshgen.workload(workload)
    n = dims[0] * dims[1] * dims[2]
    out = np.empty(n, np.float32)
    t0 = time.perf_counter()
    _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out)   # fresh pages
    first = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.make_level_set3(v, t, o, dx, *dims, 1, _lib.LAYOUT_ARRAY3, out=out)
    el = (time.perf_counter() - t0) / reps
    return {"value": round(n / el / 1e6, 3), "unit": "Mvoxels/s", "ms_per_call": round(el * 1e3, 3),
            "first_call_ms": round(first * 1e3, 3),
            "what": "sdfgen_hip_make_level_set3: host tri/xyz in, host Array3f (i-fastest) out, PCIe included; "
                    "value = steady state into a reused output array, first_call_ms = into a fresh one"}


# The reference's own published benchmark (tests/benchmark_performance.cpp:151, 181-185; README.md:256-260):
# test_x3y4z5_bin.stl (36 triangles) on proportional grids with padding 2, timed around one whole
# make_level_set3 call with host arrays (std::chrono).  RTX 4090 (its CUDA backend, a different far-field
# algorithm: SURVEY K2) and i9-13900K (cpu_lib, 1 / 20 threads) in ms.
REF_PUBLISHED = {"x3y4z5_prop64": {"label": "64^3", "rtx4090_gpu_ms": 111, "cpu_1thread_ms": 738, "cpu_20thread_ms": 93},
                 "x3y4z5_prop128": {"label": "128^3", "rtx4090_gpu_ms": 358, "cpu_1thread_ms": 5980, "cpu_20thread_ms": 748},
                 "x3y4z5_prop256": {"label": "256^3", "rtx4090_gpu_ms": 1290, "cpu_1thread_ms": 48600, "cpu_20thread_ms": 4180}}


def measure_ref_benchmark(dev, steps=5):
    """The reference's published workload on this GPU: per grid the device-resident rate (inputs and phi
    in HBM), the host-array call the reference times (PCIe included), the phase split and the parity
    against the reference's own digest (tests/golden/hashes.json)."""
    out = []
    for name, pub in REF_PUBLISHED.items():
        r = measure_single(name, steps, 1, dev, True)
        h = measure_host(name)
        out.append({"workload": name, "label": pub["label"], "dims": list(r["dims"]), "triangles": r["triangles"],
                    "value": round(r["value"], 3), "unit": "Mvoxels/s", "ms_per_step": round(r["ms_per_step"], 4),
                    "host_io_ms": h["ms_per_call"], "host_io_value": h["value"], "phases_ms": r["phases"],
                    "parity": r["parity"], "published_ms": {k: v for k, v in pub.items() if k != "label"},
                    "vs_rtx4090_host_io": round(pub["rtx4090_gpu_ms"] / h["ms_per_call"], 2)})
    return out


def step_latency(dev):
    """Isolated per-step time of the tile wavefront: a grid one tile wide (1024 x 9 x 9), so the
    first-pass launch is ONE tile per sweep in series -- no contention, pure step latency."""
    from sdfgenfast_amd import _hiprt, _lib, meshgen

    v, t = meshgen.bumpy_sphere(200, 61)
    dims = (1024, 9, 9)
    o, dx = meshgen.grid_mode2b(v, *dims, 2)
    dv, dt = _hiprt.DeviceBuffer.from_array(v), _hiprt.DeviceBuffer.from_array(t)
    out = _hiprt.DeviceBuffer(int(np.prod(dims)) * 4)
    best = None
    for _ in range(3):
        _lib.make_level_set3_device(dev, dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, *dims, 1,
                                    _lib.LAYOUT_ARRAY3, out.ptr, 0)
        p = _lib.last_profile()
        if p["tile_multi"] > 1 and p["chain_steps"] > 0:
            us = p["sweep_launch_ms"][0] * 1e3 / p["chain_steps"]
            best = us if best is None else min(best, us)
    for b in (dv, dt, out):
        b.close()
    return best


def _build_id():
    from sdfgenfast_amd import _lib
    return _lib.build_id()


def roofline(r, step_us, workload, whole_grid=True):
    """whole_grid=False (a Z-slab rank): the PMC summary holds the ONE-GPU launch over the whole
    grid, not this slab's launch, so no traffic is reported for it."""
    achieved = r["bytes_per_launch"] / (r["launch_ms"] * 1e-3) / 1e9 if r["launch_ms"] > 0 else 0.0
    traffic, traffic_src = None, None
    tp = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not whole_grid:
        traffic_src = "n/a: profiles/pmc_summary.json is the one-GPU whole-grid launch, not a slab's"
    elif os.path.exists(tp):
        rec = json.load(open(tp))
        k = rec.get("kernels", {}).get("k_sweep_tile")
        if rec.get("workload") == workload and k:
            if rec.get("build_id") == _build_id():
                traffic, traffic_src = k["hbm_bytes_per_launch"], f"profiles/pmc_summary.json (build {rec['build_id']})"
            else:   # counters of another build of the library: not this run's traffic
                traffic_src = f"stale: profiles/pmc_summary.json is of build {rec.get('build_id')}, not {_build_id()}"
    lat = None
    if step_us and r["chain_steps"] > 0 and r["launch_ms"] > 0:
        bound_ms = r["chain_steps"] * step_us * 1e-3
        lat = {"chain_steps": round(r["chain_steps"], 1), "step_us_isolated": round(step_us, 4),
               "bound_ms": round(bound_ms, 4), "launch_ms": round(r["launch_ms"], 4),
               "frac": round(bound_ms / r["launch_ms"], 4),
               "what": "modelled critical path of the launch (tile steps; tile_sweep_multi's schedule) x the "
                       "per-step time of an isolated tile (1024x9x9 grid): the launch time if only the "
                       "dependency chain bounded it"}
    # "bound" names the roofline the fraction is priced against (the contract's hbm | mfma); what
    # actually limits the launch is its dependency chain -- "limiter" and the "latency" object say so
    return {"bound": "hbm", "limiter": "latency (dependency chain)" if lat else None,
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": traffic_src, "kernel": "k_sweep_tile", "sweeps_per_launch": r["sweeps_per_launch"],
            "launches_per_step": r["launches"], "avg_launch_ms": round(r["launch_ms"], 5),
            "algorithmic_bytes_per_launch": int(r["bytes_per_launch"]), "latency": lat}


def valu(r, workload):
    """SURVEY 8.d caveat: the sweep's VALU issue rate (SQ_INSTS_VALU per launch, profiles/
    pmc_sq_summary.json from tools/pmc_sq.sh) against one wave64 VALU per 2 cycles per SIMD."""
    sp = os.path.join(ROOT, "profiles", "pmc_sq_summary.json")
    if not os.path.exists(sp) or r["launch_ms"] <= 0:
        return None
    rec = json.load(open(sp))
    k = next((v for n, v in rec.get("kernels", {}).items() if n.startswith("k_sweep_tile")), None)
    if rec.get("workload") != workload or not k or "SQ_INSTS_VALU" not in k:
        return None
    if rec.get("build_id") != _build_id():
        return {"kernel": "k_sweep_tile", "insts_per_launch": None, "frac": None,
                "source": f"stale: profiles/pmc_sq_summary.json is of build {rec.get('build_id')}, not {_build_id()}"}
    rate = k["SQ_INSTS_VALU"] / (r["launch_ms"] * 1e-3)
    return {"kernel": "k_sweep_tile", "insts_per_launch": int(k["SQ_INSTS_VALU"]), "achieved": round(rate / 1e9, 2),
            "peak": round(VALU_ISSUE_PEAK / 1e9, 1), "unit": "G wave-instructions/s",
            "frac": round(rate / VALU_ISSUE_PEAK, 4), "source": f"profiles/pmc_sq_summary.json (build {rec['build_id']})"}


def summary(r, world, mode, t1_ms=None):
    d = {"workload": r["workload"], "n_gpus": world, "parallelism": mode, "value": round(r["value"], 3),
         "unit": "Mvoxels/s", "ms_per_step": round(r["ms_per_step"], 3), "phases_ms": r["phases"],
         "parity": r["parity"]}
    if "tile_cfg" in r:
        d["tile_cfg"] = r["tile_cfg"]
    if t1_ms:
        d["single_gpu_ms"] = round(t1_ms, 3)
        d["efficiency"] = round(t1_ms / (world * r["ms_per_step"]), 4)
    if r.get("slab_phases"):
        d["slab_phases"] = r["slab_phases"]
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=C3)
    ap.add_argument("--mode", choices=["auto", "single", "replicas", "zslab"], default="auto")
    ap.add_argument("--c4-workload", default=C4, help="the Z-slab side measurement's grid")
    ap.add_argument("--no-side", action="store_true", help="headline only (no zslab_c4 / replicas / host)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the isolated-tile step timing (profiling runs: its launches would mix into the counters)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    mode = args.mode
    if mode == "auto":
        mode = "single" if world == 1 else "zslab"
    if (mode == "single") != (world == 1):
        raise SystemExit(f"--mode {mode} needs {'1 rank' if mode == 'single' else 'several ranks'}, got {world}")
    verify = not args.no_verify

    dist = None
    if world > 1:
        # Control plane (barriers, max of the wall time, IPC-handle exchange): gloo on the host.
        # No collective sits on the data path.  torch is imported BEFORE the
        # backend so one HIP runtime serves both.
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")

    from sdfgenfast_amd import _hiprt, _lib  # noqa: F401

    ndev = max(_lib.device_count(), 1)
    dev = local_rank % ndev   # = local_rank on a node with a GPU per rank
    shared = world > ndev     # a rehearsal with several slabs per GPU (one-GPU box)
    if shared and "SDFGEN_SLABS_PER_DEVICE" not in os.environ:
        # Co-resident slabs of several processes: the library caps each slab's persistent grids (first
        # pass and repair) from the occupancy query and the slab count per device; it counts its own
        # process's sessions, so ranks sharing a GPU tell it how many share (sdfgen_hip.hip slab_share)
        os.environ["SDFGEN_SLABS_PER_DEVICE"] = str((world + ndev - 1) // ndev)
    _hiprt.set_device(dev)
    topo = None
    if world > 1:
        # which GPU each rank drives (device, PCI bus id) and the node's peer-access matrix, so that a
        # mapping failure or watchdog on a multi-GPU node can be tied to the rank pair (the library's
        # slab errors name slab, device and PCI id of both sides)
        # (an A/B library built before ABI 4 has no sdfgen_hip_topology: the line records null then)
        t = _lib.topology() if hasattr(_lib.lib, "sdfgen_hip_topology") else None
        me = {"rank": rank, "local_rank": local_rank, "device": dev, "host": socket.gethostname(),
              "pci_bus_id": t["pci_bus_ids"][dev] if t and dev < len(t["pci_bus_ids"]) else None}
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        topo = None if t is None else {"ranks": ranks, "devices": t["devices"], "pci_bus_ids": t["pci_bus_ids"],
                                       "peer_access": t["peer_access"]}
    step_us = step_latency(dev) if rank == 0 and not args.no_latency else None

    res_side = {}
    zs_err = None
    if world == 1:
        r = measure_single(args.workload, args.steps, args.warmup, dev, verify)
        parallelism, scaling = "single-gpu", "weak"
        if not args.no_side:
            c4 = measure_single(args.c4_workload, 2, 1, dev, verify)
            res_side["zslab_c4"] = summary(c4, 1, "single-gpu", c4["ms_per_step"])
            res_side["host"] = measure_host(args.workload)
            res_side["ref_benchmark"] = measure_ref_benchmark(dev)
    else:
        # single-GPU reference times for the efficiencies: rank 0 alone, the others wait
        t1 = [None, None]
        if rank == 0 and mode == "zslab":
            t1[0] = measure_single(args.workload, 2, 1, dev, False)["ms_per_step"]
            if not args.no_side:
                t1[1] = measure_single(args.c4_workload, 2, 1, dev, False)["ms_per_step"]
        box = [t1]
        dist.broadcast_object_list(box, src=0)
        t1 = box[0]
        r = None
        if mode == "zslab":
            try:
                r = measure_zslab(args.workload, args.steps, args.warmup, dev, dist, world, rank, verify)
            except Exception as e:   # reported; the headline falls back to the replicas run below
                zs_err = f"{type(e).__name__}: {e}"[:400]
                log(f"bench rank {rank}: Z-slab run failed: {zs_err}")
            errs = [None] * world
            dist.all_gather_object(errs, zs_err)
            zs_err = next((x for x in errs if x), None)
            if zs_err:
                r = None
        rep = None
        if mode == "replicas" or r is None or not args.no_side:
            rep = measure_single(args.workload, args.steps if r is None else 2, args.warmup if r is None else 1,
                                 dev, verify, dist)
            rep["value"] *= world   # N grids per step, whole job
        if r is None:
            r, parallelism, scaling = rep, f"replicas{world}", "weak"
        else:
            parallelism, scaling = f"zslab{world}", "strong"
            if rep is not None:
                res_side["replicas"] = summary(rep, world, f"replicas{world}")
            if t1[0]:
                res_side["efficiency"] = round(t1[0] / (world * r["ms_per_step"]), 4)
                res_side["single_gpu_ms"] = round(t1[0], 3)
            if not args.no_side:
                try:
                    c4 = measure_zslab(args.c4_workload, 2, 1, dev, dist, world, rank, verify)
                    res_side["zslab_c4"] = summary(c4, world, f"zslab{world}", t1[1])
                except Exception as e:
                    res_side["zslab_c4"] = {"workload": args.c4_workload, "n_gpus": world,
                                            "error": f"{type(e).__name__}: {e}"[:400]}

    if rank == 0:
        ni, nj, nk = r["dims"]
        res = {
            "metric": METRIC,
            "value": round(r["value"], 3),
            "unit": "Mvoxels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 1M-triangle bumpy UV-sphere, sdfgenfast_amd/meshgen.py)",
            "config": {"workload": args.workload, "grid": [ni, nj, nk], "triangles": r["triangles"],
                       "exact_band": 1, "parallelism": parallelism, "inputs": "HBM-resident",
                       "ranks_per_gpu": (world + ndev - 1) // ndev},
            "roofline": roofline(r, step_us, args.workload, whole_grid=(world == 1 or parallelism.startswith("replica"))),
            "valu": valu(r, args.workload) if world == 1 else None,
            "phases_ms": r["phases"],
            "sweep_impl": r["sweep_impl"],
            "tile_cfg": r.get("tile_cfg"),
            "parity": r["parity"],
            "build_id": _build_id(),
        }
        if topo:
            res["topology"] = topo
        if r.get("slab_phases"):
            res["slab_phases"] = r["slab_phases"]   # per rank: where each slab's time went
        res.update(res_side)
        if "host" in res_side:
            # SURVEY 8.d's definition of t: one call with host arrays in and a host Array3f out
            # (PCIe included), next to the HBM-resident `value`
            res["value_host_io"] = res_side["host"]["value"]
            res["ms_per_call_host_io"] = res_side["host"]["ms_per_call"]
        if zs_err:
            res["zslab_error"] = zs_err
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.workload)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
