"""Benchmark: make_level_set3 on MI355X (BASELINE.json metric: Mvoxels/s at 256^3, 1M-tri mesh).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--mode MODE]

One step = one complete make_level_set3 (prep, band + ray parity, 16 sweeps,
sign) on the deterministic 1M-triangle bumpy sphere with inputs already
resident in HBM and phi written to HBM (sdfgen_hip_make_level_set3_device).

Modes:
  single    N = 1: the whole grid on one GPU.
  replicas  N > 1 default, weak scaling: every rank computes the whole workload on
            its own GPU (a batch of N SDF jobs, one per GPU; no data-path exchange).
            value = N grids / the slowest rank's time.
  zslab     strong scaling of ONE grid: rank r owns nk/N k-planes and the sweeps'
            wavefront runs across the GPUs (boundary planes move GPU to GPU inside
            the running kernels, sdfgenfast_amd/distributed.py).
Unless --no-zslab, the line also carries `zslab`: the C4 grid (512^3, the
north_star's Z-slab configuration) split over the same N GPUs.  For N > 1 it runs
as a child torch.distributed job BEFORE this process touches the GPU, so a
failure there cannot take the main measurement with it; for N = 1 it is the
single-GPU C4 run, the reference point of the Z-slab efficiency.

Rank 0 prints one JSON line with the driver's contract fields plus `roofline`
(dominant kernel = the tile-wavefront sweep, HIP-event timed inside the library
on the launch stream) and `cpu_baseline` (N=1 only: the reference's own CPU path,
multi-threaded on this host, on the full workload; the oracle on a sample when the
reference build is absent).
"""
import argparse
import hashlib
import json
import os
import signal
import socket
import subprocess
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
    """The reference's own CPU path (cpu_lib/makelevelset3.cpp compiled from /root/reference into
    oracle/_ref/ by `make -C oracle ref`; the built .so travels with the tree) with its
    multi-threaded sweep on this host's cores, on the FULL workload -- about 10 s.  Its k-split
    sweep races, so this is a timing baseline only.  Without oracle/_ref: the C
    restatement (oracle/sdf_oracle.c, 1 thread) on a bounded sample (same mesh at 128^3)."""
    from oracle import oracle as O
    from sdfgenfast_amd import meshgen

    if O.ref_available():
        v, t, o, dx, dims = meshgen.workload(workload)
        th = _host_threads()
        t0 = time.perf_counter()
        O.ref_make_level_set3(v, t, o, dx, *dims, 1, num_threads=th)
        el = time.perf_counter() - t0
        n = dims[0] * dims[1] * dims[2]
        return {"value": round(n / el / 1e6, 4), "unit": "Mvoxels/s", "cores": th, "kind": "reference",
                "sample": f"reference cpu_lib make_level_set3 (oracle/_ref), num_threads={th}, the full "
                          f"{workload} workload ({n} voxels, {t.shape[0]} triangles), {el:.2f} s; 1 thread: "
                          f"see tests/golden/hashes.json ref_seconds_1thread"}
    w = meshgen.WORKLOADS[workload]
    v, t = meshgen.bumpy_sphere(w["nu"], w["nv"])
    n = 128
    o, dx = meshgen.grid_mode2b(v, n, n, n, w["padding"])
    t0 = time.perf_counter()
    O.make_level_set3(v, t, o, dx, n, n, n, 1)
    el = time.perf_counter() - t0
    return {"value": round(n ** 3 / el / 1e6, 4), "unit": "Mvoxels/s", "cores": 1, "kind": "port",
            "sample": f"oracle/sdf_oracle.c single-thread, same {t.shape[0]}-triangle mesh on a {n}^3 grid "
                      f"({n ** 3} voxels), {el:.2f} s"}


def _golden(workload):
    hp = os.path.join(ROOT, "tests", "golden", "hashes.json")
    return json.load(open(hp)).get(workload) if os.path.exists(hp) else None


def measure(workload, mode, steps, warmup, dev, dist, world, rank, verify=True):
    """Time `steps` calls after `warmup` untimed ones.  Returns a dict (every rank)."""
    from sdfgenfast_amd import _hiprt, _lib, meshgen

    v, t, o, dx, dims = meshgen.workload(workload)
    ni, nj, nk = dims
    ncell = ni * nj * nk
    dv = _hiprt.DeviceBuffer.from_array(v)
    dt = _hiprt.DeviceBuffer.from_array(t)
    sess = None
    if mode == "zslab":
        from sdfgenfast_amd import distributed as D
        sess = D._gpu_session(dist, None, dev, dims, world, rank)
        out = _hiprt.DeviceBuffer(ni * nj * (sess.k_end - sess.k_begin) * 4)

        def step():
            sess.enqueue(dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx, 1, _lib.LAYOUT_ARRAY3, out.ptr)
            return sess.finish(v.shape[0])
    else:
        out = _hiprt.DeviceBuffer(ncell * 4)

        def step():
            _lib.make_level_set3_device(dev, dt.ptr, t.shape[0], dv.ptr, v.shape[0], o, dx,
                                        ni, nj, nk, 1, _lib.LAYOUT_ARRAY3, out.ptr, 0)
            return _lib.last_profile()

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(warmup):
        step()
    _hiprt.synchronize()
    barrier()
    t0 = time.perf_counter()
    profs = [step() for _ in range(steps)]
    _hiprt.synchronize()
    el = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        x = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())

    grids = world if mode == "replicas" else 1   # whole grids computed per step by the job
    r = {"workload": workload, "dims": dims, "triangles": int(t.shape[0]), "el": el,
         "ms_per_step": el / steps * 1e3, "value": grids * ncell * steps / el / 1e6}
    # Dominant kernel: the tile-wavefront sweep (k_sweep_tile), one launch per first-pass
    # sweep.  Its per-launch duration is the library's HIP-event time around that launch on
    # the launch stream; algorithmic bytes per launch = 16 B per swept cell.
    last = profs[-1]
    n_tile = last["sparse_first"] if last["sparse_sweeps"] else 16
    A, B, C = ni - 1, nj - 1, nk - 1
    tile_ms = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile)]
    multi = last.get("tile_multi", 0)   # the first pass as one overlapped launch of `multi` sweeps
    launches = 1 if multi > 1 else max(len(tile_ms), 1)
    launch_ms = sum(tile_ms) / launches
    sweeps_per_launch = multi if multi > 1 else 1
    bytes_per_launch = SWEEP_BYTES_PER_CELL * A * B * C * sweeps_per_launch
    if sess is not None:   # this rank's slab; the slab sessions run all 16 sweeps as tile wavefronts
        bytes_per_launch = SWEEP_BYTES_PER_CELL * A * B * (sess.k_end - sess.k_begin)
    sparse_ms = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile, 16)]
    phases = {k: round(sum(p[k] for p in profs) / len(profs), 4)
              for k in ("prep_ms", "band_ms", "sweep_ms", "sign_ms", "total_ms")}
    phases["tile_sweeps_ms"] = round(sum(tile_ms), 4)
    phases["sparse_sweeps_ms"] = round(sum(sparse_ms), 4)
    r.update(n_tile=launches, launch_ms=launch_ms, bytes_per_launch=bytes_per_launch, phases=phases,
             sweep_impl=last["sweep_impl"], sweeps_per_launch=sweeps_per_launch)

    r["parity"] = None
    if verify:
        rec = _golden(workload)
        got = out.download(np.float32, out.nbytes // 4)
        if mode == "zslab":   # assemble the slabs on rank 0 (outside the timed region)
            parts = [None] * world if rank == 0 else None
            dist.gather_object(got, parts, dst=0)
            got = np.concatenate(parts) if rank == 0 else None
        ok = None
        if rec and got is not None:
            ok = hashlib.sha256(got.astype("<f4").tobytes()).hexdigest() == rec["sha256_phi"]
        if mode == "replicas":   # every replica must match
            oks = [None] * world
            dist.all_gather_object(oks, ok)
            ok = None if any(x is None for x in oks) else all(oks)
        if ok is not None:
            r["parity"] = PARITY_OK if ok else "MISMATCH vs reference sha256"
    for b in (dv, dt, out):
        b.close()
    return r


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def zslab_child(world, workload, timeout=600):
    """Z-slab strong scaling of `workload` over `world` GPUs, as a child torch.distributed
    job (run before this process touches a GPU).  Returns the summary dict or an error."""
    env = {k: v for k, v in os.environ.items()
           if not (k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                         "ROLE_NAME", "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
                   or k.startswith("TORCHELASTIC_") or k.startswith("TORCH_ELASTIC"))}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--mode", "zslab", "--workload", workload, "--steps", "2", "--warmup", "1",
           "--no-zslab", "--no-cpu-baseline"]
    t0 = time.time()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        # the launcher and its ranks share the new session's process group: end all of them,
        # so no orphaned rank keeps a GPU busy under the measurement that follows
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.communicate()
        return {"workload": workload, "n_gpus": world, "error": f"timed out after {timeout} s"}
    lines = [x for x in out.splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        tail = (err or "").strip().splitlines()[-3:]
        return {"workload": workload, "n_gpus": world, "error": f"rc={p.returncode}: {' | '.join(tail)[-400:]}"}
    res = json.loads(lines[-1])
    return {"workload": workload, "n_gpus": world, "parallelism": res["config"]["parallelism"],
            "value": res["value"], "unit": "Mvoxels/s", "ms_per_step": res["ms_per_step"],
            "phases_ms": res["phases_ms"], "parity": res["parity"], "wall_s": round(time.time() - t0, 1)}


def zslab_summary(r, world):
    return {"workload": r["workload"], "n_gpus": world,
            "parallelism": f"zslab{world}" if world > 1 else "single-gpu", "value": round(r["value"], 3),
            "unit": "Mvoxels/s", "ms_per_step": round(r["ms_per_step"], 3), "phases_ms": r["phases"],
            "parity": r["parity"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3_sphere1m_256")
    ap.add_argument("--mode", choices=["auto", "single", "replicas", "zslab"], default="auto")
    ap.add_argument("--zslab-workload", default="c4_sphere1m_512")
    ap.add_argument("--no-zslab", action="store_true", help="skip the Z-slab side measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    mode = args.mode
    if mode == "auto":
        mode = "single" if world == 1 else "replicas"
    if (mode == "single") != (world == 1):
        raise SystemExit(f"--mode {mode} needs {'1 rank' if mode == 'single' else 'several ranks'}, got {world}")

    dist = None
    if world > 1:
        # Control plane (barriers, max of the wall time, IPC-handle exchange for zslab): gloo
        # on the host.  No collective sits on the data path.
        # torch is imported BEFORE the backend so one HIP runtime serves both.
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")

    zs = None
    if not args.no_zslab and mode == "replicas":
        if rank == 0:
            zs = zslab_child(world, args.zslab_workload)
        dist.barrier()

    from sdfgenfast_amd import _hiprt, _lib

    dev = local_rank % max(_lib.device_count(), 1)   # = local_rank on a node with a GPU per rank
    _hiprt.set_device(dev)
    r = measure(args.workload, mode, args.steps, args.warmup, dev, dist, world, rank, not args.no_verify)
    if not args.no_zslab and mode == "single":
        zs = zslab_summary(measure(args.zslab_workload, "single", 2, 1, dev, None, 1, 0, not args.no_verify), 1)

    if rank == 0:
        ni, nj, nk = r["dims"]
        achieved = r["bytes_per_launch"] / (r["launch_ms"] * 1e-3) / 1e9 if r["launch_ms"] > 0 else 0.0
        tp = os.path.join(ROOT, "profiles", "pmc_summary.json")
        traffic, traffic_src = None, None
        if os.path.exists(tp) and mode != "zslab":
            rec = json.load(open(tp))
            k = rec.get("kernels", {}).get("k_sweep_tile")
            if rec.get("workload") == args.workload and k:
                traffic, traffic_src = k["hbm_bytes_per_launch"], "profiles/pmc_summary.json"
        # SURVEY 8.d caveat: the sweep is latency/VALU-bound, so also report its VALU issue rate
        # (SQ_INSTS_VALU per launch from profiles/pmc_sq_summary.json, tools/pmc_sq.sh) against
        # the chip's: one wave64 VALU instruction per 2 cycles per SIMD (MI355X_MICROARCH.md)
        valu = None
        sp = os.path.join(ROOT, "profiles", "pmc_sq_summary.json")
        if os.path.exists(sp) and mode != "zslab" and r["launch_ms"] > 0:
            rec = json.load(open(sp))
            k = next((v for n, v in rec.get("kernels", {}).items() if n.startswith("k_sweep_tile")), None)
            if rec.get("workload") == args.workload and k and "SQ_INSTS_VALU" in k:
                peak = VALU_ISSUE_PEAK
                rate = k["SQ_INSTS_VALU"] / (r["launch_ms"] * 1e-3)
                valu = {"kernel": "k_sweep_tile", "insts_per_launch": int(k["SQ_INSTS_VALU"]),
                        "achieved": round(rate / 1e9, 2), "peak": round(peak / 1e9, 1),
                        "unit": "G wave-instructions/s", "frac": round(rate / peak, 4),
                        "source": "profiles/pmc_sq_summary.json"}
        res = {
            "metric": METRIC,
            "value": round(r["value"], 3),
            "unit": "Mvoxels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": "strong" if mode == "zslab" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 1M-triangle bumpy UV-sphere, sdfgenfast_amd/meshgen.py)",
            "config": {"workload": args.workload, "grid": [ni, nj, nk], "triangles": r["triangles"],
                       "exact_band": 1,
                       "parallelism": {"single": "single-gpu", "replicas": f"replicas{world}",
                                       "zslab": f"zslab{world}"}[mode],
                       "inputs": "HBM-resident"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": "k_sweep_tile",
                         "sweeps_per_launch": r["sweeps_per_launch"],
                         "launches_per_step": r["n_tile"], "avg_launch_ms": round(r["launch_ms"], 5),
                         "algorithmic_bytes_per_launch": int(r["bytes_per_launch"])},
            "valu": valu,
            "phases_ms": r["phases"],
            "sweep_impl": r["sweep_impl"],
            "parity": r["parity"],
        }
        if zs is not None:
            res["zslab"] = zs
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.workload)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
