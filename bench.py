"""Benchmark: make_level_set3 on MI355X (BASELINE.json metric: Mvoxels/s at 256^3, 1M-tri mesh).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

One step = one complete make_level_set3 (prep, band + ray parity, 16 sweeps,
sign) on the deterministic 1M-triangle bumpy sphere with inputs already
resident in HBM and phi written to HBM (sdfgen_hip_make_level_set3_device).
For N > 1 (launched by torch.distributed.run, one rank per GPU) the same grid is
split into N Z-slabs (sdfgenfast_amd/distributed.py): each rank owns nk/N planes and the
sweeps' wavefront runs across the GPUs (strong scaling); see DESIGN.md §7.

Rank 0 prints one JSON line with the driver's contract fields plus
`roofline` (dominant kernel = the sweep, HIP-event timed inside the library
on the launch stream) and `cpu_baseline` (the oracle, 1 thread, on a bounded
sample; N=1 only).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mvoxels/sec at 256³ (1M-tri mesh); achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SWEEP_BYTES_PER_CELL = 16   # read phi+ct (8 B) + write phi+ct (8 B) per cell per sweep


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(workload: str):
    """Oracle (oracle/sdf_oracle.c, 1 thread) on a bounded sample: the same 1M-triangle
    mesh on a 128^3 grid (same mode-2b recipe) -- about 15 s of CPU work."""
    from oracle import oracle as O
    from sdfgenfast_amd import meshgen

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3_sphere1m_256")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    dist = None
    if world > 1:
        # Control plane (IPC-handle exchange, barriers, max of the wall time): gloo on the
        # host.  The data path is the slab wavefront itself: boundary planes move GPU to GPU
        # inside the sweep kernels (sdfgenfast_amd/distributed.py).
        # torch is imported BEFORE the backend so one HIP runtime serves both.
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")

    from sdfgenfast_amd import _hiprt, _lib, meshgen

    dev = local_rank % max(_lib.device_count(), 1)   # = local_rank on a node with a GPU per rank
    _hiprt.set_device(dev)
    v, t, o, dx, dims = meshgen.workload(args.workload)
    ni, nj, nk = dims
    ncell = ni * nj * nk
    dv = _hiprt.DeviceBuffer.from_array(v)
    dt = _hiprt.DeviceBuffer.from_array(t)
    if world > 1:
        from sdfgenfast_amd import distributed as D
        sess = D._gpu_session(dist, None, dev, dims, world, rank)
        nks = sess.k_end - sess.k_begin
        out = _hiprt.DeviceBuffer(ni * nj * nks * 4)

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

    for _ in range(args.warmup):
        step()
    _hiprt.synchronize()
    barrier()
    t0 = time.perf_counter()
    profs = [step() for _ in range(args.steps)]
    _hiprt.synchronize()
    el = time.perf_counter() - t0
    barrier()
    if dist is not None:
        x = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())

    ms_step = el / args.steps * 1e3
    value = ncell * args.steps / el / 1e6   # one whole grid per step (split over the ranks when N > 1)
    # Dominant kernel: the tile-wavefront sweep (k_sweep_tile), one launch per first-pass
    # sweep.  Its per-launch duration is the library's HIP-event time around that launch on
    # the launch stream; algorithmic bytes per launch = 16 B per swept cell.
    last = profs[-1]
    n_tile = last["sparse_first"] if last["sparse_sweeps"] else 16
    A, B, C = ni - 1, nj - 1, nk - 1
    tile_ms = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile)]
    launch_ms = sum(tile_ms) / max(len(tile_ms), 1)
    bytes_per_launch = SWEEP_BYTES_PER_CELL * A * B * C
    if world > 1:   # this rank's slab; the slab sessions run all 16 sweeps as tile wavefronts
        bytes_per_launch = SWEEP_BYTES_PER_CELL * A * B * (sess.k_end - sess.k_begin)
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    sparse_ms = [sum(p["sweep_launch_ms"][s] for p in profs) / len(profs) for s in range(n_tile, 16)]
    phases = {k: round(sum(p[k] for p in profs) / len(profs), 4)
              for k in ("prep_ms", "band_ms", "sweep_ms", "sign_ms", "total_ms")}
    phases["tile_sweeps_ms"] = round(sum(tile_ms), 4)
    phases["sparse_sweeps_ms"] = round(sum(sparse_ms), 4)
    traffic, traffic_src = None, None
    tp = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(tp):
        rec = json.load(open(tp))
        k = rec.get("kernels", {}).get("k_sweep_tile")
        if rec.get("workload") == args.workload and k:
            traffic, traffic_src = k["hbm_bytes_per_launch"], "profiles/pmc_summary.json"

    parity = None
    if not args.no_verify:
        hp = os.path.join(ROOT, "tests", "golden", "hashes.json")
        rec = json.load(open(hp)).get(args.workload) if os.path.exists(hp) else None
        got = out.download(np.float32, out.nbytes // 4)
        if world > 1:   # assemble the slabs on rank 0 (outside the timed region)
            parts = [None] * world if rank == 0 else None
            dist.gather_object(got, parts, dst=0)
            got = np.concatenate(parts) if rank == 0 else None
        if rank == 0 and rec:
            ok = hashlib.sha256(got.astype("<f4").tobytes()).hexdigest() == rec["sha256_phi"]
            parity = "bit-exact vs reference (sha256 of phi)" if ok else "MISMATCH vs reference sha256"

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mvoxels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 1M-triangle bumpy UV-sphere, sdfgenfast_amd/meshgen.py)",
            "config": {"workload": args.workload, "grid": list(dims), "triangles": int(t.shape[0]),
                       "exact_band": 1, "parallelism": f"zslab{world}" if world > 1 else "single-gpu",
                       "inputs": "HBM-resident"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": "k_sweep_tile",
                         "launches_per_step": n_tile, "avg_launch_ms": round(launch_ms, 5),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch)},
            "phases_ms": phases,
            "sweep_impl": profs[-1]["sweep_impl"],
            "parity": parity,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.workload)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
