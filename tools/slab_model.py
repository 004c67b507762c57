"""Per-phase model of the Z-slab run over N GPUs: predicts the C3 / C4 times and the
1 -> N strong-scaling efficiency from measured single-GPU quantities, before an 8-GPU node exists.

    python tools/slab_model.py            (the measured inputs are in INPUTS, with their sources)

Phases of one call on N slabs (every slab runs them at once; the call takes the slowest slab):
  local    prep + band + sign: no exchange, work divides by N           t_local(1) / N
  first    the one-launch first pass (sweeps 1-8): the larger of
             chain   chain_steps(N) * s_iso + 8 * (N - 1) * h_x   -- the wavefront's critical path
                     (tile steps of the task graph over ALL slabs, chain_model below) times the
                     isolated tile step, plus one cross-GPU hop per slab boundary per sweep
             work    T_first_work / N                              -- the tiles' throughput
           times a crowding factor: at one GPU the measured first pass lies above both bounds
           (C3: the loaded step is 1.7x the isolated one -- tiles on the critical path share CUs with
           the others); crowd(1) = measured / max(chain, work), and a slab of 1/N of the tiles crowds
           its GPU 1/N as much: crowd(N) = 1 + (crowd(1) - 1) / N
  second   sweeps 9-16, each: Jacobi scan + list (work, / N) + the repair chains (a few dozen
           dependent relabels; they do not shorten with N) + the neighbour handshakes
           (DONE/READY flags: 2 * h_flag per sweep) + one cross-slab hand-off per boundary a
           chain crosses (inbound ring: (N - 1) * h_x at most)
Inputs are measured on one MI355X (bench line, rocprof, tools/uc_lat): see INPUTS.  h_x, the cross-GPU
granule latency over xGMI, cannot be measured on a one-GPU box: 2 us is assumed (the on-chip
uncached system-scope round trip is 0.82 us, tools/uc_lat).
"""
import json

# ---- measured inputs (one MI355X, round 6 final build 6c8f290b) ----
INPUTS = {
    "c3_sphere1m_256": {   # bench r06z: 13.45 ms in phases; tile launch 10.25 ms (rocprof avg); 8 sparse sweeps 2.53 ms
        "dims": (256, 256, 256), "t_local": 0.7238, "t_first": 10.2500, "t_second": 2.5334,
        "t_repair_per_sweep": 0.2113,  # k_sp_recheck per sweep at C3 (profiles/r06z_c3_kernel_stats.csv, 8 x 6 calls)
        "t_first_work": 5.0,           # tile work at full throughput: C4's first pass x 1/8 of the cells
        "longest_chain": 86,           # longest relabel chain of a second-pass sweep (oracle)
    },
    "c4_sphere1m_512": {   # round 6 (bench r06z zslab_c4: 51.56 ms in phases; tile 38.44 ms rocprof avg,
        # profiles/r06z_c4_kernel_stats.csv; sparse 10.30 ms)
        "dims": (512, 512, 512), "t_local": 1.883, "t_first": 38.44, "t_second": 10.297,
        "t_repair_per_sweep": 0.62,    # repair_ms per sweep, 2-slab rehearsal (r03c_n2 zslab_c4), median
        "t_first_work": 38.44,         # throughput-bound at one GPU: the launch itself
        "longest_chain": 172,          # not measured at C4: 2 x C3's (chains scale with the grid edge)
        # round 5, one MI355X (profiles/r05d_sparse_from_c4.log, SDFGEN_SPARSE_FROM=k, per-sweep events): the
        # first pass's last sweeps as Jacobi + repair instead of inside the tile launch -- the tile launch of the
        # first k sweeps and each later first-pass sweep's own time
        "sparse_from": {8: {"tile": 42.003, "sparse_first": []},
                        7: {"tile": 36.051, "sparse_first": [35.897]},
                        6: {"tile": 32.296, "sparse_first": [30.297, 37.807]}},
    },
}
S_ISO_US = 1.056     # isolated tile step, quad-lane tiles (round 6 bench latency probe, 1024x9x9 grid: profiles/r06z_c3_bench.json.log)
H_X_US = 2.0         # cross-GPU granule hand-off over xGMI (assumed; on-chip uncached round trip 0.82 us)
H_FLAG_US = 2.0      # one DONE / READY flag hand-off between neighbour GPUs (assumed, as h_x)
LINK_IDLE_US = 1.25  # one repair chain link on an idle chip: ~4 returning atomics + 2 dependent loads, ~3,000 cycles
                     # (round 3, tools/xcd_lat); under the 1-GPU repair's own load it is ~4.7 us
ST_T = 8
DIRS = [(+1, +1, +1), (-1, -1, -1), (+1, +1, -1), (-1, -1, +1), (+1, -1, +1), (-1, +1, -1), (+1, -1, -1), (-1, +1, +1)]


def _c_range(kb, ke, nk, dk):
    if dk > 0:
        return max(kb, 1) - 1, ke - 1
    return nk - 1 - min(ke, nk - 1), nk - 1 - kb


def _tile_phys(T, c0, c1, n, d):
    xl, xh = c0 + ST_T * T, min(c0 + ST_T * T + ST_T, c1) - 1
    return (xl + 1, xh + 1) if d > 0 else (n - 2 - xh, n - 2 - xl)


def _covering(lo, hi, c0, c1, n, d):
    xl, xh = (lo - 1, hi - 1) if d > 0 else (n - 2 - hi, n - 2 - lo)
    xl, xh = max(xl, c0), min(xh, c1 - 1)
    if xl > xh:
        return None
    return (xl - c0) // ST_T, (xh - c0) // ST_T


def chain_model(ni, nj, nk, nslabs, nsw=8):
    """tile_sweep_multi's schedule model (sweep_tile.hpp) for all slabs: the critical path of the
    first-pass launch in tile steps.  Estimated starts: +1 hop per upstream tile of the same sweep
    (across slab boundaries too), + one tile duration after each previous-sweep tile it waits for.
    nsw < 8: the launch holds the first nsw sweeps only (the others run as Jacobi + repair)."""
    A, B = ni - 1, nj - 1
    nJ = (B + ST_T - 1) // ST_T
    kb = [r * nk // nslabs for r in range(nslabs + 1)]
    wc = (A + 2.0 * (ST_T - 1)) / ST_T
    cs, ce, nK = {}, {}, {}
    for q in range(nsw):
        for r in range(nslabs):
            cs[q, r], ce[q, r] = _c_range(kb[r], kb[r + 1], nk, DIRS[q][2])
            nK[q, r] = max(0, (ce[q, r] - cs[q, r] + ST_T - 1) // ST_T)
    kv = {}
    for q in range(nsw):
        d, dp = DIRS[q], DIRS[(q + 7) % 8]
        for rr in range(nslabs):
            r = rr if d[2] > 0 else nslabs - 1 - rr
            ru = r - 1 if d[2] > 0 else r + 1
            for J in range(nJ):
                for K in range(nK[q, r]):
                    v = 0.0
                    if J:
                        v = max(v, kv[q, r, J - 1, K] + 1.0)
                    if K:
                        v = max(v, kv[q, r, J, K - 1] + 1.0)
                    elif 0 <= ru < nslabs and nK[q, ru] > 0:
                        v = max(v, kv[q, ru, J, nK[q, ru] - 1] + 1.0)
                    if q:
                        jl, jh = _tile_phys(J, 0, B, nj, d[1])
                        kl, kh = _tile_phys(K, cs[q, r], ce[q, r], nk, d[2])
                        cj = _covering(jl - 1, jh + 1, 0, B, nj, dp[1])
                        ck = _covering(kl - 1, kh + 1, cs[q - 1, r], ce[q - 1, r], nk, dp[2])
                        if cj and ck:
                            for J2 in range(cj[0], cj[1] + 1):
                                for K2 in range(ck[0], ck[1] + 1):
                                    v = max(v, kv[q - 1, r, J2, K2] + wc)
                    kv[q, r, J, K] = v
    return (max(kv.values()) + wc) * ST_T


def gs_levels(ni, nj, nk, nsw=8):
    """The exact critical path of the reference's first pass at CELL granularity, in levels: node (sweep s,
    cell p) depends on (s, its upwind neighbours) and on (s - 1, p) (cpu_lib/makelevelset3.cpp:243-291,
    130-151).  The diagonal neighbours never lengthen it, so L_s(p) = 1 + max(L_{s-1}(p), L_s(p - e_x) for the
    three axes x), i.e. a running maximum with +1 per cell along each axis in the sweep's direction.  No
    schedule and no GPU count can run the first pass in fewer dependent steps at parity."""
    import numpy as np
    A, B, C = ni - 1, nj - 1, nk - 1   # oriented cells per axis (the boundary planes are fixed)
    L = np.zeros((A, B, C), np.int32)
    idx = [np.arange(n, dtype=np.int32).reshape(sh) for n, sh in
           ((A, (A, 1, 1)), (B, (1, B, 1)), (C, (1, 1, C)))]
    for q in range(nsw):
        d = DIRS[q % 8]
        L += 1
        for ax in range(3):
            v = L if d[ax] > 0 else np.flip(L, axis=ax)
            v -= idx[ax]
            np.maximum.accumulate(v, axis=ax, out=v)
            v += idx[ax]
    return int(L.max())


def ceiling(name, inp, steps_us=(1.056, 0.75, 0.49, 0.38), n=8):
    """the N-GPU efficiency this design could reach with a shorter isolated step.  First
    pass = max(levels x s, work / N) (crowding as in predict); second pass with the measured repair (does
    not shrink with N) and with every repair link at its idle-chip latency (the best case)."""
    ni, nj, nk = inp["dims"]
    lv = gs_levels(ni, nj, nk)
    base = predict(name, inp, (1,))["rows"][0]["total_ms"]
    c1 = chain_model(ni, nj, nk, 1) * S_ISO_US * 1e-3
    crowd = inp["t_first"] / max(c1, inp["t_first_work"])
    t_scan = inp["t_second"] / 8 - inp["t_repair_per_sweep"]
    hand = (2 * H_FLAG_US + (n - 1) * H_X_US) * 1e-3
    rows = []
    for s in steps_us:
        first = max(lv * s * 1e-3 + 8 * (n - 1) * H_X_US * 1e-3, inp["t_first_work"] / n) * (1.0 + (crowd - 1.0) / n)
        sec_hi = 8 * (t_scan / n + inp["t_repair_per_sweep"] + hand)
        sec_lo = 8 * (t_scan / n + min(inp["t_repair_per_sweep"], inp["longest_chain"] * LINK_IDLE_US * 1e-3) + hand)
        local = inp["t_local"] / n
        rows.append({"step_us": s, "gs_levels": lv, "first_ms": round(first, 3), "second_ms": round(sec_hi, 3),
                     "second_ms_links_idle": round(sec_lo, 3),
                     "efficiency": round(base / (n * (local + first + sec_hi)), 3),
                     "efficiency_links_idle": round(base / (n * (local + first + sec_lo)), 3)})
    return rows


def predict(name, inp, ns=(1, 2, 4, 8)):
    ni, nj, nk = inp["dims"]
    c1 = chain_model(ni, nj, nk, 1)
    chain1 = c1 * S_ISO_US * 1e-3
    crowd = inp["t_first"] / max(chain1, inp["t_first_work"])   # >= 1: sharing CUs with other tiles
    t_scan = inp["t_second"] / 8 - inp["t_repair_per_sweep"]     # Jacobi scan + list + launch gaps per sweep
    rows = []
    for n in ns:
        cn = chain_model(ni, nj, nk, n) if n > 1 else c1
        chain = cn * S_ISO_US * 1e-3 + 8 * (n - 1) * H_X_US * 1e-3
        work = inp["t_first_work"] / n
        first = max(chain, work) * (1.0 + (crowd - 1.0) / n)
        # repair term: measured at one GPU (upper: it does not shrink with N) and the longest chain at the
        # idle-chip link latency (lower: a slab of 1/N of the cells runs 1/N of the concurrent chains)
        rep_hi = inp["t_repair_per_sweep"]
        rep_lo = min(rep_hi, inp["longest_chain"] * LINK_IDLE_US * 1e-3) if n > 1 else rep_hi
        hand = (2 * H_FLAG_US + (n - 1) * H_X_US) * 1e-3 * (n > 1)
        second = 8 * (t_scan / n + rep_hi + hand)
        second_lo = 8 * (t_scan / n + rep_lo + hand)
        local = inp["t_local"] / n
        total = local + first + second
        rows.append({"n": n, "chain_steps": round(cn, 1), "first_chain_ms": round(chain, 3),
                     "first_work_ms": round(work, 3), "first_ms": round(first, 3), "second_ms": round(second, 3),
                     "second_ms_if_links_idle": round(second_lo, 3), "local_ms": round(local, 3),
                     "total_ms": round(total, 3), "total_ms_if_links_idle": round(local + first + second_lo, 3)})
    t1 = rows[0]["total_ms"]
    for r in rows:
        r["efficiency"] = round(t1 / (r["n"] * r["total_ms"]), 3)
        r["efficiency_if_links_idle"] = round(t1 / (r["n"] * r["total_ms_if_links_idle"]), 3)
    return {"workload": name, "crowd_factor_1gpu": round(crowd, 3), "inputs": inp, "s_iso_us": S_ISO_US,
            "h_x_us": H_X_US, "rows": rows}


def predict_schedules(name, inp, ns=(1, 2, 4, 8)):
    """an N-dependent split of the first pass -- its first k sweeps in the tile launch,
    sweeps k..7 as Jacobi + repair -- priced per N.  The tile part scales like the default's first pass
    (chain of the k-sweep task graph, work / N, crowding); a repair sweep is priced OPTIMISTICALLY at its
    one-GPU time / N plus the neighbour handshakes (its chains do not really shrink with N),
    so a split that loses here loses on hardware too.  Only the first-pass time changes; returns rows of
    (N, k, first-pass ms, total ms, efficiency vs the default 1-GPU run)."""
    sf = inp.get("sparse_from")
    if not sf:
        return []
    ni, nj, nk = inp["dims"]
    base = predict(name, inp, ns)["rows"]
    t1 = base[0]["total_ms"]
    rows = []
    for n, b in zip(ns, base):
        for k in sorted(sf, reverse=True):
            d = sf[k]
            c1 = chain_model(ni, nj, nk, 1, k)
            chain1 = c1 * S_ISO_US * 1e-3
            work1 = d["tile"] if inp["t_first_work"] == inp["t_first"] else inp["t_first_work"] * k / 8
            crowd = d["tile"] / max(chain1, work1)
            cn = chain_model(ni, nj, nk, n, k) if n > 1 else c1
            chain = cn * S_ISO_US * 1e-3 + k * (n - 1) * H_X_US * 1e-3
            tile = max(chain, work1 / n) * (1.0 + (crowd - 1.0) / n)
            rep = sum(t / n + (2 * H_FLAG_US + (n - 1) * H_X_US) * 1e-3 * (n > 1) for t in d["sparse_first"])
            first = tile + rep
            total = b["total_ms"] - b["first_ms"] + first
            rows.append({"n": n, "tile_sweeps": k, "first_ms": round(first, 3), "tile_ms": round(tile, 3),
                         "repair_sweeps_ms": round(rep, 3), "total_ms": round(total, 3),
                         "efficiency": round(t1 / (n * total), 3)})
    return rows


def main():
    for name, inp in INPUTS.items():
        res = predict(name, inp)
        print(json.dumps({k: v for k, v in res.items() if k != "rows"}))
        for r in res["rows"]:
            print("  ", json.dumps(r))
        for r in predict_schedules(name, inp):
            print("   schedule", json.dumps(r))
        for r in ceiling(name, inp):
            print("   ceiling n=8", json.dumps(r))


if __name__ == "__main__":
    main()
