// sweep_tile.hpp -- one Gauss-Seidel sweep direction as ONE persistent launch:
// a pipelined column wavefront over 8x8 (j,k) tiles.
//
// Why this is exact.  The reference sweep (cpu_lib/makelevelset3.cpp:130-151)
// visits k, then j, then i and updates each cell from its 7 upwind neighbours
// (:143-149).  In oriented coordinates (a,b,c) (a = i-1 for di>0, ni-2-i for di<0,
// likewise b, c) every upwind neighbour has a strictly smaller a+b+c and each cell
// is written once per sweep, so any order that finishes a cell's upwind
// neighbours first reproduces the sequential result bit-for-bit.
//
// Decomposition.  The (b,c) plane is cut into 8x8 tiles; a tile is one task for one
// workgroup of ST_NCW compute waves and one helper wave:
//   * compute waves: wave w owns the c-columns [w*CLW, (w+1)*CLW) of the tile; lane
//     (bl,cl) owns column (b0+bl, c0+cl) and at local step h updates cell
//     a = h-bl-cl.  A wave advances one anti-diagonal per step with no barrier:
//     wave w starts step h once wave w-1 has finished step h-1 and while wave w+1 is
//     at most RR-4 steps behind (LDS progress counters).  Neighbour results (label
//     AND the triangle's vertices) live in an LDS ring, so no global load sits on
//     the critical path.  The ~2 distinct candidates per cell (7 upwind labels minus
//     duplicates and the cell's own label -- exact skips, see sweep_cell in
//     sdfgen_hip.hip) are evaluated by four lanes per cell in one pass (quad tiles) or
//     compacted across the wave (ballot + mbcnt) and evaluated one or two per lane
//     (1-wave tiles), then applied in the reference's check order (strict '<', first
//     minimum wins).
//   * helper wave: batched, decoupled prefetch.  It streams each column's old
//     (phi, label) and the label's vertices into an LDS "own" ring, and fills the
//     17 halo streams (last row of tile J-1, last column of tile K-1, corner) from
//     8-byte tagged granules {epoch, label} that producer tiles publish with one
//     sc1 store each (the data is the flag: cdna_hip_programming.md G16 R2) plus a
//     gather of the triangle's vertices from the read-only soup.  Readiness and
//     ring capacity are LDS counters (capacity follows the SLOWEST compute wave);
//     the helper waits on global memory, the compute waves never do.
// Tasks are dequeued in anti-diagonal order (J+K, then J) from an atomic counter,
// so every producer tile is claimed by a running workgroup before its consumers:
// no residency assumption and no deadlock.  Every spin is bounded (watchdog).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "geom.hpp"

namespace sdfhip {

// Tunables (compile-time; -D overrides are for experiments).  Defaults were chosen on
// MI355X at 256^3: 3-wave workgroups with ~47 KB LDS let 3 tiles share
// a CU, and that beat 5-wave / 79 KB tiles (1 per CU) by 12-15 %.
#ifndef ST_NCW_DEF
#define ST_NCW_DEF 2   // compute waves per tile
#endif
#ifndef ST_RR_DEF
#define ST_RR_DEF 8    // neighbour ring slots (power of two); lead between compute waves = RR-4
#endif
#ifndef ST_RO_DEF
#define ST_RO_DEF 4    // own-column prefetch slots (power of two)
#endif
#ifndef ST_RH_DEF
#define ST_RH_DEF 8    // halo ring slots per stream (power of two)
#endif
#ifndef ST_G_DEF
#define ST_G_DEF 2     // helper batch: steps / halo entries per global round trip (2 or 4)
#endif
#ifndef ST_CWA
#define ST_CWA 1       // helper: own cells' words loaded up to ST_RC steps ahead into LDS (their gathers then wait for a
                       // free own slot only: one round trip from slot to landing instead of two)
#endif
#ifndef ST_RC_DEF
#define ST_RC_DEF 8    // ST_CWA: own cell-word slots (power of two)
#endif
#ifndef ST_HALO_FIRST
#define ST_HALO_FIRST 1   // helper: the halo batch's gathers issued, landed and published before the own batch's
#endif
#ifndef ST_HELPER_PRIO
#define ST_HELPER_PRIO 0   // the helper wave's issue priority (the compute waves step at ST_WORK_PRIO)
#endif
#ifndef ST_COMPUTE_WAIT0
#define ST_COMPUTE_WAIT0 1
#endif
#ifndef ST_WORK_PRIO
#define ST_WORK_PRIO 2   // compute waves' issue priority while stepping (0 while they wait)
#endif
#ifndef ST_TWIN
#define ST_TWIN 1      // twin lanes split each cell's candidates (needs 32-cell compute waves)
#endif
#ifndef ST_HSLEEP
#define ST_HSLEEP 16   // longest back-off (s_sleep units of 64 cycles) of an idle helper wave
#endif
#ifndef ST_CSLEEP
#define ST_CSLEEP 8    // longest back-off of a waiting compute wave
#endif
#ifndef ST_QMIN
#define ST_QMIN 1      // quad tiles: a first-minimum reduction over the quad instead of four ordered applies
#endif
#ifndef ST_GVMASK
#define ST_GVMASK 1    // 1-wave and twin-lane tiles: the same integer VALU form of the candidate mask: C4 first pass
                       // (1-wave tiles, throughput-bound) 40.10-40.15 -> 39.04-39.13 ms (profiles/r05ac_*); with the apply
                       // reading non-candidates as +inf 38.77-38.80 ms (r05ad_*)
#endif
#ifndef ST_QVMASK
#define ST_QVMASK 1    // quad tiles: the mask's tests in integer VALU arithmetic (no compare masks to combine):
                       // isolated step 1.141 -> 1.088 us, C3 / C4 first pass neutral (profiles/r05z_*)
#endif
#ifndef ST_QMASK
#define ST_QMASK 1     // quad tiles: the candidate mask split over the cell's four lanes
#endif
#ifndef ST_WPE_DEF
#define ST_WPE_DEF 3   // waves per SIMD the register budget must allow
#endif
constexpr int ST_T = 8;                       // tile edge (b and c)
constexpr int ST_NCOL = ST_T * ST_T;          // 64 columns
constexpr int ST_NSTREAM = 2 * ST_T + 1;      // halo streams: b-edge (8), c-edge (8), corner
constexpr int ST_RO = ST_RO_DEF;
constexpr int ST_RH = ST_RH_DEF;
constexpr int ST_G = ST_G_DEF;
constexpr int ST_RC = ST_RC_DEF;
typedef int i4v __attribute__((ext_vector_type(4)));
static_assert((ST_RO & (ST_RO - 1)) == 0 && ST_RO >= ST_G, "own slots: power of two >= batch");
static_assert((ST_RH & (ST_RH - 1)) == 0 && ST_RH >= 2 * ST_G, "halo slots: power of two");
static_assert((ST_RC & (ST_RC - 1)) == 0 && ST_RC >= 2 * ST_G, "own cell-word slots: power of two >= 2 batches");

// Tile kernel configuration: compute waves per tile, neighbour ring slots, twin lanes, the waves
// per SIMD the register budget must allow, and lanes per cell (4: quad lanes, 2: duo lanes).
template <int NCW_, int RR_, bool TWIN_, int WPE_, int LPC_ = 1, bool FIX_ = false, int NH_ = 1>
struct StCfg {
    static constexpr int NH = NH_;                      // helper waves: 1 (own data and halo), 2 (one each)
    static constexpr bool FIX = FIX_;                   // quad lanes with fixed slots (q = r, r + 4) in one packed pass
    static constexpr int NCW = NCW_;                    // compute waves per tile
    static constexpr int CLW = ST_T / NCW;              // c-columns per compute wave
    static constexpr int CPW = ST_T * CLW;              // cells per compute wave
    static constexpr int RR = RR_;                      // neighbour ring slots
    static constexpr bool TWIN = TWIN_;                 // lane L + 32 is the twin of cell lane L
    static constexpr int LPC = LPC_;                    // lanes per cell: lanes LPC x .. LPC x + LPC - 1 are cell x
    static constexpr bool QUAD = LPC_ > 1;              // the lanes-per-cell step (quad or duo lanes): no compaction
    static constexpr int LPC_SH = LPC_ == 8 ? 3 : (LPC_ == 4 ? 2 : (LPC_ == 2 ? 1 : 0));
    static constexpr int WPE = WPE_;
    static constexpr int LEAD = NCW > 1 ? RR - 4 : 0;   // max lead of wave w over wave w+1 (ring hazard)
    static constexpr int THREADS = 64 * (NCW + NH);     // compute waves + helper wave(s)
    static_assert(NH == 1 || NH == 2, "one helper wave, or an own-data and a halo helper");
    static constexpr int RING0 = 0;                                 // RR slots x 64 columns
    static constexpr int HALO0 = RING0 + RR * ST_NCOL;              // 17 streams x RH
    static constexpr int OWN0 = HALO0 + ST_NSTREAM * ST_RH;         // RO slots x 64 columns
    static constexpr int ENTS = OWN0 + ST_RO * ST_NCOL;
    static_assert(NCW >= 1 && (NCW <= 4 || LPC_ == 8) && ST_T % NCW == 0, "compute waves must split the tile's c-columns");
    static_assert(NCW <= 3 || QUAD, "four compute waves: the quad-lane step only");
    static_assert(!TWIN || CPW == 32, "twin lanes: a compute wave owns 32 cells (lane L + 32 is L's twin)");
    static_assert(LPC == 1 || LPC == 2 || LPC == 4 || LPC == 8, "lanes per cell: 1, 2, 4 or 8");
    static_assert(!QUAD || (CPW * LPC == 64 && !TWIN), "lanes per cell: a compute wave owns 64 / LPC cells");
    // Ring slots: a column's entry for a is last read 3 steps after it is written (as the a - 1
    // neighbour of the diagonal column), so one compute wave needs 4; several need 4 more for the
    // lead between them (RR = 4 with 2 waves measured wrong results: no lead left).
    // One compute wave reads a step's neighbours before it writes the step back, so 3 slots are enough
    // there (the entry written at step h is read last at step h + 3, before that step's write-back into
    // the same slot); 3 is not a power of two: slots by a modulo (RR_POW2 below).
    static_assert(((RR & (RR - 1)) == 0 && (RR >= 8 || (NCW == 1 && RR == 4))) || (NCW == 1 && RR == 3 && LPC == 1),
                  "ring slots: power of two, >= 8 (4 or 3 with one compute wave)");
    static constexpr bool RR_POW2 = (RR & (RR - 1)) == 0;
};
// Round 3's latency-bound tiles (SDFGEN_TILE_CFG=0 only since round 4): 2 compute waves of 32 cells
// with twin lanes; ~47 KB LDS, 3 tiles per CU.  Throughput-bound grids (C4, C5): ONE
// compute wave of 64 cells, no ring lead -- half the instructions per cell; ~35 KB LDS, 4 tiles per
// CU (first pass 512^3: 50.2 -> 44.5 ms, 1024^3: 342 -> 272 ms; 256^3: 13.75 -> 14.6 ms).
using StCfgLat = StCfg<ST_NCW_DEF, ST_RR_DEF, (ST_TWIN != 0), ST_WPE_DEF>;
#ifndef ST_THR_WPE
#define ST_THR_WPE 2
#endif
#ifndef ST_THR_RR
#define ST_THR_RR 4
#endif
using StCfgThr = StCfg<1, ST_THR_RR, false, ST_THR_WPE>;
// Latency-bound grids, quad lanes: 4 compute waves of 16 cells, four lanes per cell -- every step
// evaluates up to 4 candidates per cell in ONE pass (lane 4x + r takes the cell's r-th candidate in
// check order) and a first-minimum reduction over the quad combines them, so no step pays the
// wave-wide compaction; ~43.5 KB LDS, 3 tiles per CU (5 waves each: 128 VGPRs).
#ifndef ST_QUAD_WPE
#define ST_QUAD_WPE 4
#endif
#ifndef ST_QUAD_NH
#define ST_QUAD_NH 1   // 2: the helper split into an own-data wave and a halo wave (6 waves per tile, 2 tiles per CU)
#endif
using StCfgQuad = StCfg<4, 8, false, ST_QUAD_WPE, 4, false, ST_QUAD_NH>;
// Duo lanes (round 5): 2 compute waves of 32 cells, two lanes per cell -- lane 2x + r evaluates the
// cell's candidates of rank r, r + 2, ... in passes of one ptd_wave each (a second pass only when a cell
// of the wave has more than 2 candidates), a first-minimum reduction over the pair (one DPP move).  Half
// the compute waves of the quad tiles per step, so two tiles' compute waves share a SIMD's issue slots
// less; ~43 KB LDS, 3 tiles per CU (3 waves each: 168 VGPRs).
#ifndef ST_DUO_WPE
#define ST_DUO_WPE 3
#endif
using StCfgDuo = StCfg<2, 8, false, ST_DUO_WPE, 2>;
// Oct lanes (round 5): 8 compute waves of 8 cells (one c-column each), EIGHT lanes per cell with FIXED
// roles -- lane 0 reads the cell's own entry, lane 1 + q the entry of upwind neighbour q -- so a step is
// one batch of LDS reads (no candidate ranking, no select trees: every address is known before any label
// is), one point-triangle distance per lane, and a first-minimum reduction over the 8 lanes (three DPP
// moves); the winning lane, which holds the winner's vertices, writes the ring entry back.  Same
// instructions per cell as the quad tiles, a shorter dependent chain per step.  9 waves per tile.
#ifndef ST_OCT_WPE
#define ST_OCT_WPE 4
#endif
using StCfgOct = StCfg<8, 8, false, ST_OCT_WPE, 8>;
// Fixed quad lanes (round 5): the quad tiles' geometry (4 compute waves x 16 cells, 4 lanes per cell)
// with the oct tiles' fixed roles -- lane r of a cell holds upwind neighbour q = r and q = r + 4 (lane 3:
// q = 3 and the cell's own entry), read in ONE batch of LDS reads, both evaluated in one packed-FP32
// pass (ptd_wave2); first minima over the quad for q = 0..3 and q = 4..6, the earlier group kept on
// ties; the lane holding the winner writes back.  No candidate ranking, no select trees, no duplicate
// test (a duplicate label evaluates to the same distance and loses the tie to the earlier slot).
#ifndef ST_QFP_WPE
#define ST_QFP_WPE 4
#endif
using StCfgQfp = StCfg<4, 8, false, ST_QFP_WPE, 4, true>;

enum { ST_CFG_LAT = 0, ST_CFG_THR = 1, ST_CFG_QUAD = 2, ST_CFG_DUO = 3, ST_CFG_OCT = 4, ST_CFG_QFP = 5 };
// The configuration of a launch with `tiles` tasks per sweep: the quad-lane one while the step
// latency is what counts, the throughput one once a sweep offers far more tiles than the chip holds
// at once (768: 3 per CU).  Round 4, first pass, before the quad step's instruction-count work:
// 128^3 (256 tiles) 4.78 ms quad vs 5.52 twin lanes; 256^3 (1,024) 12.23-12.30 quad vs 13.73-13.89
// twin; 320^3 (1,600) 19.12-19.17 quad vs 18.39-18.45 throughput; 384^3 (2,304) 29.1-29.3 vs
// 23.6-23.9; 512^3 (4,096) 61.1 vs 40.6.  After it (select trees etc.): 320^3 16.24
// quad vs 17.96 throughput, 384^3 24.6-24.7 vs 23.0 -- the crossover moved to between 1,600 and
// 2,304 tiles.  SDFGEN_TILE_CFG=0/1/2 forces one (tests, A/B; 0 = the twin-lane tiles of round 3).
constexpr long long ST_QUAD_MAX_TILES = 2000;
inline int st_cfg(long long tiles)
{
    if (const char *e = getenv("SDFGEN_TILE_CFG")) return std::max(0, std::min(5, atoi(e)));
    return tiles > ST_QUAD_MAX_TILES ? ST_CFG_THR : ST_CFG_QUAD;
}
inline bool st_use_thr(long long tiles) { return st_cfg(tiles) == ST_CFG_THR; }

constexpr unsigned ST_WATCHDOG = 1u << 24;    // empty polls before giving up (~seconds)
constexpr int ST_NSTATS = 24;                 // statistics words (StParams::stats): counts, step and helper profiles

// Entry layout in LDS: [3e] = (x1, w), [3e+1] = (x2, phi -- own entries only), [3e+2] = x3,
// where w is the cell's low word (label and the sweep that set it: geom.hpp lo_word).

// The lane id, recomputed where it is used (two VALU): a volatile asm is neither hoisted nor merged with another
// copy, so a lane constant derived from it (an LDS entry base) is not held across the helper loop -- held, the
// 128-VGPR quad kernel spilled it, and the landing's scratch reload (the youngest vector-memory op) turned the
// wait for the gathers into a wait for every load in flight, the stage-1 polls included (ST_LANE_REMAT)
#ifndef ST_LANE_REMAT
#define ST_LANE_REMAT 1
#endif
__device__ __forceinline__ int st_lane_remat()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// granule = {epoch (32 bits), low word (32 bits)}: the data is the flag
__device__ __forceinline__ unsigned long long st_granule(unsigned epoch, uint32_t w)
{
    return ((unsigned long long)epoch << 32) | w;
}
__device__ __forceinline__ bool st_granule_ready(unsigned long long g, unsigned epoch) { return (uint32_t)(g >> 32) == epoch; }

// Per-sweep fields of one launch that runs several sweeps (MULTI, see k_sweep_tile).
#ifndef ST_MAXSW_DEF
#define ST_MAXSW_DEF 8
#endif
constexpr int ST_MAXSW = ST_MAXSW_DEF;   // sweeps one multi-sweep launch can hold (a power of two)
static_assert((ST_MAXSW & (ST_MAXSW - 1)) == 0, "sweep slots: a power of two");
constexpr int ST_MAXDEP = 16;   // previous-sweep tiles a tile depends on (3x3 with margins)
struct StSweep {
    unsigned long long *hb, *hc;  // this sweep's halo granule buffers
    int di, dj, dk, sweep;
    unsigned epoch;
    int seen[7];
    int cs, ce, nK;               // oriented c range of this launch's slab for this sweep, its tile rows
    const unsigned long long *hc_in;   // Z-slab inbox of this sweep (null: no upstream slab)
    unsigned long long *hc_out;        // downstream slab's inbox of this sweep (null: none)
};

struct StParams {
    const float4 *soup;           // 3 float4 per triangle (xyz; w unused)
    unsigned long long *cell;     // (phi bits << 32) | closest_tri, i-fastest
    unsigned long long *hb;       // granules of tile-row edges:  [nJ][ce - cs][A] (c - cs)
    unsigned long long *hc;       // granules of tile-column edges: [nK][B][A]
    const int2 *tasks;            // (J,K) in dequeue order
    int *queue;                   // task counter (zeroed before each launch)
    int *err;                     // watchdog bits: 2 compute wave, 16 helper wave, 8 dependency wait, 4 inbox
    unsigned long long *stats;    // optional [evaluations, compute polls, helper idle polls, compute polls on own data]
    unsigned long long *trace;    // optional [task][start, end] wall_clock64 (100 MHz) of the compute wave
    float ox, oy, oz, dx;
    int ni, nj, nk;
    int A, B, C, nJ, nK, ntasks;
    int di, dj, dk;
    unsigned epoch;
    int sweep;
    int lead;                     // max steps wave w may run ahead of wave w+1 (<= Cfg::LEAD)
    // Z-slab mode (one GPU per slab of the grid).  Tiles cover oriented c in
    // [cs, ce); the plane c = cs-1 of an upstream slab arrives in hc_in, and this slab's plane
    // c = ce-1 is published to the downstream slab's inbox hc_out.  An inbox holds one granule
    // per cell (a, b) of the plane, a and b in [-1, A) x [-1, B): index (b+1)*(A+1) + a+1.
    int cs, ce;
    int hbC;                      // c extent of hb rows (= ce - cs)
    const unsigned long long *hc_in;
    unsigned long long *hc_out;
    unsigned long long clo, chi;  // cells [clo, chi) this launch may address (bounds-checked builds)
    unsigned long long ntri;      // triangles in the soup (bounds-checked builds)
    int seen[7];   // per upwind slot q: s'+1 of the last earlier sweep in which an interior cell
                   // examined that neighbour (-1: none) -- see sweep_sparse.hpp
    // MULTI: tasks of ST_MAXSW consecutive sweeps in one launch (cross-sweep overlap)
    const int4 *mtasks;           // (J, K, sweep slot, -) in dequeue order
    const int *deps;              // [task][ST_MAXDEP]: earlier tasks (previous sweep) to wait for, -1 = none
    unsigned *done;               // [task] = call_epoch once the task's cell stores are visible
    unsigned call_epoch;
    StSweep sw[ST_MAXSW];
    unsigned long long *tm;       // Z-slab phase timers (sweep_sparse.hpp TM_*; null: not recorded)
};

__device__ __forceinline__ size_t st_inbox(const StParams &P, int a, int b)
{
    return (size_t)(b + 1) * (size_t)(P.A + 1) + (size_t)(a + 1);
}

// A watchdog that fired anywhere on this device (P.err != 0): waiting workgroups give up at
// once instead of each running into its own watchdog (a lost hand-off fails in seconds).
#ifndef ST_FASTFAIL
#define ST_FASTFAIL 1
#endif

// Diagnostic builds for the per-buffer traffic split of DESIGN.md §5 (tools/pmc_split.sh): each
// takes one buffer's accesses off the fabric; the results are wrong, the launch's flow is not.
//   1: no cell stores   2: own-label vertex gathers read the tile's dummy triangle
//   3: halo vertex gathers likewise   4: own-cell reads hit the tile's dummy line (and so do 2)
#ifndef ST_DIAG_SPLIT
#define ST_DIAG_SPLIT 0
#endif
__device__ __forceinline__ bool st_failed(const StParams &P)
{
    return ST_FASTFAIL && __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// Record a fired watchdog and close the task queue: later claims all fall past the end.
__device__ __forceinline__ void st_fail(const StParams &P, int bit)
{
    atomicOr(P.err, bit);
    atomicMax(P.err + 1, P.sweep + 1);
    atomicCAS(P.err + 2, 0, (P.sweep + 1) | (bit << 8));   // the first failure: sweep + 1, its bit
    atomicMax(P.queue, P.ntasks);
}

// v[k] of four values by a select tree on k's bits (k in 0..3)
// (__builtin_unpredictable: without it the last level became an exec-mask branch)
__device__ __forceinline__ int st_sel4(int k, int v0, int v1, int v2, int v3)
{
    const bool k0 = k & 1, k1 = k & 2;
    const int lo = __builtin_unpredictable(k0) ? v1 : v0, hi = __builtin_unpredictable(k0) ? v3 : v2;
    return __builtin_unpredictable(k1) ? hi : lo;
}

// v[k] of seven values by a select tree on k's bits (k in 0..6)
__device__ __forceinline__ int st_sel7(int k, int v0, int v1, int v2, int v3, int v4, int v5, int v6)
{
    const bool k0 = k & 1, k1 = k & 2, k2 = k & 4;
    const int s01 = __builtin_unpredictable(k0) ? v1 : v0, s23 = __builtin_unpredictable(k0) ? v3 : v2,
              s45 = __builtin_unpredictable(k0) ? v5 : v4;
    const int s03 = __builtin_unpredictable(k1) ? s23 : s01, s47 = __builtin_unpredictable(k1) ? v6 : s45;
    return __builtin_unpredictable(k2) ? s47 : s03;
}

// low word of a granule published for this sweep (bounded spin; error bit 4 on timeout)
__device__ __forceinline__ uint32_t st_inbox_word(const StParams &P, const unsigned long long *p)
{
    for (unsigned spins = 0;; ++spins) {
        const unsigned long long g = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (st_granule_ready(g, P.epoch)) return (uint32_t)g;
        if ((spins & 255u) == 255u && st_failed(P)) return 0xffffffffu;
        if (spins > ST_WATCHDOG / 4) {
            st_fail(P, 4);
            return 0xffffffffu;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

__device__ __forceinline__ size_t st_phys(const StParams &P, int a, int b, int c)
{
    const int i = P.di > 0 ? a + 1 : P.ni - 2 - a;
    const int j = P.dj > 0 ? b + 1 : P.nj - 2 - b;
    const int k = P.dk > 0 ? c + 1 : P.nk - 2 - c;
    return (size_t)i + (size_t)P.ni * ((size_t)j + (size_t)P.nj * (size_t)k);
}

__device__ __forceinline__ f3 st_gx(const StParams &P, int a, int b, int c)
{
    const int i = P.di > 0 ? a + 1 : P.ni - 2 - a;
    const int j = P.dj > 0 ? b + 1 : P.nj - 2 - b;
    const int k = P.dk > 0 ? c + 1 : P.nk - 2 - c;
    return mk3((float)i * P.dx + P.ox, (float)j * P.dx + P.oy, (float)k * P.dx + P.oz);
}

__device__ __forceinline__ f3 st_xyz(float4 v) { return mk3(v.x, v.y, v.z); }

__device__ __forceinline__ int lds_ld(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// part k (0..2) of LDS entry e (48 bytes: 3 float4): e a byte offset (EB, the quad tiles) or an index
template <bool EB>
__device__ __forceinline__ float4 &st_e(float4 *s_ent, int e, int k)
{
    if constexpr (EB) return *(float4 *)((char *)s_ent + e + 16 * k);
    else return s_ent[__umul24(e, 3) + k];
}
__device__ __forceinline__ void lds_st(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// all of this wave's LDS writes have executed before anything after this point
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


__device__ __forceinline__ void st_load_tri(const float4 *soup, int t, float4 &v0, float4 &v1, float4 &v2)
{
    if (t >= 0) {
        v0 = soup[3 * (size_t)t];
        v1 = soup[3 * (size_t)t + 1];
        v2 = soup[3 * (size_t)t + 2];
    } else {
        v0 = v1 = v2 = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// SLAB: halo granules may come from another GPU (IPC-mapped inbox), so granule loads
// and stores are made at system scope; the single-GPU build keeps agent scope.
// TRACE: per-task timestamps for tools/trace_diag.py (kept out of the normal build's loop).
// MULTI: one launch runs the tasks of several consecutive sweeps (the first pass), each task
// first waiting for the tiles of the previous sweep whose cells it reads or overwrites; the
// task order is topological, so every awaited tile is already claimed.
template <class Cfg, bool SLAB, bool TRACE, bool MULTI = false>
__global__ void __launch_bounds__(Cfg::THREADS, Cfg::WPE) k_sweep_tile(StParams P0)
{
    constexpr int ST_NCW = Cfg::NCW, ST_CLW = Cfg::CLW, ST_CPW = Cfg::CPW, ST_RR = Cfg::RR, ST_THREADS = Cfg::THREADS,
                  ST_RING0 = Cfg::RING0, ST_HALO0 = Cfg::HALO0, ST_OWN0 = Cfg::OWN0, ST_ENTS = Cfg::ENTS;
    constexpr bool TWIN = Cfg::TWIN;
    StParams P = P0;
    constexpr int GSCOPE = SLAB ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT;
    __shared__ float4 s_ent[ST_ENTS * 3];   // entry e: [3e] = (x1, label), [3e+1] = (x2, phi), [3e+2] = x3
    // per compute wave (not used by the lanes-per-cell step: one word then):
    // s_pd[w]: [0, 7 CPW) the (entry << 9 | q << 6 | lane) list, [7 CPW, 14 CPW) the distance bits of
    // candidate q for lane (q * CPW + lane), then ONE trash word per lane shared by both (the target of
    // lanes with nothing to store, so the stores need no divergent branch; one trash area instead of
    // two leaves room for a 16-slot halo ring at 3 tiles per CU)
    __shared__ int s_pd[ST_NCW][Cfg::QUAD ? 1 : 14 * ST_CPW + 64];
    // s_hdr: [0] own entries ready for steps < s_hdr[0] (helper), [1 + w] steps completed by
    // compute wave w.
    __shared__ __attribute__((aligned(16))) int s_hdr[ST_NCW < 4 ? 4 : (ST_NCW < 8 ? 8 : 12)];
    // halo entries < s_halo_ready[s] are in LDS; the extra last word is never "not ready"
    // (the stream index of lanes that read no halo stream)
    __shared__ int s_halo_ready[ST_NSTREAM + 1];
    __shared__ int s_abort;
    __shared__ int s_task;
    // ST_CWA: own cells' words (phi, label) of steps [fA, fCl) for the helper's gathers, slot (step & (RC - 1))
    __shared__ unsigned long long s_cw[ST_CWA ? ST_RC * ST_NCOL : 1];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int L = tid & 63;
    unsigned long long n_evals = 0, n_cpoll = 0, n_hpoll = 0, n_cpoll_own = 0;

    if (SLAB && !MULTI && P.hc_out) {
        // publish this slab's last plane's face cells (a = -1 or b = -1; constant during the
        // sweep) to the downstream slab before any task runs (MULTI: per task, below)
        const int nf = P.A + 1 + P.B;
        for (int f = blockIdx.x * ST_THREADS + tid; f < nf; f += gridDim.x * ST_THREADS) {
            const int a = f <= P.A ? f - 1 : -1, b = f <= P.A ? -1 : f - (P.A + 1);
            const uint32_t w = (uint32_t)P.cell[SDF_CHK(1, st_phys(P, a, b, P.ce - 1), P.clo, P.chi)];
            __hip_atomic_store(P.hc_out + SDF_CHK(9, st_inbox(P, a, b), 0, (size_t)(P.A + 1) * (P.B + 1)),
                               st_granule(P.epoch, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    for (;;) {
        if (tid == 0) s_task = atomicAdd(P.queue, 1);   // a fired watchdog pushes the counter past the end
        __syncthreads();
        const int task = s_task;
        if (task >= P.ntasks) break;
        // TRACE + MULTI (tools/trace_multi.py): [0] setup done, [1] step 0 done, [2] first b-edge halo
        // entries (from tile J - 1) landed, [3] end, [4] first own entries landed, [5] step 8 done, [6] sweep slot << 32 | J << 16 | K,
        // [7] claim time
        const unsigned long long t_claim = (TRACE && MULTI && P.trace) ? wall_clock64() : 0ull;
        int J, K;
        if (MULTI) {
            const int4 tk = P0.mtasks[task];
            J = tk.x;
            K = tk.y;
            const StSweep &sw = P0.sw[tk.z];
            P.hb = sw.hb;
            P.hc = sw.hc;
            P.di = sw.di;
            P.dj = sw.dj;
            P.dk = sw.dk;
            P.sweep = sw.sweep;
            P.epoch = sw.epoch;
#pragma unroll
            for (int q = 0; q < 7; ++q) P.seen[q] = sw.seen[q];
            if (SLAB) {
                P.cs = sw.cs;
                P.ce = sw.ce;
                P.hbC = sw.ce - sw.cs;
                P.nK = sw.nK;
                P.hc_in = sw.hc_in;
                P.hc_out = sw.hc_out;
            }
            if (wave == 0) {
                // the previous sweep's tiles under and around this one: their cell stores first
                const int dep = L < ST_MAXDEP ? P0.deps[(size_t)task * ST_MAXDEP + L] : -1;
                bool ok = dep < 0;
                for (unsigned spins = 0;; ++spins) {
                    if (!ok) ok = __hip_atomic_load(P0.done + dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                  P0.call_epoch;
                    if (__all(ok)) break;
                    if (spins > ST_WATCHDOG || ((spins & 255u) == 255u && st_failed(P))) {
                        if (L == 0) st_fail(P, 8);
                        break;
                    }
                    if (spins < 16) __builtin_amdgcn_s_sleep(1);
                    else __builtin_amdgcn_s_sleep(8);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // this CU reads them fresh
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            if (SLAB && P.hc_out && K == P.nK - 1) {
                // The tile on the slab's last plane publishes that plane's face cells it covers
                // (a = -1 for its b range; tile J = 0 also the b = -1 row): constant during this
                // sweep and final for the previous one, since its dependencies above include every
                // previous-sweep tile writing them.  (With overlapped sweeps the kernel-start
                // publish of the per-sweep launches would race the previous sweep.)
                const int b_lo = J * ST_T, b_hi = min(P.B, b_lo + ST_T);
                const int nf = (b_hi - b_lo) + (J == 0 ? P.A + 1 : 0);
                for (int f = tid; f < nf; f += ST_THREADS) {
                    const int a = f < b_hi - b_lo ? -1 : f - (b_hi - b_lo) - 1;
                    const int b = f < b_hi - b_lo ? b_lo + f : -1;
                    const uint32_t w = (uint32_t)P.cell[SDF_CHK(2, st_phys(P, a, b, P.ce - 1), P.clo, P.chi)];
                    __hip_atomic_store(P.hc_out + SDF_CHK(9, st_inbox(P, a, b), 0, (size_t)(P.A + 1) * (P.B + 1)),
                                       st_granule(P.epoch, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        } else {
            const int2 JK = P.tasks[task];
            J = JK.x;
            K = JK.y;
        }
        const int b0 = J * ST_T, c0 = P.cs + K * ST_T;
        const bool inbox = SLAB && K == 0 && P.hc_in != nullptr;   // c0-1 lives on the upstream GPU
        const int nsteps = P.A + 2 * (ST_T - 1);

        // ---------------- task setup, then one barrier ----------------
        if (wave < ST_NCW) {
            if (L < ST_CPW) {
                // a = -1 entry of each column (boundary plane, constant) -> ring slot 7
                const int bl = L & (ST_T - 1), cl = ST_CLW * wave + (L >> 3);
                const int b = b0 + bl, c = c0 + cl;
                float4 v0, v1, v2;
                uint32_t w = 0xffffffffu;
                if (b < P.B && c < P.ce) w = (uint32_t)P.cell[SDF_CHK(3, st_phys(P, -1, b, c), P.clo, P.chi)];
                st_load_tri(P.soup, lbl_of(w), v0, v1, v2);
                const int e = ST_RING0 + (ST_RR - 1) * ST_NCOL + cl * ST_T + bl;
                s_ent[3 * e] = make_float4(v0.x, v0.y, v0.z, __uint_as_float(w));
                s_ent[3 * e + 1] = v1;
                s_ent[3 * e + 2] = v2;
            }
            if (L == 0) s_hdr[1 + wave] = 0;
            if (wave == 0 && L == 0) {
                s_hdr[0] = 0;
                s_abort = 0;
                s_halo_ready[ST_NSTREAM] = 0x3fffffff;
            }
        } else if ((Cfg::NH == 1 || wave == ST_NCW) && L < ST_NSTREAM) {
            int hb_ = 0, hc_ = 0;
            bool valid;
            if (L < ST_T) { hb_ = b0 - 1; hc_ = c0 + L; valid = hc_ < P.ce; }
            else if (L < 2 * ST_T) { hb_ = b0 + (L - ST_T); hc_ = c0 - 1; valid = hb_ < P.B; }
            else { hb_ = b0 - 1; hc_ = c0 - 1; valid = true; }
            float4 v0, v1, v2;
            uint32_t w = 0xffffffffu;
            if (valid) {
                if (inbox && L >= ST_T)
                    w = st_inbox_word(P, P.hc_in + SDF_CHK(8, st_inbox(P, -1, hb_), 0, (size_t)(P.A + 1) * (P.B + 1)));
                else w = (uint32_t)P.cell[SDF_CHK(4, st_phys(P, -1, hb_, hc_), P.clo, P.chi)];
            }
            st_load_tri(P.soup, lbl_of(w), v0, v1, v2);
            const int e = ST_HALO0 + L * ST_RH + (ST_RH - 1);
            s_ent[3 * e] = make_float4(v0.x, v0.y, v0.z, __uint_as_float(w));
            s_ent[3 * e + 1] = v1;
            s_ent[3 * e + 2] = v2;
            s_halo_ready[L] = valid ? 0 : P.A;
        }
        __syncthreads();

        if (TRACE && P.trace && tid == 0) P.trace[8 * task] = wall_clock64();
        if (wave < ST_NCW) {
            // ======================= compute waves =======================
            // Nothing of this wave is in flight here (the task's set-up loads were consumed above).  Said with the
            // builtin, not an asm, so the compiler's wait-count pass knows it: its scoreboard is per function, and
            // without this it carried the helper branch's pending load registers (a role the same wave never takes)
            // into the step loop, where the 1-wave tiles then waited for their own previous step's granule and
            // cell stores (vmcnt(0) in every evaluation pass) (ST_COMPUTE_WAIT0)
            if (ST_COMPUTE_WAIT0) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt / lgkmcnt unchanged (gfx9 encoding)
            // Wave w owns the ST_CLW c-columns from ST_CLW * w on: lanes 0..31 are its 32 cells.
            // Wave w steps h only after wave w-1 finished step h-1 (its column cl-1 results) and
            // at most RR-4 steps ahead of wave w+1 (ring slots).  TWIN: lane L + 32 is the twin
            // of cell lane L -- same cell, same candidate mask; L evaluates the cell's 1st, 3rd, ...
            // candidate and L + 32 its 2nd, 4th, ..., handed back with one v_permlane32_swap.
            const int w = wave;
            // lane -> cell: cell lanes 0 .. CPW-1 (TWIN: lane L + 32 the twin of L); QUAD: cell x is lanes
            // 4x .. 4x + 3, the lane's rank qr = L & 3, and lane 4x applies and stores
            const int lcell = L >> Cfg::LPC_SH;
            const int qr = L & (Cfg::LPC - 1);
            const bool cell_lane = Cfg::QUAD ? (qr == 0) : (L < ST_CPW);
            const int bl = lcell & (ST_T - 1), cl = ST_CLW * w + ((lcell >> 3) & (ST_CLW - 1));
            const int col_id = cl * ST_T + bl;
            const int b = b0 + bl, c = c0 + cl;
            const bool colx = b < P.B && c < P.ce;   // the cell (cell lane or twin)
            const bool col = cell_lane && colx;
            __builtin_amdgcn_s_setprio(ST_WORK_PRIO);
            // neighbour q's entry at step h: nb_base[q] + ((aq & nb_mask[q]) << nb_sh[q]) (ring slots are
            // ST_NCOL = 64 entries apart, halo slots 1); quad tiles keep it as a byte offset (EB below)
            // QUAD (128 VGPRs): ring and halo slots have the same mask (RR == RH), so the shift rides in
            // the base's high bits and the three arrays are one (14 VGPRs fewer)
            constexpr bool NB_PACK = Cfg::QUAD && ST_RR == ST_RH;
            // the quad tiles address entries by byte offset (one shift-add per neighbour instead of a
            // shift-add and a multiply: C3 first pass -1.6 %); the others by index (the byte form
            // measured +0.9 % on the 1-wave tiles at 512^3)
            constexpr bool EB = NB_PACK;
            constexpr int ES = EB ? 48 : 1;   // entry stride in the addressing unit
            int nb_base[7], nb_sh[7], nb_mask[7];
            {
                static_assert(ST_NCOL == 64, "ring slot stride is a shift by 6");
                auto ring = [&](int q, int lbl, int lcl) {
                    nb_base[q] = ST_RING0 + lcl * ST_T + lbl;
                    nb_sh[q] = 6;
                    nb_mask[q] = ST_RR - 1;
                    if constexpr (NB_PACK) nb_base[q] |= 6 << 16;
                };
                auto halo = [&](int q, int s) {
                    nb_base[q] = ST_HALO0 + s * ST_RH;
                    nb_sh[q] = 0;
                    nb_mask[q] = ST_RH - 1;
                };
                ring(0, bl, cl);                                              // (a-1, b,   c)
                if (bl > 0) { ring(1, bl - 1, cl); ring(2, bl - 1, cl); }     // (.,   b-1, c)
                else { halo(1, cl); halo(2, cl); }
                if (cl > 0) { ring(3, bl, cl - 1); ring(4, bl, cl - 1); }     // (.,   b,   c-1)
                else { halo(3, ST_T + bl); halo(4, ST_T + bl); }
                if (bl > 0 && cl > 0) { ring(5, bl - 1, cl - 1); ring(6, bl - 1, cl - 1); }   // (., b-1, c-1)
                else if (bl == 0 && cl == 0) { halo(5, 2 * ST_T); halo(6, 2 * ST_T); }
                else if (bl == 0) { halo(5, cl - 1); halo(6, cl - 1); }
                else { halo(5, ST_T + bl - 1); halo(6, ST_T + bl - 1); }
                static_assert(!EB || ST_ENTS * 48 < 65536, "packed byte offsets need 16 bits");
                if constexpr (EB) {
#pragma unroll
                    for (int q = 0; q < 7; ++q) nb_base[q] = ((nb_base[q] & 0xffff) * 48) | (nb_base[q] & ~0xffff);
                }
            }
            // oct lanes: lane qr's fixed entry -- qr = 0 the cell's own (own ring), qr = 1 + q upwind
            // neighbour q -- as a byte offset o_base + ((((a - o_am) & o_mask) * 48) << o_sh)
            int o_base = 0, o_sh = 6, o_mask = ST_RO - 1, o_am = 0, o_seen = -1;
            if constexpr (Cfg::LPC == 8) {
                const int q = qr - 1, qs = qr > 0 ? q : 0;
                const int nbq = st_sel7(qs, nb_base[0], nb_base[1], nb_base[2], nb_base[3], nb_base[4], nb_base[5], nb_base[6]);
                o_base = qr > 0 ? (nbq & 0xffff) : __umul24(ST_OWN0 + col_id, 48);
                o_sh = qr > 0 ? (nbq >> 16) : 6;
                o_mask = qr > 0 ? ST_RR - 1 : ST_RO - 1;   // ring and halo slots: RR == RH (NB_PACK)
                o_am = (qr > 0 && (q & 1) == 0) ? 1 : 0;   // q = 0, 2, 4, 6 read a - 1
                o_seen = qr > 0 ? st_sel7(qs, P.seen[0], P.seen[1], P.seen[2], P.seen[3], P.seen[4], P.seen[5], P.seen[6]) : -1;
                static_assert(Cfg::LPC != 8 || (NB_PACK && ST_RR == ST_RH), "oct lanes: packed byte-offset entries");
            }
            // fixed quad lanes: slot A = neighbour q = qr (o_*), slot B = neighbour q = qr + 4, or (qr = 3) the own entry
            int f_base = 0, f_sh = 6, f_mask = ST_RO - 1, f_am = 0, f_seen = -1;
            if constexpr (Cfg::FIX) {
                const int nba = st_sel4(qr, nb_base[0], nb_base[1], nb_base[2], nb_base[3]);
                o_base = nba & 0xffff;
                o_sh = nba >> 16;
                o_mask = ST_RR - 1;
                o_am = (qr & 1) ? 0 : 1;   // q = 0, 2 read a - 1
                o_seen = st_sel4(qr, P.seen[0], P.seen[1], P.seen[2], P.seen[3]);
                const int nbb = st_sel4(qr, nb_base[4], nb_base[5], nb_base[6], nb_base[6]);
                f_base = qr < 3 ? (nbb & 0xffff) : __umul24(ST_OWN0 + col_id, 48);
                f_sh = qr < 3 ? (nbb >> 16) : 6;
                f_mask = qr < 3 ? ST_RR - 1 : ST_RO - 1;
                f_am = (qr == 0 || qr == 2) ? 1 : 0;   // q = 4, 6 read a - 1; q = 5 and the own entry read a
                f_seen = qr < 3 ? st_sel4(qr, P.seen[4], P.seen[5], P.seen[6], P.seen[6]) : -1;
                static_assert(!Cfg::FIX || (Cfg::LPC == 4 && NB_PACK && ST_RR == ST_RH), "fixed quad lanes: packed byte-offset entries");
            }
            const int hsA = (bl == 0) ? cl : ST_NSTREAM, hsB = (cl == 0) ? ST_T + bl : ST_NSTREAM,
                      hsC = (bl == 0 && cl == 0) ? 2 * ST_T : ST_NSTREAM;
            unsigned polls = 0;
            unsigned long long t_wait = 0, w_own = 0, w_halo = 0, t_comp = 0, c_comp = 0;   // trace-only
#ifdef ST_STEP_PROF   // diagnostics: where a compute step's cycles go (host prints the sums)
            unsigned long long sp_c[4] = {0, 0, 0, 0}, sp_n[4] = {0, 0, 0, 0}, sp_t = 0, sp_ev[2] = {0, 0}, sp_pw[3] = {0, 0, 0};
#endif
            for (int h = 0; h < nsteps; ++h) {
#ifdef ST_STEP_PROF
                sp_t = clock64();
#endif
                const int a = h - bl - cl;
                // ring slot of a and of a - 1 (RR = 3: a modulo; a > -2^20 here)
                const int am = Cfg::RR_POW2 ? (a & (ST_RR - 1)) : (int)((unsigned)(a + 3 * (1 << 20)) % (unsigned)ST_RR);
                const int amm = Cfg::RR_POW2 ? ((a - 1) & (ST_RR - 1)) : (am == 0 ? ST_RR - 1 : am - 1);
                const bool act = col && a >= 0 && a < P.A;
                const bool actx = ((TWIN || Cfg::QUAD) ? colx : col) && a >= 0 && a < P.A;   // the lanes that evaluate
                // ---- wait for: own data + halo (helper), wave w-1's step h-1, ring space in w+1 ----
                unsigned long long tw0 = 0;
                for (;;) {
                    // branch-free: the 4 header words + the (up to 3) halo streams this lane
                    // reads at this step (the dummy word for lanes off the tile edge), 7 ds_read_b32
                    // issued together.  (A volatile 16-byte read of s_hdr through a generic pointer
                    // compiled to a FLAT load: vector-memory latency on every poll, 8 % of the
                    // first pass at 256^3, 14 % at 512^3.)
                    int hx, pm, pp;   // own entries ready, prog[w-1] (w > 0), prog[w+1] (w < NCW - 1)
                    if constexpr (ST_NCW <= 3) {
                        const i4v H = i4v{lds_ld(&s_hdr[0]), lds_ld(&s_hdr[1]), lds_ld(&s_hdr[2]), lds_ld(&s_hdr[3])};
                        hx = H.x;
                        pm = (w == 1) ? H.y : ((w == 2) ? H.z : H.w);
                        pp = (w == 0) ? H.y : ((w == 1) ? H.z : H.w);
                    } else {
                        hx = lds_ld(&s_hdr[0]);
                        pm = lds_ld(&s_hdr[w > 0 ? w : 1]);
                        pp = lds_ld(&s_hdr[w < ST_NCW - 1 ? w + 2 : 1]);
                    }
                    const int rA = lds_ld(&s_halo_ready[hsA]), rB = lds_ld(&s_halo_ready[hsB]),
                              rC = lds_ld(&s_halo_ready[hsC]);
                    const bool own_ok = hx > h;
                    const bool ok = own_ok & ((w == 0) | (pm >= h)) & ((w == ST_NCW - 1) | (pp >= h - P.lead)) &
                                    (!act | (min(rA, min(rB, rC)) > a));
                    if (__all(ok)) break;
                    if (TRACE && P.trace && tw0 == 0) {
                        tw0 = wall_clock64();
                        if (!__all(own_ok)) ++w_own; else ++w_halo;
                    }
                    ++n_cpoll;
                    if (!__all(own_ok)) ++n_cpoll_own;
#ifdef ST_STEP_PROF
                    if (!__all((w == 0) | (pm >= h))) ++sp_pw[0];                 // waits on wave w-1
                    if (!__all((w == ST_NCW - 1) | (pp >= h - P.lead))) ++sp_pw[1];   // ... on wave w+1's ring space
                    if (!__all(!act | (min(rA, min(rB, rC)) > a))) ++sp_pw[2];     // ... on halo entries
#endif
                    // a waiting wave yields its SIMD's issue slots to the working waves there (the
                    // step is issue-latency bound: -3 % first pass at 256^3)
                    __builtin_amdgcn_s_setprio(0);
                    if (++polls > ST_WATCHDOG || lds_ld(&s_abort)) {
                        // the stuck task and its step, for st_watchdog_report: err[3] = task + 1 (the first
                        // failure only), err[10] = h + 1 (lane 0 alone: a per-lane reduction here cost the
                        // step loop 2 spilled VGPRs and ~2 % of the first pass, round 5)
                        if (polls > ST_WATCHDOG && L == 0) {
                            if (atomicCAS(P.err + 3, 0, task + 1) == 0) atomicExch(P.err + 10, h + 1);
                            st_fail(P, 2);
                        }
                        if (L == 0) lds_st(&s_abort, 1);
                        h = nsteps;
                        break;
                    }
                    // waiting tiles back off: their polls share the SIMD with the tiles they wait for
                    if (polls < 8) __builtin_amdgcn_s_sleep(1);
                    else if (polls < 64) __builtin_amdgcn_s_sleep(2);
                    else __builtin_amdgcn_s_sleep(ST_CSLEEP);
                }
                __builtin_amdgcn_s_setprio(ST_WORK_PRIO);
                asm volatile("" ::: "memory");   // no LDS read moves above the readiness poll
                if (TRACE && tw0) t_wait += wall_clock64() - tw0;
                if (h >= nsteps) break;
#ifdef ST_STEP_PROF
                { const unsigned long long t_ = clock64(); sp_c[0] += t_ - sp_t; sp_t = t_; }
#endif
                const unsigned long long tc0 = (TRACE && P.trace) ? wall_clock64() : 0ull;
                const unsigned long long cc0 = (TRACE && P.trace) ? clock64() : 0ull;
                polls = 0;
                if constexpr (Cfg::LPC == 8) {
                    // ---- oct lanes: ONE batch of LDS reads -- lane qr's entry (label + vertices) and the
                    //      cell's own label and phi -- then lane 1 + q evaluates neighbour q's triangle unless
                    //      it is none, the cell's own label or already examined (exact skips: sweep_sparse.hpp),
                    //      a first minimum over the 7 candidates in check order (ties to the lower q: the
                    //      reference's strict '<' applied in order, cpu_lib/makelevelset3.cpp:94-99, 143-149),
                    //      then '<' against phi.  The winner lane (lane 0 if nothing wins) writes back. ----
                    float4 p0 = make_float4(0.f, 0.f, 0.f, 0.f), p1 = p0, p2 = p0;
                    uint32_t ownw = 0xffffffffu;
                    float ownphi = 0.f;
                    if (actx) {
                        const int e = o_base + (__umul24((a - o_am) & o_mask, 48) << o_sh);
                        const int eo = __umul24(ST_OWN0 + (a & (ST_RO - 1)) * ST_NCOL + col_id, 48);
                        p0 = st_e<true>(s_ent, e, 0);
                        p1 = st_e<true>(s_ent, e, 1);
                        p2 = st_e<true>(s_ent, e, 2);
                        ownw = __float_as_uint(st_e<true>(s_ent, eo, 0).w);
                        ownphi = st_e<true>(s_ent, eo, 1).w;
                    }
                    const uint32_t wq = __float_as_uint(p0.w);
                    const bool interior = a <= P.A - 2 && b <= P.B - 2 && c <= P.C - 2;
                    const bool keep = actx && qr > 0 && (wq & LBL_MASK) != LBL_MASK && (wq & LBL_MASK) != (ownw & LBL_MASK) &&
                                      !(interior && lc_of(wq) <= o_seen);
#ifdef ST_STEP_PROF
                    {
                        const unsigned long long t_ = clock64();
                        sp_c[1] += t_ - sp_t;
                        sp_t = t_;
                        ++sp_n[__any(keep) ? 1 : 0];
                    }
#endif
                    float key = __builtin_inff();
                    if (__any(keep)) {
                        const float d = ptd_wave(st_gx(P, a, b, c), st_xyz(p0), st_xyz(p1), st_xyz(p2), p2.w);
                        key = (keep && d == d) ? d : __builtin_inff();
                        if (P.stats) n_evals += (L == 0) ? (unsigned long long)__popcll(__ballot(keep)) : 0ull;
                    }
                    // first minimum over the 8 lanes of the cell (keys are never NaN): partner lane^1, lane^2,
                    // then the other quad (row_half_mirror: lane i <-> 7 - i); the higher lane gives way on ties
                    int idx = qr;
                    {
                        float kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0xB1, 0xf, 0xf, false));
                        int ip = __builtin_amdgcn_mov_dpp(idx, 0xB1, 0xf, 0xf, false);
                        bool tk = (kp < key) | ((qr & 1) && kp == key);
                        key = tk ? kp : key;
                        idx = tk ? ip : idx;
                        kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0x4E, 0xf, 0xf, false));
                        ip = __builtin_amdgcn_mov_dpp(idx, 0x4E, 0xf, 0xf, false);
                        tk = (kp < key) | ((qr & 2) && kp == key);
                        key = tk ? kp : key;
                        idx = tk ? ip : idx;
                        kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0x141, 0xf, 0xf, false));
                        ip = __builtin_amdgcn_mov_dpp(idx, 0x141, 0xf, 0xf, false);
                        tk = (kp < key) | ((qr & 4) && kp == key);
                        key = tk ? kp : key;
                        idx = tk ? ip : idx;
                    }
#ifdef ST_STEP_PROF
                    { const unsigned long long t_ = clock64(); sp_c[2] += t_ - sp_t; sp_ev[0] += t_ - sp_t; sp_t = t_; }
#endif
                    const bool take = key < ownphi;   // NaN phi: nothing replaces it, as in the reference
                    if (actx && qr == (take ? idx : 0)) {
                        const uint32_t w_new = take ? lo_word((int)(wq & LBL_MASK), P.sweep + 1) : ownw;
                        const float phi_new = take ? key : ownphi;
                        const int slot = __umul24(ST_RING0 + (a & (ST_RR - 1)) * ST_NCOL + col_id, 48);
                        st_e<true>(s_ent, slot, 0) = make_float4(p0.x, p0.y, p0.z, __uint_as_float(w_new));
                        st_e<true>(s_ent, slot, 1) = make_float4(p1.x, p1.y, p1.z, phi_new);
                        st_e<true>(s_ent, slot, 2) = p2;
                        if (take && ST_DIAG_SPLIT != 1)
                            P.cell[SDF_CHK(5, st_phys(P, a, b, c), P.clo, P.chi)] =
                                ((unsigned long long)__float_as_uint(phi_new) << 32) | w_new;
                        const unsigned long long gran = st_granule(P.epoch, w_new);
                        if (bl == ST_T - 1 && J < P.nJ - 1)
                            __hip_atomic_store(P.hb + ((size_t)J * P.hbC + (c - P.cs)) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                        if (cl == ST_T - 1 && K < P.nK - 1)
                            __hip_atomic_store(P.hc + ((size_t)K * P.B + b) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                        if (SLAB && P.hc_out && c == P.ce - 1)
                            __hip_atomic_store(P.hc_out + st_inbox(P, a, b), gran, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                } else if constexpr (Cfg::FIX) {
                    // ---- fixed quad lanes: one batch of LDS reads (lane qr: neighbours qr and qr + 4, lane 3 the
                    //      own entry as its second slot; every lane the own label and phi), one packed pass
                    //      (ptd_wave2), first minima over the quad for q = 0..3 and q = 4..6 (ties to the lower
                    //      q; the q = 0..3 group wins ties against q = 4..6), then '<' against phi -- the
                    //      reference's strict '<' in check order (cpu_lib/makelevelset3.cpp:94-99, 143-149) ----
                    float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, b0_ = a0, b1_ = a0, b2_ = a0;
                    uint32_t ownw = 0xffffffffu;
                    float ownphi = 0.f;
                    const int ea = o_base + (__umul24((a - o_am) & o_mask, 48) << o_sh);
                    const int eb = f_base + (__umul24((a - f_am) & f_mask, 48) << f_sh);
                    if (actx) {
                        const int eo = __umul24(ST_OWN0 + (a & (ST_RO - 1)) * ST_NCOL + col_id, 48);
                        a0 = st_e<true>(s_ent, ea, 0);
                        a1 = st_e<true>(s_ent, ea, 1);
                        a2 = st_e<true>(s_ent, ea, 2);
                        b0_ = st_e<true>(s_ent, eb, 0);
                        b1_ = st_e<true>(s_ent, eb, 1);
                        b2_ = st_e<true>(s_ent, eb, 2);
                        ownw = __float_as_uint(st_e<true>(s_ent, eo, 0).w);
                        ownphi = st_e<true>(s_ent, eo, 1).w;
                    }
                    const uint32_t wa = __float_as_uint(a0.w), wb = __float_as_uint(b0_.w);
                    const bool interior = a <= P.A - 2 && b <= P.B - 2 && c <= P.C - 2;
                    const uint32_t own_raw = ownw & LBL_MASK;
                    const bool keep_a = actx && (wa & LBL_MASK) != LBL_MASK && (wa & LBL_MASK) != own_raw &&
                                        !(interior && lc_of(wa) <= o_seen);
                    const bool keep_b = actx && qr < 3 && (wb & LBL_MASK) != LBL_MASK && (wb & LBL_MASK) != own_raw &&
                                        !(interior && lc_of(wb) <= f_seen);
#ifdef ST_STEP_PROF
                    {
                        const unsigned long long t_ = clock64();
                        sp_c[1] += t_ - sp_t;
                        sp_t = t_;
                        ++sp_n[__any(keep_a | keep_b) ? (__any(keep_b) ? 2 : 1) : 0];
                    }
#endif
                    float ka = __builtin_inff(), kb = __builtin_inff();
                    if (__any(keep_a | keep_b)) {
                        const f3 gx = st_gx(P, a, b, c);
                        float da, db;
                        ptd_wave2(gx, st_xyz(a0), st_xyz(a1), st_xyz(a2), a2.w, gx, st_xyz(b0_), st_xyz(b1_), st_xyz(b2_), b2_.w,
                                  da, db);
                        ka = (keep_a && da == da) ? da : __builtin_inff();
                        kb = (keep_b && db == db) ? db : __builtin_inff();
                        if (P.stats) n_evals += (L == 0) ? (unsigned long long)(__popcll(__ballot(keep_a)) + __popcll(__ballot(keep_b))) : 0ull;
                    }
                    // first minima over the quad (keys are never NaN), the higher lane giving way on ties
                    int ia = qr, ib = qr;
                    {
                        const bool q_odd = qr & 1, q_hi = qr & 2;
                        float kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(ka), 0xB1, 0xf, 0xf, false));
                        int ip = __builtin_amdgcn_mov_dpp(ia, 0xB1, 0xf, 0xf, false);
                        bool tk = (kp < ka) | (q_odd & (kp == ka));
                        ka = tk ? kp : ka;
                        ia = tk ? ip : ia;
                        float kq = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(kb), 0xB1, 0xf, 0xf, false));
                        int iq = __builtin_amdgcn_mov_dpp(ib, 0xB1, 0xf, 0xf, false);
                        bool tq = (kq < kb) | (q_odd & (kq == kb));
                        kb = tq ? kq : kb;
                        ib = tq ? iq : ib;
                        kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(ka), 0x4E, 0xf, 0xf, false));
                        ip = __builtin_amdgcn_mov_dpp(ia, 0x4E, 0xf, 0xf, false);
                        tk = (kp < ka) | (q_hi & (kp == ka));
                        ka = tk ? kp : ka;
                        ia = tk ? ip : ia;
                        kq = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(kb), 0x4E, 0xf, 0xf, false));
                        iq = __builtin_amdgcn_mov_dpp(ib, 0x4E, 0xf, 0xf, false);
                        tq = (kq < kb) | (q_hi & (kq == kb));
                        kb = tq ? kq : kb;
                        ib = tq ? iq : ib;
                    }
#ifdef ST_STEP_PROF
                    { const unsigned long long t_ = clock64(); sp_c[2] += t_ - sp_t; sp_ev[0] += t_ - sp_t; sp_t = t_; }
#endif
                    const bool use_b = kb < ka;   // q = 4..6 strictly closer than the best of q = 0..3
                    const float key = use_b ? kb : ka;
                    const int widx = use_b ? ib : ia;
                    const bool take = key < ownphi;   // NaN phi: nothing replaces it, as in the reference
                    // writer: the winner's lane (its slot A or B), else lane 3 (the own entry in its slot B)
                    if (actx && qr == (take ? widx : 3)) {
                        // the winner's entry read back (holding both slots' vertices through the packed
                        // pass took the register allocator past its limits)
                        const int src = (!take || use_b) ? eb : ea;
                        const float4 w0 = st_e<true>(s_ent, src, 0), w1 = st_e<true>(s_ent, src, 1), w2 = st_e<true>(s_ent, src, 2);
                        const uint32_t w_new = take ? lo_word((int)(__float_as_uint(w0.w) & LBL_MASK), P.sweep + 1) : ownw;
                        const float phi_new = take ? key : ownphi;
                        const int slot = __umul24(ST_RING0 + (a & (ST_RR - 1)) * ST_NCOL + col_id, 48);
                        st_e<true>(s_ent, slot, 0) = make_float4(w0.x, w0.y, w0.z, __uint_as_float(w_new));
                        st_e<true>(s_ent, slot, 1) = make_float4(w1.x, w1.y, w1.z, phi_new);
                        st_e<true>(s_ent, slot, 2) = w2;
                        if (take && ST_DIAG_SPLIT != 1)
                            P.cell[SDF_CHK(5, st_phys(P, a, b, c), P.clo, P.chi)] =
                                ((unsigned long long)__float_as_uint(phi_new) << 32) | w_new;
                        const unsigned long long gran = st_granule(P.epoch, w_new);
                        if (bl == ST_T - 1 && J < P.nJ - 1)
                            __hip_atomic_store(P.hb + ((size_t)J * P.hbC + (c - P.cs)) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                        if (cl == ST_T - 1 && K < P.nK - 1)
                            __hip_atomic_store(P.hc + ((size_t)K * P.B + b) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                        if (SLAB && P.hc_out && c == P.ce - 1)
                            __hip_atomic_store(P.hc_out + st_inbox(P, a, b), gran, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                } else {
                // ---- candidates: the 7 upwind labels minus exact duplicates ----
                float phi = 0.f;
                int ct = -1, win = -1;
                uint32_t own_w = 0xffffffffu;
                int lab[7], ent[7];
                unsigned fmask = 0;
                const int e_own = __umul24(ST_OWN0 + (a & (ST_RO - 1)) * ST_NCOL + col_id, ES);
                if (actx) {
                    const float4 o0 = st_e<EB>(s_ent, e_own, 0), o1 = st_e<EB>(s_ent, e_own, 1);
                    own_w = __float_as_uint(o0.w);
                    ct = lbl_of(own_w);
                    phi = o1.w;
                    int lcq[7];
                    const int t48a = __umul24(a & (ST_RR - 1), 48), t48m = __umul24((a - 1) & (ST_RR - 1), 48);
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
                        const int aq = (q & 1) == 0 ? a - 1 : a;   // q = 0,2,4,6 read a-1
                        if constexpr (EB)
                            ent[q] = (nb_base[q] & 0xffff) + (((q & 1) == 0 ? t48m : t48a) << (nb_base[q] >> 16));
                        else if constexpr (!Cfg::RR_POW2)   // ring entries (shift 6) by slot, halo entries by mask
                            ent[q] = nb_base[q] + ((nb_sh[q] == 6 ? ((q & 1) == 0 ? amm : am) : (aq & nb_mask[q])) << nb_sh[q]);
                        else
                            ent[q] = nb_base[q] + ((aq & nb_mask[q]) << nb_sh[q]);
                        const uint32_t wq = __float_as_uint(st_e<EB>(s_ent, ent[q], 0).w);
                        lab[q] = (int)(wq & LBL_MASK);   // raw (LBL_MASK = none): a candidate is never 'none'
                        lcq[q] = lc_of(wq);
                    }
                    // interior cells took part in every earlier sweep (sweep_sparse.hpp: exact skip)
                    const bool interior = a <= P.A - 2 && b <= P.B - 2 && c <= P.C - 2;
                    if constexpr (Cfg::LPC == 4 && ST_QMASK) {
                        // The quad splits the test: lane qr decides candidates q = qr and q = qr + 4
                        // (the 21 pairwise duplicate compares become at most 5 + 8 per lane), and an OR
                        // over the quad (two DPP moves) gives every lane the cell's mask.  Same rule as
                        // below, on raw labels (LBL_MASK = none; lbl_of is one-to-one on them).
                        uint32_t raw[7];
#pragma unroll
                        for (int q = 0; q < 7; ++q) raw[q] = (uint32_t)lab[q];
                        const uint32_t own_raw = own_w & LBL_MASK;
                        // (select trees on qr's bits: nested '?:' on qr compiled to exec-mask branches)
                        const uint32_t xa = (uint32_t)st_sel4(qr, (int)raw[0], (int)raw[1], (int)raw[2], (int)raw[3]);
                        const int la = st_sel4(qr, lcq[0], lcq[1], lcq[2], lcq[3]);
                        const int sa = st_sel4(qr, P.seen[0], P.seen[1], P.seen[2], P.seen[3]);
                        const uint32_t xb = (uint32_t)st_sel4(qr, (int)raw[4], (int)raw[5], (int)raw[6], (int)raw[6]);
                        const int lb = st_sel4(qr, lcq[4], lcq[5], lcq[6], lcq[6]);
                        const int sb = st_sel4(qr, P.seen[4], P.seen[5], P.seen[6], P.seen[6]);
#if ST_QVMASK
                        // integer VALU form (as sweep_sparse.hpp SP_VMASK): d = min of label ^ (none, own,
                        // earlier slots) is 0 exactly for a skipped label; bit 31 of (d | -d) is d != 0, bit
                        // 31 of (seen - lc) is lc > seen.  The lane's "earlier slot" terms it must not test
                        // are forced to all-ones (never 0) by per-lane masks.
                        auto opq = [](uint32_t x) { asm volatile("" : "+v"(x)); return x; };
                        const uint32_t m1 = qr < 1 ? ~0u : 0u, m2 = qr < 2 ? ~0u : 0u, m3 = qr < 3 ? ~0u : 0u;
                        const uint32_t itr = opq(interior ? ~0u : 0u);
                        uint32_t da = min(min(xa ^ LBL_MASK, xa ^ own_raw), (xa ^ raw[0]) | m1);
                        da = min(da, min((xa ^ raw[1]) | m2, (xa ^ raw[2]) | m3));
                        uint32_t db = min(min(xb ^ LBL_MASK, xb ^ own_raw), min(xb ^ raw[0], xb ^ raw[1]));
                        db = min(db, min(min(xb ^ raw[2], xb ^ raw[3]), min((xb ^ raw[4]) | m1, (xb ^ raw[5]) | m2)));
                        da = opq(da);
                        db = opq(db);
                        const uint32_t ka = (da | (0u - da)) & ((uint32_t)(sa - la) | ~itr);
                        const uint32_t kb = (db | (0u - db)) & ((uint32_t)(sb - lb) | ~itr) & m3;   // (lane 3 has no slot B)
                        unsigned bits = ((ka >> 31) << qr) | ((kb >> 31) << (qr + 4));
#else
                        const bool keep_a = (xa != LBL_MASK) & (xa != own_raw) & !(interior & (la <= sa)) &
                                            ((qr < 1) | (xa != raw[0])) & ((qr < 2) | (xa != raw[1])) &
                                            ((qr < 3) | (xa != raw[2]));
                        const bool keep_b = (qr < 3) & (xb != LBL_MASK) & (xb != own_raw) & !(interior & (lb <= sb)) &
                                            (xb != raw[0]) & (xb != raw[1]) & (xb != raw[2]) & (xb != raw[3]) &
                                            ((qr < 1) | (xb != raw[4])) & ((qr < 2) | (xb != raw[5]));
                        unsigned bits = ((keep_a ? 1u : 0u) << qr) | ((keep_b ? 1u : 0u) << (qr + 4));
#endif
                        bits |= (unsigned)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xf, 0xf, false);   // quad_perm(1,0,3,2)
                        bits |= (unsigned)__builtin_amdgcn_mov_dpp((int)bits, 0x4E, 0xf, 0xf, false);   // quad_perm(2,3,0,1)
                        fmask = bits;
                    } else if constexpr (Cfg::LPC == 2 && ST_QMASK) {
                        // Duo lanes: lane qr decides candidates q = qr, qr + 2, qr + 4 (and lane 0 also q = 6),
                        // an OR with the partner lane (one DPP move) gives both the cell's mask.
                        uint32_t raw[7];
#pragma unroll
                        for (int q = 0; q < 7; ++q) raw[q] = (uint32_t)lab[q];
                        const uint32_t own_raw = own_w & LBL_MASK;
                        const bool q1 = qr & 1;
                        const uint32_t xa = q1 ? raw[1] : raw[0], xb = q1 ? raw[3] : raw[2], xc = q1 ? raw[5] : raw[4], xd = raw[6];
                        const int la = q1 ? lcq[1] : lcq[0], lb = q1 ? lcq[3] : lcq[2], lc = q1 ? lcq[5] : lcq[4];
                        const int sa = q1 ? P.seen[1] : P.seen[0], sb = q1 ? P.seen[3] : P.seen[2], sc = q1 ? P.seen[5] : P.seen[4];
                        const bool keep_a = (xa != LBL_MASK) & (xa != own_raw) & !(interior & (la <= sa)) & (!q1 | (xa != raw[0]));
                        const bool keep_b = (xb != LBL_MASK) & (xb != own_raw) & !(interior & (lb <= sb)) & (xb != raw[0]) &
                                            (xb != raw[1]) & (!q1 | (xb != raw[2]));
                        const bool keep_c = (xc != LBL_MASK) & (xc != own_raw) & !(interior & (lc <= sc)) & (xc != raw[0]) &
                                            (xc != raw[1]) & (xc != raw[2]) & (xc != raw[3]) & (!q1 | (xc != raw[4]));
                        const bool keep_d = !q1 & (xd != LBL_MASK) & (xd != own_raw) & !(interior & (lcq[6] <= P.seen[6])) &
                                            (xd != raw[0]) & (xd != raw[1]) & (xd != raw[2]) & (xd != raw[3]) & (xd != raw[4]) &
                                            (xd != raw[5]);
                        unsigned bits = ((keep_a ? 1u : 0u) << qr) | ((keep_b ? 1u : 0u) << (qr + 2)) |
                                        ((keep_c ? 1u : 0u) << (qr + 4)) | ((keep_d ? 1u : 0u) << 6);
                        bits |= (unsigned)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xf, 0xf, false);   // quad_perm(1,0,3,2)
                        fmask = bits;
                    } else {
#if ST_GVMASK
                    // integer VALU form of the test below (as ST_QVMASK / sweep_sparse.hpp SP_VMASK)
                    auto opq = [](uint32_t x) { asm volatile("" : "+v"(x)); return x; };
                    const uint32_t own_raw = own_w & LBL_MASK, itr = opq(interior ? ~0u : 0u);
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
                        const uint32_t x = (uint32_t)lab[q];
                        uint32_t d = min(x ^ LBL_MASK, x ^ own_raw);
#pragma unroll
                        for (int r = 0; r < q; ++r) d = min(d, x ^ (uint32_t)lab[r]);
                        d = opq(d);
                        const uint32_t keep = (d | (0u - d)) & ((uint32_t)(P.seen[q] - lcq[q]) | ~itr);
                        fmask |= (keep >> 31) << q;
                    }
#else
#pragma unroll
                    for (int q = 0; q < 7; ++q) {   // bitwise, no short-circuit branches
                        bool skip = (lab[q] == (int)LBL_MASK) | (lab[q] == (int)(own_w & LBL_MASK));   // none, or the own label
#pragma unroll
                        for (int r = 0; r < q; ++r) skip = skip | (lab[r] == lab[q]);
                        skip = skip | (interior & (lcq[q] <= P.seen[q]));   // seen[q] = -1: never
                        fmask |= (skip ? 0u : 1u) << q;
                    }
#endif
                    }
                }
#ifdef ST_LDS_PROBE   // diagnostics: a dependent chain of N extra LDS reads per compute step
                {
                    int x_ = 0;
#pragma unroll
                    for (int i_ = 0; i_ < ST_LDS_PROBE; ++i_) x_ = lds_ld(&s_abort + (x_ & 0x40000000));
                    asm volatile("" ::"v"(x_));
                }
#endif
#ifdef ST_VALU_PROBE   // diagnostics: a dependent chain of N extra VALU per compute step
                {
                    int x_ = L;
#pragma unroll
                    for (int i_ = 0; i_ < ST_VALU_PROBE; ++i_) asm volatile("v_add_u32 %0, %0, 1" : "+v"(x_));
                }
#endif
                bool twin_done = false;   // wave-uniform
                if constexpr (Cfg::QUAD) {
                // ---- quad lanes: lane r of the cell's quad evaluates the cell's r-th candidate (and, in a
                //      second pass only for cells with more than 4, its (r+4)-th); the quad's results are
                //      combined as the reference's check order would (strict '<', first minimum wins:
                //      cpu_lib/makelevelset3.cpp:94-99, 143-149) -- by a first-minimum reduction over the
                //      quad (ST_QMIN) or, with ST_QMIN=0, by DPP broadcasts applied in rank order.  A rank
                //      with no candidate never wins -- like a skipped check. ----
                    twin_done = true;
#ifdef ST_STEP_PROF
                    {
                        const unsigned long long t_ = clock64();
                        sp_c[1] += t_ - sp_t;
                        sp_t = t_;
                        ++sp_n[!__any(fmask != 0u) ? 0 : (__any(__popc(fmask) > 4u) ? 2 : 1)];
                    }
#endif
                    const f3 gx = st_gx(P, a, b, c);
                    const unsigned f1 = fmask & (fmask - 1u), f2 = f1 & (f1 - 1u), f3 = f2 & (f2 - 1u);
#if ST_QMIN
                    // Each lane evaluates its rank's candidate; a first-minimum reduction over the quad
                    // (two DPP butterflies) then gives every lane the winner, which is applied once.  Applying
                    // the ranks one by one with strict '<' (the reference) takes the FIRST candidate whose
                    // distance is the minimum, if it is below phi: the reduction keeps the earlier rank on
                    // ties and maps 'no candidate' and NaN distances (which never pass '<') to +inf, which
                    // never passes '<' either.  The winner's label is read back with its entry at write-back.
                    const int e0 = ent[0], e1_ = ent[1], e2 = ent[2], e3 = ent[3], e4 = ent[4], e5 = ent[5], e6 = ent[6];
                    auto eval_rank = [&](unsigned fr, float &key, int &e) {
                        const bool has = fr != 0u;
                        const int qa = has ? __builtin_ctz(fr) : 0;
                        // ent[qa] by a select tree on qa's bits over values, not the array (an indexed
                        // read of it became a private array promoted to LDS: 9 KB more per tile)
                        const int e1 = has ? st_sel7(qa, e0, e1_, e2, e3, e4, e5, e6) : e_own;   // no candidate: a valid entry
                        const float4 v3 = st_e<EB>(s_ent, e1, 2);
                        const float dd = ptd_wave(gx, st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)), st_xyz(v3),
                                                  v3.w);
                        key = (has && dd == dd) ? dd : __builtin_inff();
                        e = e1;
                        if (P.stats) n_evals += (L == 0) ? (unsigned long long)__popcll(__ballot(has)) : 0ull;   // (counted runs only)
                    };
                    const bool q_odd = qr & 1, q_hi = qr & 2;
                    if constexpr (Cfg::LPC == 2) {
                        // duo lanes: pass p evaluates ranks 2p (lane 0) and 2p + 1 (lane 1); the pair's first
                        // minimum (lane 1 gives way on ties) is applied after each pass with strict '<', so an
                        // earlier pass keeps ties -- the reference's check order, pass after pass
                        if (__any(fmask != 0u)) {
                            unsigned fr = fmask;   // the candidates not yet evaluated
                            do {
                                const unsigned fq = fr & (fr - 1u);
                                float key;
                                int e;
                                eval_rank(q_odd ? fq : fr, key, e);
                                const float kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0xB1, 0xf, 0xf, false));
                                const int ep = __builtin_amdgcn_mov_dpp(e, 0xB1, 0xf, 0xf, false);
                                const bool tp = (kp < key) | (q_odd & (kp == key));
                                key = tp ? kp : key;
                                e = tp ? ep : e;
                                const bool take = key < phi;
                                phi = take ? key : phi;
                                win = take ? e : win;
                                fr = fq & (fq - 1u);
                            } while (__any(fr != 0u));
                        }
                    } else {
                    auto quad_first_min = [&](float &key, int &e) {
                        // partner lane^1, then lane^2; the lane holding the later rank(s) gives way on ties
                        float kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0xB1, 0xf, 0xf, false));
                        int ep = __builtin_amdgcn_mov_dpp(e, 0xB1, 0xf, 0xf, false);
                        // (keys are never NaN: kp <= key is !(key < kp))
                        bool take = (kp < key) | (q_odd & (kp == key));
                        key = take ? kp : key;
                        e = take ? ep : e;
                        kp = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0x4E, 0xf, 0xf, false));
                        ep = __builtin_amdgcn_mov_dpp(e, 0x4E, 0xf, 0xf, false);
                        take = (kp < key) | (q_hi & (kp == key));
                        key = take ? kp : key;
                        e = take ? ep : e;
                    };
                    if (__any(fmask != 0u)) {
                        float key;
                        int e;
                        eval_rank((unsigned)st_sel4(qr, (int)fmask, (int)f1, (int)f2, (int)f3), key, e);
                        quad_first_min(key, e);
                        bool take = key < phi;
                        phi = take ? key : phi;
                        win = take ? e : win;
                        if (__any(__popc(fmask) > 4u)) {   // ranks 4 .. 6 (at most 7 candidates)
                            const unsigned f4 = f3 & (f3 - 1u), f5 = f4 & (f4 - 1u), f6 = f5 & (f5 - 1u);
                            eval_rank((unsigned)st_sel4(qr, (int)f4, (int)f5, (int)f6, 0), key, e);
                            quad_first_min(key, e);
                            take = key < phi;
                            phi = take ? key : phi;
                            win = take ? e : win;
                        }
                    }
                    }   // LPC == 4
#else
                    static_assert(Cfg::LPC == 4, "duo lanes: the first-minimum reduction only (ST_QMIN)");
                    auto eval_rank = [&](unsigned fr, float &d, int &t, int &e) {
                        const bool has = fr != 0u;
                        const int qa = has ? __builtin_ctz(fr) : 0;
                        int e1 = ent[0], t1 = lab[0];
#pragma unroll
                        for (int q = 1; q < 7; ++q) {   // static indices: no register-array indexing
                            e1 = (qa == q) ? ent[q] : e1;
                            t1 = (qa == q) ? lab[q] : t1;
                        }
                        e1 = has ? e1 : e_own;   // lanes without a candidate read a valid entry
                        const float4 v3 = st_e<EB>(s_ent, e1, 2);
                        const float dd = ptd_wave(gx, st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)), st_xyz(v3),
                                                  v3.w);
                        d = has ? dd : __builtin_nanf("");
                        t = t1;
                        e = e1;
                        n_evals += (L == 0) ? (unsigned long long)__popcll(__ballot(has)) : 0ull;
                    };
                    auto apply = [&](float d, int t, int e) {
                        const bool take = d < phi;
                        phi = take ? d : phi;
                        ct = take ? t : ct;
                        win = take ? e : win;
                    };
                    // lane k of each quad, broadcast (DPP quad_perm(k, k, k, k))
#define ST_QB(x, k) __builtin_amdgcn_mov_dpp((x), (k) * 0x55, 0xf, 0xf, false)
                    auto apply_quad = [&](float d, int t, int e, int nr) {
                        const int di = __float_as_int(d);
                        apply(__int_as_float(ST_QB(di, 0)), ST_QB(t, 0), ST_QB(e, 0));
                        if (nr > 1) apply(__int_as_float(ST_QB(di, 1)), ST_QB(t, 1), ST_QB(e, 1));
                        if (nr > 2) apply(__int_as_float(ST_QB(di, 2)), ST_QB(t, 2), ST_QB(e, 2));
                        if (nr > 3) apply(__int_as_float(ST_QB(di, 3)), ST_QB(t, 3), ST_QB(e, 3));
                    };
                    if (__any(fmask != 0u)) {
                        float d;
                        int t, e;
                        eval_rank(qr == 0 ? fmask : (qr == 1 ? f1 : (qr == 2 ? f2 : f3)), d, t, e);
                        apply_quad(d, t, e, 4);
                        if (__any(__popc(fmask) > 4u)) {   // ranks 4 .. 6 (at most 7 candidates)
                            const unsigned f4 = f3 & (f3 - 1u), f5 = f4 & (f4 - 1u), f6 = f5 & (f5 - 1u);
                            eval_rank(qr == 0 ? f4 : (qr == 1 ? f5 : (qr == 2 ? f6 : 0u)), d, t, e);
                            apply_quad(d, t, e, 3);
                        }
                    }
#undef ST_QB
#endif
                } else if constexpr (TWIN) {
                // ---- candidates in pairs: the cell lane takes the lowest remaining one, its twin
                //      the next; one ptd per lane per pass, applied in the reference check order
                //      (strict '<', first minimum wins: cpu_lib/makelevelset3.cpp:94-99, 143-149) ----
#ifdef ST_STEP_PROF
                { const unsigned long long t_ = clock64(); sp_c[1] += t_ - sp_t; sp_t = t_; }
                {
                    const unsigned mp_ = __popc(fmask);
                    if (!__any(mp_ != 0u)) ++sp_n[0];
                    else if (!__any(mp_ > 2u)) ++sp_n[1];
                    else ++sp_n[2];
                }
#endif
                // at most 2 candidates per cell (else the wave-wide compaction below balances them)
                if (__all(__popc(fmask) <= 2u)) {
                    twin_done = true;
                    const f3 gx = st_gx(P, a, b, c);
                    unsigned fm = cell_lane ? fmask : (fmask & (fmask - 1u));
                    if (__any(fm != 0u)) {
                        const bool has = fm != 0u;
                        const int qa = has ? __builtin_ctz(fm) : 0;
                        int e1 = ent[0], t1 = lab[0];
#pragma unroll
                        for (int q = 1; q < 7; ++q) {   // static indices: no register-array indexing
                            e1 = (qa == q) ? ent[q] : e1;
                            t1 = (qa == q) ? lab[q] : t1;
                        }
                        const float4 v3 = st_e<EB>(s_ent, e1, 2);
                        const float d1 = ptd_wave(gx, st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)), st_xyz(v3), v3.w);
                        n_evals += (L == 0) ? (unsigned long long)__popcll(__ballot(has)) : 0ull;
#ifdef ST_STEP_PROF
                        ++sp_n[3];
#endif
                        // the twin's distance, label and entry (lanes 32..63 -> 0..31)
                        const float d2 = __uint_as_float(
                            __builtin_amdgcn_permlane32_swap(__float_as_uint(d1), __float_as_uint(d1), false, false)[1]);
                        const int t2 = (int)__builtin_amdgcn_permlane32_swap((unsigned)t1, (unsigned)t1, false, false)[1];
                        const int e2 = (int)__builtin_amdgcn_permlane32_swap((unsigned)e1, (unsigned)e1, false, false)[1];
                        const bool has2 = (fm & (fm - 1u)) != 0u;   // (cell lane) the pair's second candidate
                        const bool take1 = has & (d1 < phi);
                        phi = take1 ? d1 : phi;
                        ct = take1 ? t1 : ct;
                        win = take1 ? e1 : win;
                        const bool take2 = has2 & (d2 < phi);
                        phi = take2 ? d2 : phi;
                        ct = take2 ? t2 : ct;
                        win = take2 ? e2 : win;
                    }
                } else {
                    fmask = cell_lane ? fmask : 0u;   // the compaction below lists each cell's pairs once
                }
                }
                if (!Cfg::QUAD && !twin_done) {
                // ---- at most one candidate per cell (the common case away from the surface):
                //      each cell lane evaluates its own, no compaction and no LDS exchange ----
                const bool single = __all(__popc(fmask) <= 1);
#ifdef ST_STEP_PROF
                if constexpr (!TWIN) {
                    { const unsigned long long t_ = clock64(); sp_c[1] += t_ - sp_t; sp_t = t_; }
                    if (single) ++sp_n[__any(fmask != 0u) ? 1 : 0];
                    else ++sp_n[2];
                }
#endif
                if (single) {
                    if (__any(fmask != 0u)) {
                        // the one candidate's entry and label by select trees (an if per slot compiled
                        // to exec-mask branches); lanes without one evaluate their own entry, unused
                        const bool has = fmask != 0u;
                        const int qa = __builtin_ctz(fmask | 0x80u);
                        const int e1 = has ? st_sel7(qa, ent[0], ent[1], ent[2], ent[3], ent[4], ent[5], ent[6]) : e_own;
                        const int t1 = st_sel7(qa, lab[0], lab[1], lab[2], lab[3], lab[4], lab[5], lab[6]);
                        const float4 v3 = st_e<EB>(s_ent, e1, 2);
                        const float d = ptd_wave(st_gx(P, a, b, c), st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)),
                                               st_xyz(v3), v3.w);
                        const bool take = has & (d < phi);
                        phi = take ? d : phi;
                        ct = take ? t1 : ct;
                        win = take ? e1 : win;
                    }
                    if (P.stats) n_evals += (L == 0) ? (unsigned long long)__popcll(__ballot(fmask != 0)) : 0ull;
                } else {
                // ---- compact (cell, candidate) pairs across the wave ----
                int total = 0;
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    const bool f = (fmask >> q) & 1u;
                    const unsigned long long m = __ballot(f);
                    const int pos = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    s_pd[w][f ? pos : 14 * ST_CPW + L] = (ent[q] << 9) | (q << 6) | L;
                    total += (int)__popcll(m);
                }
                // ---- evaluate (<= 112 pairs): one per lane, a second chain only if needed ----
                for (int k = L; k < total; k += 128) {
                    const int p1 = s_pd[w][k];
                    const bool has2 = k + 64 < total;
                    const int l1 = p1 & 63, e1 = p1 >> 9;
                    const f3 g1 = st_gx(P, h - (l1 & 7) - (ST_CLW * w + (l1 >> 3)), b0 + (l1 & 7),
                                        c0 + ST_CLW * w + (l1 >> 3));
                    if (__any(has2)) {
                        const int p2 = has2 ? s_pd[w][k + 64] : p1;
                        const int l2 = p2 & 63, e2 = p2 >> 9;
                        const f3 g2 = st_gx(P, h - (l2 & 7) - (ST_CLW * w + (l2 >> 3)), b0 + (l2 & 7),
                                            c0 + ST_CLW * w + (l2 >> 3));
                        float d1, d2;
                        const float4 v13 = st_e<EB>(s_ent, e1, 2), v23 = st_e<EB>(s_ent, e2, 2);
                        ptd_wave2(g1, st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)), st_xyz(v13), v13.w, g2,
                                  st_xyz(st_e<EB>(s_ent, e2, 0)), st_xyz(st_e<EB>(s_ent, e2, 1)), st_xyz(v23), v23.w, d1, d2);
                        s_pd[w][7 * ST_CPW + ((p1 >> 6) & 7) * ST_CPW + l1] = __float_as_int(d1);
                        s_pd[w][7 * ST_CPW + (has2 ? ((p2 >> 6) & 7) * ST_CPW + l2 : 7 * ST_CPW + L)] = __float_as_int(d2);
                    } else {
                        s_pd[w][7 * ST_CPW + ((p1 >> 6) & 7) * ST_CPW + l1] = __float_as_int(
                            ptd_wave(g1, st_xyz(st_e<EB>(s_ent, e1, 0)), st_xyz(st_e<EB>(s_ent, e1, 1)), st_xyz(st_e<EB>(s_ent, e1, 2)),
                                     st_e<EB>(s_ent, e1, 2).w));
                    }
                }
                n_evals += (L == 0) ? (unsigned long long)total : 0ull;
#ifdef ST_STEP_PROF
                if constexpr (!TWIN) sp_n[3] += (unsigned long long)total;
#endif
                // ---- apply in the reference check order: strict '<', first minimum wins ----
                if (act) {   // branch-free: all 7 slots read at once, non-candidates masked out
                    float dq[7];
#pragma unroll
                    for (int q = 0; q < 7; ++q) dq[q] = __int_as_float(s_pd[w][7 * ST_CPW + q * ST_CPW + L]);
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
#if ST_GVMASK
                        // a slot that is not a candidate reads as +inf, which never passes '<' (one compare,
                        // no mask to combine on the scalar unit)
                        const uint32_t cm = 0u - ((fmask >> q) & 1u);
                        const float dv = __uint_as_float((__float_as_uint(dq[q]) & cm) | (0x7f800000u & ~cm));
                        const bool take = dv < phi;
#else
                        const bool take = ((fmask >> q) & 1u) && dq[q] < phi;
                        const float dv = dq[q];
#endif
                        phi = take ? dv : phi;
                        ct = take ? lab[q] : ct;
                        win = take ? ent[q] : win;
                    }
                }
                }
                }   // !twin_done
#ifdef ST_STEP_PROF
                { const unsigned long long t_ = clock64(); sp_c[2] += t_ - sp_t; sp_ev[twin_done ? 0 : 1] += t_ - sp_t; sp_t = t_; }
#endif
                if (act) {
                    const int src = win < 0 ? e_own : win;
                    const float4 w0 = st_e<EB>(s_ent, src, 0);
                    const float4 w1 = st_e<EB>(s_ent, src, 1), w2 = st_e<EB>(s_ent, src, 2);
                    const int slot = __umul24(ST_RING0 + am * ST_NCOL + col_id, ES);
                    // a winner always carries a new label (the own label is never a candidate); quad
                    // tiles (ST_QMIN) take it from the winner's entry, the word its candidate test read
                    const uint32_t w_new = win < 0 ? own_w
                                           : (Cfg::QUAD && ST_QMIN) ? lo_word((int)(__float_as_uint(w0.w) & LBL_MASK), P.sweep + 1)
                                                                    : lo_word(ct, P.sweep + 1);
                    st_e<EB>(s_ent, slot, 0) = make_float4(w0.x, w0.y, w0.z, __uint_as_float(w_new));
                    st_e<EB>(s_ent, slot, 1) = w1;
                    st_e<EB>(s_ent, slot, 2) = w2;
                    if (win >= 0 && ST_DIAG_SPLIT != 1)
                        P.cell[SDF_CHK(5, st_phys(P, a, b, c), P.clo, P.chi)] =
                            ((unsigned long long)__float_as_uint(phi) << 32) | w_new;
                    const unsigned long long gran = st_granule(P.epoch, w_new);
                    if (bl == ST_T - 1 && J < P.nJ - 1)
                        __hip_atomic_store(P.hb + ((size_t)J * P.hbC + (c - P.cs)) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                    if (cl == ST_T - 1 && K < P.nK - 1)
                        __hip_atomic_store(P.hc + ((size_t)K * P.B + b) * P.A + a, gran, __ATOMIC_RELAXED, GSCOPE);
                    if (SLAB && P.hc_out && c == P.ce - 1)
                        __hip_atomic_store(P.hc_out + st_inbox(P, a, b), gran, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                }
                }   // LPC != 8
                if (TRACE && P.trace) {
                    t_comp += wall_clock64() - tc0;
                    c_comp += clock64() - cc0;
                }
                lds_drain();
                if (L == 0) lds_st(&s_hdr[1 + w], h + 1);
#ifdef ST_STEP_PROF
                sp_c[3] += clock64() - sp_t;
#endif
                if (TRACE && P.trace && w == 0 && L == 0 && (h == 0 || h == (MULTI ? 8 : nsteps / 2)))
                    P.trace[8 * task + (h == 0 ? 1 : (MULTI ? 5 : 2))] = wall_clock64();   // MULTI: [5] = step 8 done
            }
            __builtin_amdgcn_s_setprio(0);
#ifdef ST_STEP_PROF
            if (P.stats && L == 0) {
                for (int i_ = 0; i_ < 4; ++i_) atomicAdd(P.stats + 4 + i_, sp_c[i_]);
                for (int i_ = 0; i_ < 4; ++i_) atomicAdd(P.stats + 8 + i_, sp_n[i_]);
                atomicAdd(P.stats + 12, sp_ev[0]);
                atomicAdd(P.stats + 13, sp_ev[1]);
                atomicAdd(P.stats + 14, sp_pw[0]);
                atomicAdd(P.stats + 15, sp_pw[1] | (sp_pw[2] << 32));
            }
#endif
            if (TRACE && P.trace && w == 0 && L == 0) {
                P.trace[8 * task + 3] = wall_clock64();
                if (!MULTI) {
                    P.trace[8 * task + 4] = t_wait;
                    P.trace[8 * task + 5] = w_own + (w_halo << 32);
                }
                if (MULTI) {
                    P.trace[8 * task + 6] = ((unsigned long long)P0.mtasks[task].z << 32) | ((unsigned)J << 16) | (unsigned)K;
                    P.trace[8 * task + 7] = t_claim;
                } else {
                    P.trace[8 * task + 6] = c_comp;
                    P.trace[8 * task + 7] = t_comp;
                }
            }
        } else {
            // ======================= helper wave(s) =======================
            // ROLE 0: the one helper wave (own data and halo); with Cfg::NH == 2 the first helper wave takes ROLE 1
            // (own columns only) and the second ROLE 2 (halo streams only): each round trip then carries half the
            // loads, and neither kind waits behind the other's gathers.  (A constant 0 with one helper: the role
            // tests fold away and the code is the one-helper loop instruction for instruction -- a lambda per role
            // cost the default build 2 % in register allocation, round 5.)
            const int ROLE = Cfg::NH == 1 ? 0 : (wave == ST_NCW ? 1 : 2);
            if (ST_HELPER_PRIO) __builtin_amdgcn_s_setprio(ST_HELPER_PRIO);
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            const int bl = L & (ST_T - 1), cl = L >> 3;   // helper lane L prefetches column (bl, cl)
            const int b = b0 + bl, c = c0 + cl;
            const bool col = ROLE != 2 && b < P.B && c < P.ce;
            // stream geometry (lanes < 17)
            const bool hlane = ROLE != 1 && L < ST_NSTREAM;
            int hbs = 0, hcs = 0, hoff = 0;
            bool hvalid = false, hbound = true;
            const unsigned long long *hsrc = nullptr;
            if (hlane) {
                if (L < ST_T) {
                    hbs = b0 - 1; hcs = c0 + L; hoff = L; hvalid = hcs < P.ce; hbound = (J == 0);
                    if (!hbound) hsrc = P.hb + ((size_t)(J - 1) * P.hbC + (hcs - P.cs)) * P.A;
                } else if (L < 2 * ST_T) {
                    hbs = b0 + (L - ST_T); hcs = c0 - 1; hoff = L - ST_T; hvalid = hbs < P.B;
                    hbound = (K == 0) && !inbox;
                    if (inbox) hsrc = P.hc_in + st_inbox(P, 0, hbs);
                    else if (!hbound) hsrc = P.hc + ((size_t)(K - 1) * P.B + hbs) * P.A;
                } else {
                    hbs = b0 - 1; hcs = c0 - 1; hoff = 0; hvalid = true;
                    hbound = (J == 0 || K == 0) && !inbox;
                    if (inbox) hsrc = P.hc_in + st_inbox(P, 0, hbs);
                    else if (!hbound) hsrc = P.hb + ((size_t)(J - 1) * P.hbC + (hcs - P.cs)) * P.A;
                }
            }
            if (!hvalid || hbound) hsrc = P.hb;   // any valid address: unused lanes load harmlessly
            // Two-stage software pipeline, one global round trip per iteration:
            //   stage 1 (batch B): the columns' old cells and the halo granules;
            //   stage 2 (batch A, loaded last iteration): gather the labels' vertices,
            //   land them in LDS and publish readiness.
            // All loads are unconditional (invalid slots read a clamped address and are
            // ignored), so hipcc's waitcnt pass can count them and waits for the stage-2
            // gathers only, leaving the younger stage-1 loads in flight.
            // unused load slots read the tile's first column start: one cached line per tile, so
            // not one hot address for the chip, and inside the slab (a Z-slab holds only its own
            // planes: (0, 0, 0) may lie in another GPU's slab).  (b0, c0: the tile's corner,
            // before the batch registers below shadow the name c0.)
            // (one line for the whole wave: a per-lane dummy -- each lane its own column start, 47
            // non-halo lanes' granule slots among them -- cost every load instruction up to 64 line
            // requests; one shared line took the first pass 14.2 -> 13.9 ms at 256^3, 53.9 -> 51.6
            // ms at 512^3)
            const size_t dummy = st_phys(P, 0, b0, c0);
            // gathers with nothing to fetch read a per-tile triangle: triangle 0 for every tile was one
            // hot line for the whole chip (first pass 14.0 -> 13.9 ms at 256^3, 51.4 -> 50.6 ms at 512^3)
            // (0 when the triangle count is unknown: ntri is ~0 until a pipeline sets it)
            const int gdum = (P.ntri >= 1 && P.ntri < 0x7fffffffull) ? (int)((unsigned)(J * 40503 + K * 9973 + 17) % (unsigned)P.ntri) : 0;
            int fA = ROLE == 2 ? nsteps : 0, gA = 0;   // own steps [fA, fA+gA) whose cells are in c0..c3 (ROLE 2: none)
            // ST_CWA: the own steps' cell words run ahead of the gathers -- [fA, fCl) are in s_cw, [fCl, fCl + gCl)
            // in flight in c0..c3; gA is then the batch gathered in this iteration
            int fCl = fA, gCl = 0;
            int hA = hvalid ? 0 : P.A, hcA = 0;    // halo entries [hA, hA+hcA) whose granules are in q0..q3
            unsigned long long c0 = ~0ull, c1 = ~0ull, c2 = ~0ull, c3 = ~0ull;   // ST_G == 4 (named, never an array:
            unsigned long long q0 = 0, q1 = 0, q2 = 0, q3 = 0;                 //  arrays here landed in scratch)
            static_assert(ST_G == 4 || ST_G == 2, "helper pipeline is written out for 2- or 4-element batches");
            unsigned idle = 0;
            unsigned long long t_idle = 0;   // Z-slab: wall ticks this helper spent backing off (TM_*)
#ifdef ST_STEP_PROF   // helper iterations that landed data: count, cycles (since the previous one), own steps, halo lanes
            unsigned long long hp_n = 0, hp_cyc = 0, hp_own = 0, hp_halo = 0, hp_t0 = 0;
#endif
            bool tr_halo = false, tr_own = false;   // TRACE + MULTI: first landings recorded
            for (;;) {
                // Ring capacity follows the slowest compute wave.  Not simply the last one: wave w
                // may finish step h while wave w-1 is still on step h (it needs only h-1 of it).
                int prog = lds_ld(&s_hdr[1]);
#pragma unroll
                for (int w = 1; w < ST_NCW; ++w) prog = min(prog, lds_ld(&s_hdr[1 + w]));
                if (lds_ld(&s_abort)) break;
                if (idle && (ST_CWA ? gCl : gA) == 0 && hcA == 0) {
                    // Nothing in flight and the last round found nothing to do: wait cheaply (LDS
                    // progress, at most one granule probe per halo lane) instead of running the
                    // whole pipeline body on dummy loads -- idle helpers steal VALU issue slots
                    // from the compute waves sharing their SIMD.
                    if (__all(fA >= nsteps && hA >= P.A)) break;
                    const int own_n = min(ST_G, min(nsteps - fA, min(prog + ST_RO - fA, ST_CWA ? fCl - fA : ST_G)));
                    const int halo_n = hvalid ? min(ST_G, min(P.A - hA, prog + ST_RH - hoff - 2 - hA)) : 0;
                    bool go = own_n > 0 || (ST_CWA && fCl < min(nsteps, fA + ST_RC));
                    if (halo_n > 0)
                        go = go || hbound ||
                             st_granule_ready(__hip_atomic_load(hsrc + hA, __ATOMIC_RELAXED, GSCOPE), P.epoch);
                    if (!__any(go)) {
                        ++n_hpoll;
                        if (++idle > ST_WATCHDOG || ((idle & 255u) == 0u && st_failed(P))) {
                            if (L == 0) { lds_st(&s_abort, 1); st_fail(P, 16); }   // 16: a helper gave up
                            break;
                        }
                        const unsigned long long ts = (SLAB && P.tm) ? wall_clock64() : 0ull;
                        if (idle < 4) __builtin_amdgcn_s_sleep(1);
                        else if (idle < 16) __builtin_amdgcn_s_sleep(4);
                        else __builtin_amdgcn_s_sleep(ST_HSLEEP);
                        if (SLAB && P.tm) t_idle += wall_clock64() - ts;
                        continue;
                    }
                }
                // The batch-A loads were issued one iteration ago: wait for them once, and hand
                // the registers back through the asm so the compiler does not track them as
                // pending (its per-use waits would otherwise serialise the gathers below).
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(q0), "+v"(q1),
                             "+v"(q2), "+v"(q3)::"memory");
#if ST_CWA
                // the cell words that landed go to their slots; batch A = the next own steps with a word and a
                // free own slot (a wave-uniform count), its words read back from LDS
                if (0 < gCl) s_cw[(fCl & (ST_RC - 1)) * ST_NCOL + L] = c0;
                if (1 < gCl) s_cw[((fCl + 1) & (ST_RC - 1)) * ST_NCOL + L] = c1;
#if ST_G_DEF > 2
                if (2 < gCl) s_cw[((fCl + 2) & (ST_RC - 1)) * ST_NCOL + L] = c2;
                if (3 < gCl) s_cw[((fCl + 3) & (ST_RC - 1)) * ST_NCOL + L] = c3;
#endif
                fCl += gCl;
                gA = max(0, min(ST_G, min(nsteps - fA, min(prog + ST_RO - fA, fCl - fA))));
                const unsigned long long u0 = s_cw[(fA & (ST_RC - 1)) * ST_NCOL + L],
                                         u1 = s_cw[((fA + 1) & (ST_RC - 1)) * ST_NCOL + L];
#if ST_G_DEF > 2
                const unsigned long long u2 = s_cw[((fA + 2) & (ST_RC - 1)) * ST_NCOL + L],
                                         u3 = s_cw[((fA + 3) & (ST_RC - 1)) * ST_NCOL + L];
#endif
#define ST_OWNW(g) u##g
#else
#define ST_OWNW(g) c##g
#endif
                // ---- stage 2: vertices for batch A ----
                int hp = 0;   // ready prefix of the halo batch (tag == epoch; boundary planes always)
                const bool r0 = hbound || st_granule_ready(q0, P.epoch);
                const bool r1 = hbound || st_granule_ready(q1, P.epoch);
                const bool r2 = hbound || st_granule_ready(q2, P.epoch);
                const bool r3 = hbound || st_granule_ready(q3, P.epoch);
                if (0 < hcA && r0) { hp = 1; if (1 < hcA && r1) { hp = 2; if (2 < hcA && r2) { hp = 3; if (3 < hcA && r3) hp = 4; } } }
#define ST_OWN_OK(g) ((g) < gA && col && fA + (g) - bl - cl >= 0 && fA + (g) - bl - cl < P.A)
// (the role tests are conditional operators on ROLE, a constant with one helper wave: clang emits only the
// live arm, so the one-helper code is the original's instruction for instruction)
// (exec-masking the gathers and stage-1 loads to the lanes that use them instead of a dummy read in every lane
// measured slower: C3 first pass 10.5 -> 13.6 ms, C4 38.6 -> 42.0 ms)
#define ST_GATHER_O(g, cg)                                                                             \
    const size_t so##g = 3 * SDF_CHK(11, (ST_DIAG_SPLIT != 2 && ST_OWN_OK(g) && lbl_of((uint32_t)(cg)) >= 0 ? lbl_of((uint32_t)(cg)) : gdum), 0, P.ntri); \
    const float4 oa##g = ROLE != 2 ? P.soup[so##g] : z4, ob##g = ROLE != 2 ? P.soup[so##g + 1] : z4,    \
                 oc##g = ROLE != 2 ? P.soup[so##g + 2] : z4;
#define ST_GATHER_H(g, qg)                                                                             \
    const size_t sh##g = 3 * SDF_CHK(12, (ST_DIAG_SPLIT != 3 && (g) < hp && lbl_of((uint32_t)(qg)) >= 0 ? lbl_of((uint32_t)(qg)) : gdum), 0, P.ntri); \
    const float4 ha##g = ROLE != 1 ? P.soup[sh##g] : z4, hb##g = ROLE != 1 ? P.soup[sh##g + 1] : z4,    \
                 hc##g = ROLE != 1 ? P.soup[sh##g + 2] : z4;
#if ST_HALO_FIRST
                // the halo batch's gathers first: its landing then waits for them alone (loads return in order)
                ST_GATHER_H(0, q0)
                ST_GATHER_H(1, q1)
#if ST_G_DEF > 2
                ST_GATHER_H(2, q2)
                ST_GATHER_H(3, q3)
#endif
                ST_GATHER_O(0, ST_OWNW(0))
                ST_GATHER_O(1, ST_OWNW(1))
#if ST_G_DEF > 2
                ST_GATHER_O(2, ST_OWNW(2))
                ST_GATHER_O(3, ST_OWNW(3))
#endif
#else
                ST_GATHER_O(0, ST_OWNW(0))
                ST_GATHER_H(0, q0)
                ST_GATHER_O(1, ST_OWNW(1))
                ST_GATHER_H(1, q1)
#if ST_G_DEF > 2
                ST_GATHER_O(2, ST_OWNW(2))
                ST_GATHER_H(2, q2)
                ST_GATHER_O(3, ST_OWNW(3))
                ST_GATHER_H(3, q3)
#endif
#endif
                // ---- stage 1: issue batch B (ST_CWA: the cell words of own steps [fI, fI + gI), up to ST_RC
                //      steps past batch A) and the halo granules ----
                const int fB = fA + gA;
#if ST_CWA
                const int fI = fCl, gI = max(0, min(ST_G, min(nsteps - fI, fB + ST_RC - fI)));
#else
                const int fI = fB, gI = max(0, min(ST_G, min(nsteps - fB, prog + ST_RO - fB)));
#endif
                const int hB = hA + hp;
                int hcB = 0;
                if (hvalid) {
                    hcB = min(ST_G, min(P.A - hB, prog + ST_RH - hoff - 2 - hB));
                    if (hcB < 0) hcB = 0;
                }
#define ST_ISSUE(g, cn, qn)                                                                            \
    {                                                                                                  \
        const int a_ = fI + (g) - bl - cl;                                                             \
        const bool ok_ = (g) < gI && col && a_ >= 0 && a_ < P.A;                                       \
        const size_t ix_ = (ok_ && ST_DIAG_SPLIT != 4) ? st_phys(P, a_, b, c) : dummy;                 \
        cn = ROLE != 2 ? P.cell[SDF_CHK(6, ix_, P.clo, P.chi)] : ~0ull;                                \
        const unsigned long long *src_ =                                                               \
            (g) >= hcB ? P.cell + SDF_CHK(7, dummy, P.clo, P.chi)                                      \
                       : (hbound ? P.cell + SDF_CHK(10, st_phys(P, hB + (g), hbs, hcs), P.clo, P.chi) : hsrc + hB + (g)); \
        qn = ROLE != 1 ? __hip_atomic_load(src_, __ATOMIC_RELAXED, GSCOPE) : 0ull;                     \
    }
                // Always issued (a fixed count keeps the waits below precise); slots with nothing
                // to fetch read a cached dummy, and idle helpers back off, so waiting tiles do
                // not flood the fabric with granule polls.
                unsigned long long n0, n1, n2, n3, m0, m1, m2, m3;
                ST_ISSUE(0, n0, m0)
                ST_ISSUE(1, n1, m1)
#if ST_G_DEF > 2
                ST_ISSUE(2, n2, m2)
                ST_ISSUE(3, n3, m3)
#else
                n2 = n3 = ~0ull;
                m2 = m3 = 0ull;
#endif
#ifdef ST_HALO_DELAY   // diagnostics: the first pass's sensitivity to the tile-hop latency
                if (__any(hp > 0)) __builtin_amdgcn_s_sleep(ST_HALO_DELAY);
#endif
                // ---- land batch A in LDS, then publish readiness ----
#define ST_LAND_O(g, cg)                                                                               \
    if (ST_OWN_OK(g)) {                                                                                \
        const int e_ = ST_OWN0 + ((fA + (g) - bl - cl) & (ST_RO - 1)) * ST_NCOL + LR;                  \
        s_ent[3 * e_] = make_float4(oa##g.x, oa##g.y, oa##g.z, __uint_as_float((uint32_t)(cg)));      \
        s_ent[3 * e_ + 1] = make_float4(ob##g.x, ob##g.y, ob##g.z, __uint_as_float((uint32_t)((cg) >> 32))); \
        s_ent[3 * e_ + 2] = oc##g;                                                                     \
    }
#define ST_LAND_H(g, qg)                                                                               \
    if ((g) < hp) {                                                                                    \
        const int e_ = ST_HALO0 + LR * ST_RH + ((hA + (g)) & (ST_RH - 1));                             \
        s_ent[3 * e_] = make_float4(ha##g.x, ha##g.y, ha##g.z, __uint_as_float((uint32_t)(qg)));      \
        s_ent[3 * e_ + 1] = hb##g;                                                                     \
        s_ent[3 * e_ + 2] = hc##g;                                                                     \
    }
                const int LR = ST_LANE_REMAT ? st_lane_remat() : L;   // (== L)
#if ST_HALO_FIRST
                // the halo entries land and are published as soon as their gathers are back (the tile hop is
                // on the critical path: DESIGN.md §6), then the own entries
                ST_LAND_H(0, q0)
                ST_LAND_H(1, q1)
#if ST_G_DEF > 2
                ST_LAND_H(2, q2)
                ST_LAND_H(3, q3)
#endif
                lds_drain();
                if (hvalid && hp) lds_st(&s_halo_ready[LR], hB);
                ST_LAND_O(0, ST_OWNW(0))
                ST_LAND_O(1, ST_OWNW(1))
#if ST_G_DEF > 2
                ST_LAND_O(2, ST_OWNW(2))
                ST_LAND_O(3, ST_OWNW(3))
#endif
                lds_drain();
                if (L == 0 && gA) lds_st(&s_hdr[0], fB);
#else
                ST_LAND_O(0, ST_OWNW(0))
                ST_LAND_H(0, q0)
                ST_LAND_O(1, ST_OWNW(1))
                ST_LAND_H(1, q1)
#if ST_G_DEF > 2
                ST_LAND_O(2, ST_OWNW(2))
                ST_LAND_H(2, q2)
                ST_LAND_O(3, ST_OWNW(3))
                ST_LAND_H(3, q3)
#endif
                lds_drain();
                if (L == 0 && gA) lds_st(&s_hdr[0], fB);
                if (hvalid && hp) lds_st(&s_halo_ready[LR], hB);
#endif
#undef ST_OWNW
#undef ST_OWN_OK
#undef ST_GATHER_O
#undef ST_GATHER_H
#undef ST_ISSUE
#undef ST_LAND_O
#undef ST_LAND_H
                if (TRACE && MULTI && P.trace) {   // [2] first halo entries landed, [4] first own entries landed
                    const bool h_now = __any(hvalid && hp > 0 && L < ST_T), o_now = gA > 0;   // b-edge streams (from J - 1)
                    if (h_now && !tr_halo && L == 0) P.trace[8 * task + 2] = wall_clock64();
                    if (o_now && !tr_own && L == 0) P.trace[8 * task + 4] = wall_clock64();
                    tr_halo |= h_now;
                    tr_own |= o_now;
                }
                const bool moved = gA > 0 || hp > 0 || gI > 0;   // a halo poll that lands nothing is idle
#ifdef ST_STEP_PROF
                if (P.stats && __any(moved)) {
                    const unsigned long long t_ = clock64();
                    if (hp_t0) {
                        hp_n += 1;
                        hp_cyc += t_ - hp_t0;
                        hp_own += (unsigned long long)gA;
                        hp_halo += (unsigned long long)__popcll(__ballot(hp > 0)) ;
                    }
                    hp_t0 = t_;
                }
#endif
                fA = fB; hA = hB; hcA = hcB;
                if (ST_CWA) gCl = gI; else gA = gI;
                c0 = n0; c1 = n1; c2 = n2; c3 = n3;
                q0 = m0; q1 = m1; q2 = m2; q3 = m3;
                if (__all(fB >= nsteps && (ST_CWA || gI == 0) && hB >= P.A)) break;
                if (__any(moved)) {
                    idle = 0;
                } else {
                    // back off (64..1024 cycles): hundreds of waiting tiles must not flood the
                    // memory system with granule polls (MI355X_MICROARCH.md polling-cost)
                    ++n_hpoll;
                    if (++idle > ST_WATCHDOG || ((idle & 255u) == 0u && st_failed(P))) {
                        if (L == 0) { lds_st(&s_abort, 1); st_fail(P, 16); }
                        break;
                    }
                    const unsigned long long ts = (SLAB && P.tm) ? wall_clock64() : 0ull;
                    if (idle < 4) __builtin_amdgcn_s_sleep(1);
                    else if (idle < 16) __builtin_amdgcn_s_sleep(4);
                    else __builtin_amdgcn_s_sleep(ST_HSLEEP);
                    if (SLAB && P.tm) t_idle += wall_clock64() - ts;
                }
            }
#ifdef ST_STEP_PROF
            if (P.stats && L == 0) {
                atomicAdd(P.stats + 16, hp_n);
                atomicAdd(P.stats + 17, hp_cyc);
                atomicAdd(P.stats + 18, hp_own);
                atomicAdd(P.stats + 19, hp_halo);
            }
#endif
            if (SLAB && P.tm && L == 0 && ROLE != 1) {   // where the slab boundary's tiles wait for the upstream GPU
                atomicAdd(P.tm + (inbox ? TM_INBOX_IDLE : TM_OTHER_IDLE), t_idle);
                atomicAdd(P.tm + (inbox ? TM_INBOX_TASKS : TM_OTHER_TASKS), 1ull);
            }
        }
        if (MULTI) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's cell stores done
        __syncthreads();
        if (MULTI && tid == 0) {   // ... then one release and the flag (MI355X_MICROARCH.md visibility)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(P0.done + task, P0.call_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (P.stats && L == 0) {
        if (n_evals) atomicAdd(P.stats, n_evals);
        if (n_cpoll) atomicAdd(P.stats + 1, n_cpoll);
        if (n_hpoll) atomicAdd(P.stats + 2, n_hpoll);
        if (n_cpoll_own) atomicAdd(P.stats + 3, n_cpoll_own);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

struct TileSweepWorkspace {
    unsigned long long *hb = nullptr, *hc = nullptr, *stats = nullptr, *trace = nullptr;
    size_t cap_trace = 0;
    int trace_sweep = -1;      // which sweep (0..15) to trace, -1 = none
    bool trace_multi = false;  // trace every task of the one-launch first pass (diagnostics)
    int cur_sweep = 0;
    int grid_override = 0;     // diagnostics: cap on resident workgroups
    int share = 1;             // slab sessions sharing this device (st_share_grid caps the grid when > 1)
    int lead_override = -1;    // diagnostics: smaller inter-wave lead (>= 0)
    bool skip_seen = true;     // the "already examined" skip (diagnostics can turn it off)
    unsigned long long clo = 0, chi = ~0ull, ntri = ~0ull;   // address bounds for bounds-checked builds
    unsigned long long *tm = nullptr;   // Z-slab phase timers (owned by the slab session; null: none)
    size_t cap_hb = 0, cap_hc = 0;
    // task tables (dequeue order) for up to two tile grids: a Z-slab alternates between
    // two c extents (k-up and k-down sweeps), and a table must not be rewritten while a
    // kernel still on the stream reads it
    int2 *tasks[2] = {nullptr, nullptr};
    size_t cap_tasks[2] = {0, 0};
    int task_nJ[2] = {-1, -1}, task_nK[2] = {-1, -1};
    int task_next = 0;
    int *ctrl = nullptr;   // [0] queue counter, [1] error bits
    unsigned epoch = 0;
    bool count = false;
    // MULTI launches (tile_sweep_multi): per-sweep halo buffers, task graph, completion flags
    unsigned long long *mhb = nullptr, *mhc = nullptr;
    size_t cap_mhb = 0, cap_mhc = 0;
    int4 *mtasks = nullptr;
    int *mdeps = nullptr;
    unsigned *mdone = nullptr;
    size_t cap_mtasks = 0;
    long long mkey = -1;   // (ni, nj, nk, first sweep, count) of the uploaded graph
    double chain_steps = 0.0;   // modelled critical path of that graph, in steps
    int cfg = ST_CFG_LAT;       // the last multi-sweep launch's tile configuration (ST_CFG_*)
    unsigned mepoch = 0;
    int last_ntasks = 0;        // tasks of the last multi-sweep launch (watchdog report) ...
    int last_A = 0, last_B = 0, last_nJ = 0, last_ns = 0, last_nK[ST_MAXSW] = {0}, last_hbC[ST_MAXSW] = {0};
    size_t last_nhb = 0, last_nhc = 0;
};

inline bool tile_sweep_supported(int ni, int nj, int nk) { return ni >= 2 && nj >= 2 && nk >= 2; }

// Memsets and uploads of these helpers go on the caller's stream (then, where the host data
// dies, a sync of THAT stream): a synchronous hipMemset/hipMemcpy was measured to block until
// other streams' kernels finished -- with Z-slabs driven from one thread those kernels wait on
// the very slab being set up.
// Returns 0, or -5 / -4 with the failing status in sdf_last_hip (a sticky fault of an earlier kernel
// fails the hipFree or hipMalloc here with that fault's name, not as an allocation failure).
inline int st_grow(unsigned long long **p, size_t *cap, size_t need, hipStream_t st)
{
    if (*p && *cap >= need) return 0;
    if (*p) {
        const hipError_t e = hipFree(*p);
        *p = nullptr;
        *cap = 0;
        if (e != hipSuccess) return sdf_hip_rc(e);
    }
    *p = nullptr;
    *cap = 0;
    if (hipError_t e = hipMalloc((void **)p, need * sizeof(unsigned long long)); e != hipSuccess) {
        *p = nullptr;
        return sdf_hip_rc(e);
    }
    // tags are epochs >= 1: zeroed granules can never look published
    if (hipError_t e = hipMemsetAsync(*p, 0, need * sizeof(unsigned long long), st); e != hipSuccess) return sdf_hip_rc(e);
    *cap = need;
    return 0;
}
// Drain the stream before a buffer it may still read is replaced; a failed earlier kernel shows here.
inline int st_sync(hipStream_t st)
{
    const hipError_t e = hipStreamSynchronize(st);
    return e == hipSuccess ? 0 : sdf_hip_rc(e);
}
// "GPU tile sweep: <what>: <HIP status>" (every set-up failure names the runtime's status)
inline int st_fail_msg(char *err, size_t errlen, int code, const char *what)
{
    if (err && errlen) {
        if (code == -4 || code == -5) snprintf(err, errlen, "GPU tile sweep: %s: %s", what, sdf_last_hip_name());
        else snprintf(err, errlen, "GPU tile sweep: %s", what);
    }
    return code;
}

// Z-slab part of one sweep: oriented c range of this slab and its inboxes.
struct TileSlab {
    bool on = false;
    int cs = 0, ce = 0;                       // this slab's oriented c range
    const unsigned long long *in = nullptr;   // inbox: plane cs-1 from the upstream slab (null: first)
    unsigned long long *out = nullptr;        // downstream slab's inbox for plane ce-1 (null: last)
};

// Buffers and the task table of one sweep over oriented c in [cs, ce).  Growing a buffer or
// replacing a task table synchronises the stream (a running launch may still use the old one).
// *ti: the task table slot.  Returns 0 or a negative SDFGEN_HIP_E* code.
inline int st_prepare(TileSweepWorkspace &W, hipStream_t st, int ni, int nj, int cs, int ce, int *ti_out)
{
    const int A = ni - 1, B = nj - 1;
    const int nJ = (B + ST_T - 1) / ST_T, nK = (ce - cs + ST_T - 1) / ST_T;
    const int ntasks = nJ * nK;
    const size_t nhb = (size_t)nJ * (ce - cs) * A;
    if (W.cap_hb < nhb || W.cap_hc < (size_t)nK * B * A)
        if (int rc = st_sync(st)) return rc;
    if (int rc = st_grow(&W.hb, &W.cap_hb, nhb, st)) return rc;
    if (int rc = st_grow(&W.hc, &W.cap_hc, (size_t)nK * B * A, st)) return rc;
    if (!W.ctrl) {
        if (hipError_t e = hipMalloc((void **)&W.ctrl, 16 * sizeof(int)); e != hipSuccess) return sdf_hip_rc(e);
        if (hipError_t e = hipMalloc((void **)&W.stats, ST_NSTATS * sizeof(unsigned long long)); e != hipSuccess) return sdf_hip_rc(e);
        if (hipError_t e = hipMemsetAsync(W.ctrl, 0, 16 * sizeof(int), st); e != hipSuccess) return sdf_hip_rc(e);
    }
    int ti = (W.task_nJ[0] == nJ && W.task_nK[0] == nK) ? 0 : (W.task_nJ[1] == nJ && W.task_nK[1] == nK) ? 1 : -1;
    if (ti < 0) {
        ti = W.task_next;
        W.task_next ^= 1;
        if (int rc = st_sync(st)) return rc;   // the slot being replaced may still be read by a running launch
        std::vector<int2> t;
        t.reserve(ntasks);
        for (int d = 0; d <= nJ + nK - 2; ++d)
            for (int J = 0; J < nJ; ++J) {
                const int K = d - J;
                if (K >= 0 && K < nK) t.push_back(make_int2(J, K));
            }
        if ((size_t)ntasks > W.cap_tasks[ti]) {
            if (W.tasks[ti]) (void)hipFree(W.tasks[ti]);
            W.tasks[ti] = nullptr;
            W.cap_tasks[ti] = 0;
            if (hipError_t e = hipMalloc((void **)&W.tasks[ti], std::max(ntasks, 1) * sizeof(int2)); e != hipSuccess) {
                W.tasks[ti] = nullptr;
                return sdf_hip_rc(e);
            }
            W.cap_tasks[ti] = std::max(ntasks, 1);
        }
        if (ntasks) {
            hipError_t e = hipMemcpyAsync(W.tasks[ti], t.data(), ntasks * sizeof(int2), hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return sdf_hip_rc(e);
        }
        W.task_nJ[ti] = nJ;
        W.task_nK[ti] = nK;
    }
    *ti_out = ti;
    return 0;
}

// Resident workgroups of k_sweep_tile<cfg> on the current device (occupancy query x CUs).
template <class Cfg, bool SLAB, bool MULTI>
inline int st_resident_cfg()
{
    int occ = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_sweep_tile<Cfg, SLAB, false, MULTI>, Cfg::THREADS, 0) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        return 768;
    }
    return occ * cus;
}
// A slab's persistent tile grid when `share` slab sessions run on this device: half of the chip's resident
// workgroups of that configuration split between them (share 8, quad tiles: 48 each), so every slab keeps
// workgroups resident -- a slab waiting on its upstream neighbour must not hold the CUs that neighbour
// needs -- with room left for the other slabs' second-pass kernels and for uneven placement.
template <bool SLAB, bool MULTI>
inline int st_share_grid(int cfg, int share)
{
    int r;
    if (cfg == ST_CFG_THR) r = st_resident_cfg<StCfgThr, SLAB, MULTI>();
    else if (cfg == ST_CFG_QUAD) r = st_resident_cfg<StCfgQuad, SLAB, MULTI>();
    else if (cfg == ST_CFG_DUO) r = st_resident_cfg<StCfgDuo, SLAB, MULTI>();
    else if (cfg == ST_CFG_OCT) r = st_resident_cfg<StCfgOct, SLAB, MULTI>();
    else if (cfg == ST_CFG_QFP) {
        if constexpr (MULTI) r = st_resident_cfg<StCfgQfp, SLAB, MULTI>();
        else r = st_resident_cfg<StCfgQuad, SLAB, MULTI>();   // (st_launch: the quad tiles serve it)
    }
    else r = st_resident_cfg<StCfgLat, SLAB, MULTI>();
    return std::max(8, r / (2 * std::max(share, 1)));
}

// Launch k_sweep_tile with the configuration `cfg` selects (st_cfg: ST_CFG_*), its lead cap applied.
template <class Cfg, bool SLAB, bool TRACE, bool MULTI>
inline void st_launch_cfg(const char *name, int grid, hipStream_t st, StParams &P, int lead_override)
{
    P.lead = (lead_override >= 0 && lead_override < Cfg::LEAD) ? lead_override : Cfg::LEAD;
    if (getenv("SDFGEN_OCC")) {   // diagnostics: resident workgroups per CU
        const void *f = (const void *)k_sweep_tile<Cfg, SLAB, TRACE, MULTI>;
        int occ = -1;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, f, Cfg::THREADS, 0);
        hipFuncAttributes fa;
        (void)hipFuncGetAttributes(&fa, f);
        fprintf(stderr, "k_sweep_tile<%s>: occupancy %d WG/CU, regs %d, lds %zu, local %zu\n", name, occ, fa.numRegs,
                fa.sharedSizeBytes, fa.localSizeBytes);
    }
    hipLaunchKernelGGL((k_sweep_tile<Cfg, SLAB, TRACE, MULTI>), dim3(grid), dim3(Cfg::THREADS), 0, st, P);
}
template <bool SLAB, bool TRACE, bool MULTI>
inline void st_launch(int cfg, int grid, hipStream_t st, StParams &P, int lead_override)
{
    if (cfg == ST_CFG_THR) st_launch_cfg<StCfgThr, SLAB, TRACE, MULTI>("thr", grid, st, P, lead_override);
    else if (cfg == ST_CFG_QUAD) st_launch_cfg<StCfgQuad, SLAB, TRACE, MULTI>("quad", grid, st, P, lead_override);
    else if (cfg == ST_CFG_DUO) st_launch_cfg<StCfgDuo, SLAB, TRACE, MULTI>("duo", grid, st, P, lead_override);
    else if (cfg == ST_CFG_OCT) st_launch_cfg<StCfgOct, SLAB, TRACE, MULTI>("oct", grid, st, P, lead_override);
    else if (cfg == ST_CFG_QFP) {
        // (the per-sweep launch of the fixed quad lanes crashed hipcc 7.2's greedy register allocator:
        // the quad tiles serve it)
        if constexpr (MULTI) st_launch_cfg<StCfgQfp, SLAB, TRACE, MULTI>("qfp", grid, st, P, lead_override);
        else {
            static bool told = false;   // say so once: a per-sweep launch asked for qfp runs the quad tiles
            if (!told) {
                told = true;
                fprintf(stderr, "sdfgen: SDFGEN_TILE_CFG=5 (qfp) exists only for the one-launch first pass; "
                                "this per-sweep tile launch runs the quad tiles\n");
            }
            st_launch_cfg<StCfgQuad, SLAB, TRACE, MULTI>("quad", grid, st, P, lead_override);
        }
    }
    else st_launch_cfg<StCfgLat, SLAB, TRACE, MULTI>("lat", grid, st, P, lead_override);
}

// Enqueue one sweep direction on `st`.  Returns 0 or a negative SDFGEN_HIP_E* code.
inline int tile_sweep(TileSweepWorkspace &W, hipStream_t st, const float4 *soup, unsigned long long *cell,
                      const float origin[3], float dx, int ni, int nj, int nk, int di, int dj,
                      int dk, char *err, size_t errlen, const TileSlab &slab = TileSlab())
{
    const int A = ni - 1, B = nj - 1, C = nk - 1;
    const int cs = slab.on ? slab.cs : 0, ce = slab.on ? slab.ce : C;
    const int nJ = (B + ST_T - 1) / ST_T, nK = (ce - cs + ST_T - 1) / ST_T;
    const int ntasks = nJ * nK;
    sdf_last_hip = hipSuccess;
    auto fail = [&](int code, const char *msg) { return st_fail_msg(err, errlen, code, msg); };
    int ti = -1;
    if (int rc = st_prepare(W, st, ni, nj, cs, ce, &ti)) return fail(rc, "buffer or task table set-up");
    if (++W.epoch == 0) ++W.epoch;   // 0 = never published
    if (hipError_t e = zero_async(W.ctrl, sizeof(int), st); e != hipSuccess) return fail(sdf_hip_rc(e), "control word reset");
    StParams P;
    memset(&P, 0, sizeof(P));   // every field this launch does not use is null / 0 (P.tm was not: the
                                // Z-slab launches then added their timers through a stray pointer)
    P.soup = soup;
    P.cell = cell;
    P.hb = W.hb;
    P.hc = W.hc;
    P.tasks = W.tasks[ti];
    P.queue = W.ctrl;
    P.err = W.ctrl + 1;
    P.stats = W.count ? W.stats : nullptr;
    P.trace = nullptr;
    if (W.trace_sweep >= 0 && W.trace_sweep == W.cur_sweep) {
        if (int rc = st_grow(&W.trace, &W.cap_trace, 8 * (size_t)ntasks, st)) return fail(rc, "trace buffer");
        P.trace = W.trace;
    }
    P.ox = origin[0];
    P.oy = origin[1];
    P.oz = origin[2];
    P.dx = dx;
    P.ni = ni;
    P.nj = nj;
    P.nk = nk;
    P.A = A;
    P.B = B;
    P.C = C;
    P.nJ = nJ;
    P.nK = nK;
    P.ntasks = ntasks;
    P.di = di;
    P.dj = dj;
    P.dk = dk;
    P.epoch = W.epoch;
    P.sweep = W.cur_sweep;
    for (int q = 0; q < 7; ++q) {   // same table as sweep_sparse.hpp
        const int m = q + 1;
        P.seen[q] = -1;
        for (int s2 = W.cur_sweep - 1; s2 >= 0 && W.skip_seen; --s2) {
            static const int D[8][3] = {{+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
                                        {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};
            const int *d = D[s2 % 8];
            if ((!(m & 1) || d[0] == di) && (!(m & 2) || d[1] == dj) && (!(m & 4) || d[2] == dk)) {
                P.seen[q] = s2 + 1;
                break;
            }
        }
    }
    P.clo = W.clo;
    P.chi = W.chi;
    P.ntri = W.ntri;
    P.cs = cs;
    P.ce = ce;
    P.hbC = ce - cs;
    P.hc_in = slab.on ? slab.in : nullptr;
    P.hc_out = slab.on ? slab.out : nullptr;
    P.tm = slab.on ? W.tm : nullptr;
    if (ntasks <= 0) return 0;
    int grid = ntasks < 2048 ? ntasks : 2048;
    const int cfg = st_cfg(ntasks);
    if (W.grid_override > 0 && W.grid_override < grid) grid = W.grid_override;
    else if (W.grid_override <= 0 && W.share > 1 && slab.on) grid = std::min(grid, st_share_grid<true, false>(cfg, W.share));
    if (slab.on) st_launch<true, false, false>(cfg, grid, st, P, W.lead_override);
    else if (P.trace) st_launch<false, true, false>(cfg, grid, st, P, W.lead_override);
    else st_launch<false, false, false>(cfg, grid, st, P, W.lead_override);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return fail(sdf_hip_rc(e), "launch");
    return 0;
}

// Oriented c range [cs, ce) of Z-slab [kb, ke) of an nk-plane grid for a sweep with k direction dk:
// the slab's own planes, c = k - 1 (dk > 0) or nk - 2 - k (dk < 0); DESIGN.md §7.
inline void st_slab_c_range(int kb, int ke, int nk, int dk, int *cs, int *ce)
{
    if (dk > 0) {
        *cs = std::max(kb, 1) - 1;
        *ce = ke - 1;
    } else {
        *cs = nk - 1 - std::min(ke, nk - 1);
        *ce = nk - 1 - kb;
    }
}

// Physical index range [lo, hi] of oriented tile T (edge ST_T) over oriented [c0, c1) of an axis of
// n cells swept in direction d (oriented x = p - 1 for d > 0, n - 2 - p for d < 0).
inline void st_tile_phys(int T, int c0, int c1, int n, int d, int *lo, int *hi)
{
    const int xl = c0 + ST_T * T, xh = std::min(c0 + ST_T * T + ST_T, c1) - 1;
    if (d > 0) { *lo = xl + 1; *hi = xh + 1; }
    else { *lo = n - 2 - xh; *hi = n - 2 - xl; }
}

// Tiles [*t0, *t1] of the oriented range [c0, c1) (direction d) that cover any physical index in
// [lo, hi]; false if none.
inline bool st_tiles_covering(int lo, int hi, int c0, int c1, int n, int d, int *t0, int *t1)
{
    int xl, xh;   // oriented image of [lo, hi]
    if (d > 0) { xl = lo - 1; xh = hi - 1; }
    else { xl = n - 2 - hi; xh = n - 2 - lo; }
    xl = std::max(xl, c0);
    xh = std::min(xh, c1 - 1);
    if (xl > xh) return false;
    *t0 = (xl - c0) / ST_T;
    *t1 = (xh - c0) / ST_T;
    return true;
}

// Z-slab plan of a multi-sweep launch: the slab boundaries of the whole grid (so every slab
// derives the same global schedule), this launch's slab and its per-sweep inboxes.
struct StSlabPlan {
    int nslabs = 1, slab = 0;
    std::vector<int> kb;                               // nslabs + 1 plane boundaries
    const unsigned long long *in[ST_MAXSW] = {};       // per sweep: this slab's inbox (null: no upstream)
    unsigned long long *out[ST_MAXSW] = {};            // per sweep: the downstream slab's inbox (null: none)
};

// Sweeps s0 .. s0+ns-1 (first pass) in ONE persistent launch: the tasks of all of them in a
// topological order by an estimated start time, so a sweep's first tiles start while the
// previous sweep's last tiles still run.  Each task waits for the tiles of
// the previous sweep that cover its columns (one cell of margin on every side: the face
// cells it reads and the cells a neighbour tile of the previous sweep reads).
// Z-slabs (plan.nslabs > 1): the schedule is computed for the tiles of ALL slabs -- a tile on a
// slab's first plane follows the upstream slab's tile on its last plane like any upstream tile --
// and this launch runs its own slab's tasks in that global order.  Every wait of a task (its
// previous-sweep tiles in this slab, the upstream slab's granules of this sweep) is on a task
// earlier in the global order, so the globally earliest unfinished task can always be claimed
// and run: no cross-GPU deadlock whatever the residency.
inline int tile_sweep_multi(TileSweepWorkspace &W, hipStream_t st, const float4 *soup, unsigned long long *cell,
                            const float origin[3], float dx, int ni, int nj, int nk, int s0, int ns,
                            const int (*dirs)[3], char *err, size_t errlen, const StSlabPlan *plan = nullptr,
                            bool prepare_only = false)
{
    const int A = ni - 1, B = nj - 1, C = nk - 1;
    const int nJ = (B + ST_T - 1) / ST_T;
    sdf_last_hip = hipSuccess;
    auto fail = [&](int code, const char *msg) { return st_fail_msg(err, errlen, code, msg); };
    StSlabPlan one;
    if (!plan) {
        one.kb = {0, nk};
        plan = &one;
    }
    const int nsl = plan->nslabs, me = plan->slab;
    if (ns < 1 || ns > ST_MAXSW || nJ <= 0 || (int)plan->kb.size() != nsl + 1) return fail(-1, "bad multi-sweep request");
    // per (sweep q, slab r): oriented c range and tile rows
    std::vector<int> cs((size_t)ns * nsl), ce((size_t)ns * nsl), nKq((size_t)ns * nsl);
    for (int q = 0; q < ns; ++q)
        for (int r = 0; r < nsl; ++r) {
            const size_t x = (size_t)q * nsl + r;
            st_slab_c_range(plan->kb[r], plan->kb[r + 1], nk, dirs[(s0 + q) % 8][2], &cs[x], &ce[x]);
            nKq[x] = std::max(0, (ce[x] - cs[x] + ST_T - 1) / ST_T);
        }
    // this slab's halo buffers: hb [nJ][ce - cs][A], hc [nK][B][A] per sweep
    size_t nhb = 0, nhc = 0;
    for (int q = 0; q < ns; ++q) {
        const size_t x = (size_t)q * nsl + me;
        nhb = std::max(nhb, (size_t)nJ * (size_t)std::max(ce[x] - cs[x], 0) * A);
        nhc = std::max(nhc, (size_t)nKq[x] * B * A);
    }
    nhb = std::max<size_t>(nhb, 1);
    nhc = std::max<size_t>(nhc, 1);
    // (the sync's status is checked: a fault of an earlier kernel on the stream -- the band, a previous
    // call -- is sticky and must be reported as that fault, not as the allocation after it failing)
    if (W.cap_mhb < ns * nhb || W.cap_mhc < ns * nhc)
        if (int rc = st_sync(st)) return fail(rc, "stream sync before growing the halo buffers (an earlier kernel failed)");
    if (int rc = st_grow(&W.mhb, &W.cap_mhb, ns * nhb, st)) return fail(rc, "halo buffer (b edges)");
    if (int rc = st_grow(&W.mhc, &W.cap_mhc, ns * nhc, st)) return fail(rc, "halo buffer (c edges)");
    if (!W.ctrl) {
        if (hipError_t e = hipMalloc((void **)&W.ctrl, 16 * sizeof(int)); e != hipSuccess) return fail(sdf_hip_rc(e), "control words");
        if (hipError_t e = hipMalloc((void **)&W.stats, ST_NSTATS * sizeof(unsigned long long)); e != hipSuccess)
            return fail(sdf_hip_rc(e), "statistics words");
        if (hipError_t e = hipMemsetAsync(W.ctrl, 0, 16 * sizeof(int), st); e != hipSuccess) return fail(sdf_hip_rc(e), "control word reset");
    }
    int ntasks = 0;
    for (int q = 0; q < ns; ++q) ntasks += nJ * nKq[(size_t)q * nsl + me];
    long long key = ((((long long)ni * 65536 + nj) * 65536 + nk) * 64 + s0) * 16 + ns;
    key = key * 131 + nsl * 17 + me;
    if (const char *e = getenv("SDFGEN_TILE_WC")) key ^= (long long)(atof(e) * 1000.0) << 50;
    if (W.mkey != key) {
        if (int rc = st_sync(st)) return fail(rc, "stream sync before the task graph upload (an earlier kernel failed)");
        // Global tile ids: sweep q, slab r, tile (J, K).  Estimated starts (in units of one tile
        // hop = ST_T steps): +1 per upstream tile of the same sweep (across slab boundaries too),
        // + the tile duration after each previous-sweep tile of the same slab it waits for.
        double wc = (A + 2.0 * (ST_T - 1)) / ST_T;
        if (const char *e = getenv("SDFGEN_TILE_WC")) wc *= atof(e);   // diagnostics: schedule model
        if (!(wc > 0.0)) wc = 1.0;
        std::vector<size_t> base((size_t)ns * nsl + 1, 0);
        for (size_t x = 0; x < (size_t)ns * nsl; ++x) base[x + 1] = base[x] + (size_t)nJ * nKq[x];
        const size_t nall = base[(size_t)ns * nsl];
        auto gid = [&](int q, int r, int J, int K) { return base[(size_t)q * nsl + r] + (size_t)J * nKq[(size_t)q * nsl + r] + K; };
        std::vector<double> kv(nall, 0.0);
        std::vector<std::vector<int>> dep;   // this slab's tasks only: global ids of awaited tiles
        std::vector<size_t> mine;            // global ids of this slab's tasks
        for (int q = 0; q < ns; ++q) {
            const int *d = dirs[(s0 + q) % 8], *dp = dirs[(s0 + q + 7) % 8];
            // slabs in flow order: the k-up sweep enters at slab 0, the k-down sweep at the last
            for (int rr = 0; rr < nsl; ++rr) {
                const int r = d[2] > 0 ? rr : nsl - 1 - rr;
                const int ru = d[2] > 0 ? r - 1 : r + 1;   // upstream slab of this sweep
                const size_t x = (size_t)q * nsl + r;
                for (int J = 0; J < nJ; ++J)
                    for (int K = 0; K < nKq[x]; ++K) {
                        double v = 0.0;
                        if (J) v = std::max(v, kv[gid(q, r, J - 1, K)] + 1.0);
                        if (K) v = std::max(v, kv[gid(q, r, J, K - 1)] + 1.0);
                        else if (ru >= 0 && ru < nsl && nKq[(size_t)q * nsl + ru] > 0)
                            v = std::max(v, kv[gid(q, ru, J, nKq[(size_t)q * nsl + ru] - 1)] + 1.0);
                        std::vector<int> dj;
                        if (q) {
                            const size_t xp = (size_t)(q - 1) * nsl + r;
                            int jl, jh, kl, kh;
                            st_tile_phys(J, 0, B, nj, d[1], &jl, &jh);
                            st_tile_phys(K, cs[x], ce[x], nk, d[2], &kl, &kh);
                            int J0, J1, K0, K1;
                            if (st_tiles_covering(jl - 1, jh + 1, 0, B, nj, dp[1], &J0, &J1) &&
                                st_tiles_covering(kl - 1, kh + 1, cs[xp], ce[xp], nk, dp[2], &K0, &K1))
                                for (int J2 = J0; J2 <= J1; ++J2)
                                    for (int K2 = K0; K2 <= K1; ++K2) {
                                        const size_t u = gid(q - 1, r, J2, K2);
                                        v = std::max(v, kv[u] + wc);
                                        if (r == me) dj.push_back((int)u);
                                    }
                        }
                        kv[gid(q, r, J, K)] = v;
                        if (r == me) {
                            if (dj.size() > (size_t)ST_MAXDEP) return fail(-1, "tile dependency overflow");
                            mine.push_back(gid(q, r, J, K));
                            dep.push_back(std::move(dj));
                        }
                    }
            }
        }
        if ((int)mine.size() != ntasks) return fail(-1, "task count mismatch");
        // modelled critical path of the launch (all slabs), in compute steps: the latency
        // roofline's chain length (bench.py roofline.latency)
        double kmax = 0.0;
        for (double x : kv) kmax = std::max(kmax, x);
        W.chain_steps = (kmax + wc) * ST_T;
        // this slab's tasks by estimated start (ties: global id), then local positions of the deps
        std::vector<int> order((size_t)ntasks);
        for (int t = 0; t < ntasks; ++t) order[t] = t;
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return kv[mine[x]] < kv[mine[y]]; });
        std::vector<int> pos_of_gid_local;   // global id -> local position (this slab's tasks)
        std::vector<std::pair<size_t, int>> gpos((size_t)ntasks);
        for (int rnk = 0; rnk < ntasks; ++rnk) gpos[rnk] = std::make_pair(mine[order[rnk]], rnk);
        std::sort(gpos.begin(), gpos.end());
        auto local_pos = [&](size_t g) {
            auto it = std::lower_bound(gpos.begin(), gpos.end(), std::make_pair(g, -1));
            return (it != gpos.end() && it->first == g) ? it->second : -1;
        };
        std::vector<int4> mt((size_t)ntasks);
        std::vector<int> md((size_t)ntasks * ST_MAXDEP, -1);
        for (int rnk = 0; rnk < ntasks; ++rnk) {
            const int t = order[rnk];
            const size_t g = mine[t];
            int q = 0;
            while (g >= base[(size_t)(q + 1) * nsl]) ++q;
            const size_t x = (size_t)q * nsl + me;
            const int J = (int)((g - base[x]) / nKq[x]), K = (int)((g - base[x]) % nKq[x]);
            int m = 0;
            for (int u : dep[t]) {
                const int pu = local_pos((size_t)u);
                if (pu < 0 || pu >= rnk) return fail(-1, "tile order not topological");
                md[(size_t)rnk * ST_MAXDEP + m++] = pu;
            }
            mt[rnk] = make_int4(J, K, q, 0);
        }
        if (W.cap_mtasks < (size_t)ntasks) {
            (void)hipFree(W.mtasks);
            (void)hipFree(W.mdeps);
            (void)hipFree(W.mdone);
            W.mtasks = nullptr;
            W.mdeps = nullptr;
            W.mdone = nullptr;
            W.cap_mtasks = 0;
            if (hipMalloc((void **)&W.mtasks, std::max(ntasks, 1) * sizeof(int4)) != hipSuccess ||
                hipMalloc((void **)&W.mdeps, (size_t)std::max(ntasks, 1) * ST_MAXDEP * sizeof(int)) != hipSuccess ||
                hipMalloc((void **)&W.mdone, std::max(ntasks, 1) * sizeof(unsigned)) != hipSuccess)
                return fail(sdf_hip_rc(hipGetLastError()), "task graph allocation");
            if (hipError_t e = hipMemsetAsync(W.mdone, 0, std::max(ntasks, 1) * sizeof(unsigned), st); e != hipSuccess)
                return fail(sdf_hip_rc(e), "completion flag reset");
            W.cap_mtasks = std::max(ntasks, 1);
        }
        if (ntasks) {
            hipError_t e = hipMemcpyAsync(W.mtasks, mt.data(), ntasks * sizeof(int4), hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipMemcpyAsync(W.mdeps, md.data(), md.size() * sizeof(int), hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return fail(sdf_hip_rc(e), "task graph upload");
        }
        W.mkey = key;
    }
    if (prepare_only) return 0;   // buffers and tables in place (Z-slabs: before anything is enqueued)
    if (++W.mepoch == 0) ++W.mepoch;   // completion flags of this launch (0 = never)
    if (hipError_t e = zero_async(W.ctrl, sizeof(int), st); e != hipSuccess) return fail(sdf_hip_rc(e), "control word reset");
    StParams P;
    memset(&P, 0, sizeof(P));
    P.soup = soup;
    P.cell = cell;
    P.queue = W.ctrl;
    P.err = W.ctrl + 1;
    P.stats = W.count ? W.stats : nullptr;
    P.trace = nullptr;
    P.ox = origin[0];
    P.oy = origin[1];
    P.oz = origin[2];
    P.dx = dx;
    P.ni = ni;
    P.nj = nj;
    P.nk = nk;
    P.A = A;
    P.B = B;
    P.C = C;
    P.nJ = nJ;
    P.nK = nKq[me];
    P.ntasks = ntasks;
    P.cs = cs[me];
    P.ce = ce[me];
    P.hbC = ce[me] - cs[me];
    P.clo = W.clo;
    P.chi = W.chi;
    P.ntri = W.ntri;
    P.mtasks = W.mtasks;
    P.deps = W.mdeps;
    P.done = W.mdone;
    P.call_epoch = W.mepoch;
    P.tm = nsl > 1 ? W.tm : nullptr;
    for (int q = 0; q < ns; ++q) {
        const int sw = s0 + q, *d = dirs[sw % 8];
        const size_t x = (size_t)q * nsl + me;
        StSweep &S = P.sw[q];
        S.hb = W.mhb + q * nhb;
        S.hc = W.mhc + q * nhc;
        S.di = d[0];
        S.dj = d[1];
        S.dk = d[2];
        S.sweep = sw;
        if (++W.epoch == 0) ++W.epoch;   // one epoch per sweep, as tile_sweep: slabs stay in step
        S.epoch = W.epoch;
        S.cs = cs[x];
        S.ce = ce[x];
        S.nK = nKq[x];
        S.hc_in = nsl > 1 ? plan->in[q] : nullptr;
        S.hc_out = nsl > 1 ? plan->out[q] : nullptr;
        for (int qq = 0; qq < 7; ++qq) {   // the "already examined" rule, as in tile_sweep
            const int m = qq + 1;
            S.seen[qq] = -1;
            for (int s2 = sw - 1; s2 >= 0 && W.skip_seen; --s2) {
                const int *e = dirs[s2 % 8];
                if ((!(m & 1) || e[0] == d[0]) && (!(m & 2) || e[1] == d[1]) && (!(m & 4) || e[2] == d[2])) {
                    S.seen[qq] = s2 + 1;
                    break;
                }
            }
        }
    }
    W.last_ntasks = ntasks;
    W.last_A = A;
    W.last_B = B;
    W.last_nJ = nJ;
    W.last_ns = ns;
    W.last_nhb = nhb;
    W.last_nhc = nhc;
    for (int q = 0; q < ns; ++q) {
        W.last_nK[q] = P.sw[q].nK;
        W.last_hbC[q] = P.sw[q].ce - P.sw[q].cs;
    }
    if (ntasks <= 0) return 0;
    int grid = ntasks < 2048 ? ntasks : 2048;
    // configuration by this slab's tiles per sweep (the largest sweep of the launch)
    int tiles = 0;
    for (int q = 0; q < ns; ++q) tiles = std::max(tiles, nJ * nKq[(size_t)q * nsl + me]);
    W.cfg = st_cfg(tiles);
    if (W.grid_override > 0 && W.grid_override < grid) grid = W.grid_override;
    else if (W.grid_override <= 0 && W.share > 1 && nsl > 1) grid = std::min(grid, st_share_grid<true, true>(W.cfg, W.share));
    if (nsl > 1) st_launch<true, false, true>(W.cfg, grid, st, P, W.lead_override);
    else if (W.trace_multi) {   // diagnostics: per-task timeline of the whole launch (tools/trace_multi.py)
        if (int rc = st_grow(&W.trace, &W.cap_trace, 8 * (size_t)ntasks, st)) return fail(rc, "trace buffer");
        P.trace = W.trace;
        st_launch<false, true, true>(W.cfg, grid, st, P, W.lead_override);
    } else st_launch<false, false, true>(W.cfg, grid, st, P, W.lead_override);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return fail(sdf_hip_rc(e), "launch");
    return 0;
}

// After a fired watchdog (the stream has drained): where the last multi-sweep launch stopped -- the
// task counter, the error words, per sweep the tasks whose completion flag is set, and the first
// unfinished tasks with their dependencies.  Diagnostics, written to stderr.
inline void st_watchdog_report(const TileSweepWorkspace &W, const char *who)
{
    int ctrl[12] = {0};
    if (!W.ctrl || hipMemcpy(ctrl, W.ctrl, sizeof(ctrl), hipMemcpyDeviceToHost) != hipSuccess) return;
    fprintf(stderr, "%s: tile watchdog: queue %d, error bits %d, max sweep+1 %d, first failure sweep+1 %d bit %d, "
                    "cfg %d, epoch %u, call epoch %u\n", who, ctrl[0], ctrl[1], ctrl[2], ctrl[3] & 0xff, ctrl[3] >> 8, W.cfg,
            W.epoch, W.mepoch);
    const int n = W.last_ntasks;
    if (n <= 0 || !W.mdone || !W.mtasks || !W.mdeps) return;
    std::vector<unsigned> done(n);
    std::vector<int4> tk(n);
    std::vector<int> dep((size_t)n * ST_MAXDEP);
    if (hipMemcpy(done.data(), W.mdone, n * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(tk.data(), W.mtasks, n * sizeof(int4), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(dep.data(), W.mdeps, dep.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    int per[ST_MAXSW] = {0}, tot[ST_MAXSW] = {0};
    for (int t = 0; t < n; ++t) {
        const int q = tk[t].z & (ST_MAXSW - 1);
        ++tot[q];
        per[q] += done[t] == W.mepoch;
    }
    for (int q = 0; q < ST_MAXSW; ++q)
        if (tot[q]) fprintf(stderr, "  sweep slot %d: %d of %d tasks done\n", q, per[q], tot[q]);
    int shown = 0;
    for (int t = 0; t < n && shown < 8; ++t) {
        if (done[t] == W.mepoch) continue;
        fprintf(stderr, "  task %d (J %d, K %d, slot %d) not done; deps:", t, tk[t].x, tk[t].y, tk[t].z);
        for (int m = 0; m < ST_MAXDEP; ++m) {
            const int d = dep[(size_t)t * ST_MAXDEP + m];
            if (d >= 0) fprintf(stderr, " %d%s", d, done[d] == W.mepoch ? "" : "*");
        }
        fprintf(stderr, "\n");
        ++shown;
    }
    // the stuck compute wave's halo entries at a = amin: the granules the helper polls
    // (k_sweep_tile's compute-wave watchdog records them: err[3] = ctrl[4] = task + 1, err[10] = ctrl[11] = step + 1;
    // the halo entry a cell (bl, cl) reads at step h is a = h - bl - cl: stream L of the b-edge (bl = 0, cl = L)
    // a = h - L, of the c-edge (cl = 0, bl = L - 8) a = h - (L - 8), the corner a = h)
    const int task = ctrl[4] - 1, hstep = ctrl[11] - 1;
    if ((ctrl[3] >> 8) == 2 && task >= 0 && task < n && hstep >= 0) {
        const int J = tk[task].x, K = tk[task].y, q = tk[task].z;
        const unsigned eq = W.epoch - (unsigned)(W.last_ns - 1 - q);   // slot q's epoch (one per sweep, in order)
        const int A = W.last_A, B = W.last_B, hbC = W.last_hbC[q], nK = W.last_nK[q];
        fprintf(stderr, "  task %d = tile (J %d, K %d) of slot %d (epoch %u), nJ %d nK %d, stuck at step %d; halo granules:\n",
                task, J, K, q, eq, W.last_nJ, nK, hstep);
        auto show = [&](const char *what, const unsigned long long *base, size_t row, int a) {
            if (a < 0 || a >= A) return;   // that stream is not read at this step
            unsigned long long g = 0;
            if (hipMemcpy(&g, base + row * A + a, 8, hipMemcpyDeviceToHost) != hipSuccess) return;
            fprintf(stderr, "    %-30s a = %5d: epoch %u label %d%s\n", what, a, (unsigned)(g >> 32), lbl_of((uint32_t)g),
                    (unsigned)(g >> 32) == eq ? " (ready)" : " (NOT ready)");
        };
        const unsigned long long *hb = W.mhb + (size_t)q * W.last_nhb, *hc = W.mhc + (size_t)q * W.last_nhc;
        const int b0 = J * ST_T, c0 = K * ST_T;   // one GPU: cs = 0
        char buf[64];
        if (J > 0)
            for (int L = 0; L < ST_T && c0 + L < hbC; ++L) {
                snprintf(buf, sizeof(buf), "b-edge stream %d (c %d)", L, c0 + L);
                show(buf, hb, (size_t)(J - 1) * hbC + (c0 + L), hstep - L);
            }
        if (K > 0)
            for (int L = 0; L < ST_T && b0 + L < B; ++L) {
                snprintf(buf, sizeof(buf), "c-edge stream %d (b %d)", ST_T + L, b0 + L);
                show(buf, hc, (size_t)(K - 1) * B + (b0 + L), hstep - L);
            }
        if (J > 0 && K > 0) show("corner stream 16", hb, (size_t)(J - 1) * hbC + (c0 - 1), hstep);
    }
}

inline void tile_sweep_release(TileSweepWorkspace &W)
{
    (void)hipFree(W.mhb);
    (void)hipFree(W.mhc);
    (void)hipFree(W.mtasks);
    (void)hipFree(W.mdeps);
    (void)hipFree(W.mdone);
    (void)hipFree(W.hb);
    (void)hipFree(W.hc);
    (void)hipFree(W.tasks[0]);
    (void)hipFree(W.tasks[1]);
    (void)hipFree(W.ctrl);
    (void)hipFree(W.stats);
    (void)hipFree(W.trace);
    W = TileSweepWorkspace();
}

}  // namespace sdfhip
