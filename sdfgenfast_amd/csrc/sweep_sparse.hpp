// sweep_sparse.hpp -- a sweep direction in which few labels change, computed as a
// parallel Jacobi evaluation followed by an exact, change-driven repair.
//
// Why this is exact.  In one reference sweep (cpu_lib/makelevelset3.cpp:130-151) a
// cell's result depends on its own value from before the sweep (S) and on the CURRENT
// labels of its 7 upwind neighbours -- never on their phi (:94-99).  Write the sweep
// as x_c = f(S_c, labels(x_upwind(c))).  The upwind relation is acyclic, so this system
// has exactly one solution: the Gauss-Seidel result.  We
//   1. evaluate J_c = f(S_c, labels(S_upwind(c))) for every cell at once (k_sp_jacobi);
//      J_c is already the answer for every cell none of whose upwind neighbours changes;
//   2. repair: whenever a cell's label differs from its S label (or later changes
//      again), each downstream neighbour is re-evaluated with the labels current at
//      that time (k_sp_recheck).  Every label change is followed by a re-evaluation
//      that reads it, so when the work list drains every cell satisfies its equation,
//      i.e. X is the unique solution = the reference's bits, in any processing order.
// In the second pass of sweeps only ~0.02-0.07 % of the cells change (256^3, DESIGN.md
// §4), so step 2 touches a few thousand cells instead of walking the whole
// dependency chain.
//
// Concurrency protocol (one device, all memory ops at agent scope so the 8 XCD L2s
// agree):
//   * req[c] counts outstanding recheck requests.  A request that moves it 0 -> 1 owns
//     the cell: it is queued (or run directly by the requester, depth-first).  The
//     runner reads r = req[c], evaluates, and retires r; if more requests arrived
//     meanwhile it evaluates again.  So a cell is never evaluated by two lanes at once
//     and no request is lost.
//   * a new label is published (its store completes) before the requests it triggers;
//     a runner reads labels only after the request it retires was observed: the first
//     evaluation retires just the request that handed it the cell (written after the
//     label that caused it), and every further round retires what its atomicSub saw.
//   * the work list is cut into shards; a wave appends to and takes from its home shard only.
//     The high half of a shard's tail word counts its queued or running work items (it grows
//     in the same atomic as the ring tail, one atomic per wave and iteration for all lanes'
//     new items and finished ones); the shard's workers leave when it is 0.
// Every spin is bounded (watchdog -> error bit, reported by the host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "geom.hpp"

namespace sdfhip {

// A shard's tail word: work items appended to its ring (low 32 bits) and work items queued or
// running (high 32 bits) in ONE word, so an append is one atomic round trip.
// ctl layout: words 0..7 accumulate over the call (error bits, statistics); from SP_QUEUE
// on everything is reset before each sweep: the Z-slab words, the Jacobi list counters of
// SP_JPARTS parts, one 128-byte line each (a shared line serialises the atomics of the whole
// grid: 1.4 ms per sweep at 256^3, measured), then the work-list shards' words.
// Z-slab words (reset per sweep): SP_INHEAD reservations of the inbound ring, SP_INDONE inbound
// lanes finished, SP_EXIT waves exited, SP_OUTTAIL entries this slab appended to the downstream
// slab's inbound ring.
enum { SP_ERR = 0, SP_ENQ = 1, SP_RUNS = 2, SP_DIAG = 4, SP_QUEUE = 8, SP_HEAD = 9, SP_INHEAD = 10, SP_INDONE = 11,
       SP_EXIT = 12, SP_OUTTAIL = 13,
       SP_JPARTS = 64, SP_JSTRIDE = 16, SP_JLIST = 16, SP_SHARD0 = SP_JLIST + SP_JPARTS * SP_JSTRIDE,
       SP_SHSTRIDE = 32, SP_MAXNQ = 16, SP_DIAGX = SP_SHARD0 + SP_MAXNQ * SP_SHSTRIDE,
       SP_NCTL = SP_DIAGX + 32 };   // SP_DIAGX..: diagnostics accumulated over the call
// Work-list shards (SP_NQ): shard s has its own ring (P.queue + s * P.cap), its tail+pending word
// ctl[SP_SHARD0 + s * SP_SHSTRIDE] and its head word 16 words (128 bytes) further.  A wave appends
// to and takes from its home shard only, so every shard is a closed system that drains on its
// own; one shared word serialised the returning atomics of all 64 repair waves.
// SP_ERR bits: 1 repair watchdog, 2 ring overflow, 4 Jacobi list overflow, 8 inbound ring overflow
// (Z-slab), 16 a neighbour slab's flag never came (Z-slab watchdog).
// Z-slab flag words in the uncached communication block (sdfgen_hip.hip SlabSession), one 128-byte
// line each, written by a NEIGHBOUR: SP_FL_DONE + side (its repair finished: every push it made is
// in place), SP_FL_READY + side (it has initialised its live halo: pushes may start),
// SP_FL_COUNT + side (entries it appended to our inbound ring).  side 0 = the lower slab, 1 = upper.
enum { SP_FL_DONE = 0, SP_FL_READY = 2, SP_FL_COUNT = 4, SP_FL_WORDS = 6, SP_FL_STRIDE = 16 };
constexpr unsigned long long SP_PENDING_ONE = 1ull << 32;
constexpr unsigned long long SP_TAIL_LIMIT = 0xF0000000ull;   // appends per sweep (error beyond)
constexpr unsigned SP_WATCHDOG = 1u << 24;   // empty polls (~1 s) before giving up
constexpr int SP_WORKERS = 512;              // max one-wave workgroups of the repair kernel
constexpr int SP_WORKERS_DEFAULT = 256;   // 64-thread repair workgroups (C3: 64 -> 4.75 ms, 256 -> 4.6; C4: 128 -> 21.2, 256 -> 19.5)
// Repair workgroups for a repair over n cells: 512 above 2^25 cells (C4 second pass 12.9-13.1 ->
// 12.2-12.4 ms, more concurrent change chains; C3 neutral: profiles/r03_ab_workers_c{3,4}.log)
inline int sp_workers_for(unsigned long long n) { return n > (1ull << 25) ? SP_WORKERS : SP_WORKERS_DEFAULT; }
#ifndef SP_NQ
#define SP_NQ 8        // work-list shards (fewer where NQ rings of n cells would pass 2^31 entries)
#endif
static_assert(SP_NQ >= 1 && SP_NQ <= 16 && (SP_NQ & (SP_NQ - 1)) == 0, "work-list shards: a power of two <= 16");
// shards for n cells: every shard's ring holds n cells (it can never overflow), all rings together
// at most 2^31 entries (8 GB)
inline unsigned sp_shards(unsigned long long n)
{
    unsigned q = SP_NQ;
    while (q > 1 && (unsigned long long)q * n > (1ull << 31)) q >>= 1;
    return q;
}
constexpr unsigned SP_INLANES = 64u;   // Z-slab inbound-ring workers (workgroup 0's lanes)
#ifndef SP_SPLIT_APPEND
#define SP_SPLIT_APPEND 1   // k_sp_recheck: the append's atomic overlaps the next iteration's first round trip
#endif
#ifndef SP_REQ_BRANCHFREE
#define SP_REQ_BRANCHFREE 1   // the 7 request atomics issued together (else one round trip each)
#endif
#ifndef SP_IDLE_SLEEP
#define SP_IDLE_SLEEP 2
#endif
#ifndef SP_LOCAL_LANES
#define SP_LOCAL_LANES 32   // k_sp_recheck: lanes per wave that take no ring tickets (sp_hand_local)
#endif
static_assert(SP_LOCAL_LANES >= 0 && SP_LOCAL_LANES < 64, "a wave keeps at least one ring lane");
#ifndef SP_DIRECT_POLL
#define SP_DIRECT_POLL 1   // k_sp_recheck: a waiting ring lane polls its slot in the same round trip as the
                           // wave's tail read (the tail only decides the shard's drain), not after it.
                           // Alone neutral (round 5: C3 second pass 2.951-2.962 vs 2.957-2.969 ms,
                           // profiles/r05b_ab_directpoll.log); what it enables, SP_BUSY_NO_TAIL, is not
#endif
#ifndef SP_BUSY_NO_TAIL
#define SP_BUSY_NO_TAIL 1   // with SP_DIRECT_POLL: a wave with an evaluating lane skips the tail read (it only
                            // decides the drain, and a busy wave cannot leave this iteration anyway): second
                            // pass C3 2.82-2.85 -> 2.73-2.76 ms, C4 11.85-12.18 -> 11.45-11.65 ms
                            // (profiles/r05h_ab_repair_c{3,4}.log, interleaved, with SP_SINGLE_PASS)
#endif
#ifndef SP_BUSY_NO_TICKET
#define SP_BUSY_NO_TICKET 0 // a wave with an evaluating lane takes no new ring tickets (lanes holding one keep
                            // polling their slot)
#endif
static_assert(!SP_BUSY_NO_TAIL || SP_DIRECT_POLL, "skipping the tail read needs the direct slot poll");
#ifndef SP_LATE_APPEND
#define SP_LATE_APPEND 0   // k_sp_recheck (SP_SPLIT_APPEND): wait for the previous iteration's append atomic at the
                           // end of this iteration instead of before the evaluation (its ring slots fill later)
#endif
#ifndef SP_SINGLE_PASS
#define SP_SINGLE_PASS 1   // sp_eval_w: a pass in which no lane has a second candidate evaluates one distance per lane
                          // (second pass C3 2.95-2.97 -> 2.82-2.85 ms, C4 11.99-12.33 -> 11.85-12.18 ms,
                          // profiles/r05h_ab_repair_c{3,4}.log)
#endif
#ifndef SP_VMASK
#define SP_VMASK 1   // sp_mask_w in integer VALU arithmetic instead of compare masks: Jacobi scan SALU 1.69e8 -> 0.99e8
                     // per C4 launch; second pass C4 11.54-11.61 -> 11.40-11.42 ms, C3 neutral (profiles/r05w_ab_vmask_c{3,4}.log,
                     // r05x_sq_{cur,vmask}_c4.log)
#endif
#ifndef SP_JLIST_PER_PART
#define SP_JLIST_PER_PART 128  // list-pass workgroups per Jacobi list part (one device): 32 -> 128, C4 list pass 282 -> 262 us per
                               // sweep, C3 39.5 -> 38 us (profiles/r05bd_jlist_grid.txt; 256 the same, 512 slower)
#endif
#ifndef SP_JBLOCKS
#define SP_JBLOCKS 16384   // most 256-thread workgroups of the Jacobi scan (a multiple of 8 XCDs x SP_JPARTS)
#endif
#ifndef SP_JSCAN_FAST
#define SP_JSCAN_FAST 1   // k_sp_jacobi on one device below 2^29 cells: scalar neighbour bases, one 32-bit offset, and
                          // only "any candidate" (sp_any_scan) -- the scan is VALU-issue-bound since SP_VMASK
#endif
#ifndef SP_JSCAN_PAIR
#define SP_JSCAN_PAIR 2   // the fast scan as k_sp_jscan2<NP>: 2 NP cells per lane, 16-byte loads (needs SP_PAD cells of
                          // padding past the grid in both state buffers: sp_pad); 0 = the 8-load k_sp_jacobi<false, true>;
                          // SDFGEN_JSCAN_NP (diagnostics) overrides: 0, 1, 2.  Second pass, interleaved A/B
                          // (profiles/r06g_ab_jscan_c{3,4}.log): C4 11.05 (0) / 10.44 (1) / 10.43-10.46 ms (2),
                          // C3 2.60 / 2.66 / 2.57-2.60 ms; scan launch C4 630 -> 518 us (2)
#endif
#ifndef SP_JSCAN_K
#define SP_JSCAN_K 1   // the pair scan streaming along k (k_sp_jscan3): two pair loads per plane instead of four;
                       // SDFGEN_JSCAN_K=0 (diagnostics) runs k_sp_jscan2
#endif
#ifndef SP_JACOBI_CHUNK
#define SP_JACOBI_CHUNK 1   // k_sp_jacobi: a contiguous chunk per block (L2 reuse of the upwind plane)
#endif

// Ring slot of work-list position t.  Positions restart at 0 every sweep and a sweep appends far
// fewer items than a ring holds, so the 64-bit remainder (~100 instructions, x7 in an append) is
// only a cold fallback kept out of the repair loop's hot path.
__device__ __forceinline__ unsigned long long sp_slot(unsigned long long t, unsigned long long cap)
{
    if (t >= cap) t %= cap;
    return t;
}

// the reference's 8 sweep directions in pass order (cpu_lib/makelevelset3.cpp:243-291)
constexpr int SP_DIRS[8][3] = {{+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
                               {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};

struct SpParams {
    const float4 *soup;                // 3 float4 per triangle
    const unsigned long long *S;       // (phi bits << 32) | label before the sweep, i-fastest
    unsigned long long *X;             // result of the sweep
    unsigned long long *sv;            // in place (S == X; one GPU): the pre-sweep value of every cell
                                       // that changed in this sweep, stored before its first change
                                       // (its stamp says it changed); null: S and X are two buffers
    unsigned *req;                     // per-cell recheck requests (zero between sweeps)
    unsigned *queue;                   // ring of cell+1 (0 = empty)
    unsigned *jlist;                   // Jacobi list: SP_JPARTS parts of jcap cells
    unsigned long long jcap;
    unsigned long long *ctl;           // SP_* counters
    unsigned long long cap;            // ring slots per work-list shard
    unsigned nq;                       // work-list shards (sp_shards)
    unsigned long long n;              // cells
    float ox, oy, oz, dx;
    int ni, nj, nk;
    int di, dj, dk;
    int sweep;                         // index (0..15) of this sweep
    int seen[7];                       // per neighbour slot q: s'+1 of the last earlier sweep in which
                                       // an interior cell examined that neighbour (-1: none)
    unsigned long long c_lo;           // first cell of this launch's range (n cells from c_lo)
    int k_lo, k_hi;                    // planes whose cells this launch owns (whole grid: 0, nk)
    // ---- Z-slab (SLAB kernels): the neighbour planes live in uncached halo planes
    // indexed i + ni*j, the upstream slab's changes arrive as pushes ----
    int k_first, k_last;               // this slab's first / last plane in the sweep's k direction
    int up_side;                       // side of the upstream slab (0 lower, 1 upper)
    const uint32_t *hS_up;             // upstream plane's low words before the sweep
    uint32_t *hX_up;                   // ... live (pushed by the upstream slab)
    uint32_t *push_down_halo;          // downstream slab's live halo of our last plane (remote; null: none)
    uint32_t *push_down_ring;          // downstream slab's inbound ring (remote)
    uint32_t *push_up_halo;            // upstream slab's halo of our first plane for its NEXT sweep (remote)
    uint32_t *in_ring;                 // our inbound ring: cell + 1 of upstream cells that changed (null: none)
    unsigned long long ring_cap;
    unsigned long long *flags;         // our flag words (written by the neighbours)
    unsigned long long *up_flags, *down_flags;   // the neighbours' flag words (remote; null: none)
    unsigned long long epoch;          // this sweep's synchronisation epoch
    unsigned long long ntri;           // triangles in the soup (bounds-checked builds)
    unsigned long long *tm;            // Z-slab phase timers (TM_*; null: not recorded)
    int tm_m;                          // second-pass sweep index 0..7 for tm
};

typedef uint32_t sp_u32x4 __attribute__((ext_vector_type(4), aligned(8)));   // two 8-byte cells, 8-byte aligned

__device__ __forceinline__ unsigned long long sp_ld64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sp_st64(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Every shared word of the repair pass (X, req, queue, ctl) is accessed with agent-scope
// (sc1) atomics, which are coherent across the XCD L2s; ordering between two of them
// only needs the first to have completed before the second issues.  That is a
// vmcnt wait -- not __threadfence(), whose L2 write-back is for plain stores.
__device__ __forceinline__ void sp_order() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned sp_ld32(const unsigned *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sp_st32(unsigned *p, unsigned v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// cell inside the reference's loop range for this direction (i0..i1 of :243-291)
__device__ __forceinline__ bool sp_in(const SpParams &P, int i, int j, int k)
{
    return (P.di > 0 ? i >= 1 : i <= P.ni - 2) && (P.dj > 0 ? j >= 1 : j <= P.nj - 2) &&
           (P.dk > 0 ? k >= 1 : k <= P.nk - 2);
}

// f(own, upwind labels) in the reference's check order (:143-149): strict '<', first
// minimum wins; labels equal to the cell's own original label or to an earlier
// candidate are skipped (their distance cannot win -- sweep_cell).
// One more exact skip: phi_c always equals d(c, label_c) and only decreases, so once c
// has examined label L, d(c, L) >= phi_c for ever after.  An interior cell examined
// neighbour u in the last earlier sweep s' whose direction makes u upwind of c (seen[q]);
// if u's label has not changed since (the sweep stamped in u's low word is <= s'), c has
// already seen that label.  A label set in this very sweep carries this sweep's stamp,
// so the LIVE (repair) evaluation needs no extra check.
// the low words (label, stamp) of the 7 upwind neighbours: half the bytes of the 8-byte cells (a
// 32-bit load of a 64-bit atomically stored word sees one of its stored values' halves)
template <bool LIVE, bool SLAB = false>
__device__ __forceinline__ void sp_nb_words(const SpParams &P, const unsigned long long *L, int i, int j, int k,
                                            size_t c, uint32_t (&w)[7])
{
    const long long si = P.di, sj = (long long)P.dj * P.ni, sk = (long long)P.dk * P.ni * P.nj;
    const long long cc = (long long)c;
    const long long nb[7] = {cc - si, cc - sj, cc - si - sj, cc - sk, cc - si - sk, cc - sj - sk, cc - si - sj - sk};
    // Z-slab: the k-upwind plane of the slab's first plane is the upstream slab's (halo plane)
    const bool halo = SLAB && (k - P.dk < P.k_lo || k - P.dk >= P.k_hi);
    const long long hp = (long long)i + (long long)P.ni * j;   // plane index of (i, j)
    const long long hnb[3] = {hp, hp - P.di, hp - (long long)P.dj * P.ni};   // q = 3 (k), 4 (i,k), 5 (j,k); 6 below
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        if (SLAB && q >= 3 && halo) {
            const long long hq = q == 6 ? hp - P.di - (long long)P.dj * P.ni : hnb[q - 3];
            const uint32_t *hw = (LIVE ? P.hX_up : P.hS_up) + SDF_CHK(23, hq, 0, (size_t)P.ni * P.nj);
            w[q] = __hip_atomic_load(hw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            const uint32_t *lw = reinterpret_cast<const uint32_t *>(L + SDF_CHK(22, nb[q], P.c_lo, P.c_lo + P.n));
            w[q] = LIVE ? sp_ld32(lw) : *lw;
        }
    }
}

// the candidate mask from the neighbours' low words
__device__ __forceinline__ unsigned sp_mask_w(const SpParams &P, int i, int j, int k, unsigned long long own,
                                              const uint32_t (&w)[7], int (&lab)[7], bool live)
{
    int lcq[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        lab[q] = lbl_of(w[q]);
        lcq[q] = lc_of(w[q]);
    }
    const bool interior = i >= 1 && i <= P.ni - 2 && j >= 1 && j <= P.nj - 2 && k >= 1 && k <= P.nk - 2;
#if SP_VMASK
    (void)live;
    // The same test in integer VALU arithmetic (no compare masks to combine: the compare form's
    // ~60 SGPR-mask ORs/ANDs per 64 cells made the Jacobi scan issue-bound on the CU's one scalar
    // unit).  On raw 27-bit labels: d = min over {none, own, earlier slots} of (label ^ that) is 0
    // exactly when the slot's label is none, the cell's own or a duplicate; bit 31 of (d | -d) is
    // d != 0; bit 31 of (seen[q] - lc) is lc > seen[q] (both small; seen = -1: never).
    auto opq = [](uint32_t x) { asm volatile("" : "+v"(x)); return x; };   // keeps it arithmetic
    const uint32_t rown = (uint32_t)own & LBL_MASK;
    const uint32_t itr = opq(interior ? 0xffffffffu : 0u);
    uint32_t rl[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) rl[q] = w[q] & LBL_MASK;
    unsigned f = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        uint32_t d = min(rl[q] ^ LBL_MASK, rl[q] ^ rown);
#pragma unroll
        for (int r = 0; r < q; ++r) d = min(d, rl[q] ^ rl[r]);
        d = opq(d);
        const uint32_t keep = (d | (0u - d)) & ((uint32_t)(P.seen[q] - lcq[q]) | ~itr);
        f |= (keep >> 31) << q;
    }
#else
    const int ct0 = lbl_of((uint32_t)own);
    unsigned f = 0;   // candidates to evaluate, one bit per upwind slot q
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int t = lab[q];
        bool skip = (t < 0) | (t == ct0);
#pragma unroll
        for (int r = 0; r < q; ++r) skip = skip | (lab[r] == t);
        skip = skip | (interior & (lcq[q] <= P.seen[q]));   // seen[q] = -1: never
        f |= (skip ? 0u : 1u) << q;
    }
#endif
#ifdef SP_JACOBI_NOEVAL   // diagnostics only: the Jacobi pass's memory floor (wrong results)
    if (!live) f = 0;
#endif
    return f;
}

// Whether sp_mask_w's mask is non-zero, for the Jacobi scan's list decision (which needs nothing more):
// the same tests on the raw words, with the keep bit formed as ~(d - 1) (d < 2^27, so bit 31 of d - 1 is
// d == 0) and the seven keep words OR-ed together instead of packed into a mask -- 83 instead of ~105
// VALU per cell.
__device__ __forceinline__ bool sp_any_scan(const SpParams &P, uint32_t own, const uint32_t (&w)[7], bool interior)
{
    auto opq = [](uint32_t x) { asm volatile("" : "+v"(x)); return x; };   // keeps it arithmetic (sp_mask_w)
    const uint32_t itr = opq(interior ? 0xffffffffu : 0u);
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        uint32_t d = min((w[q] ^ LBL_MASK) & LBL_MASK, (w[q] ^ own) & LBL_MASK);
#pragma unroll
        for (int r = 0; r < q; ++r) d = min(d, (w[q] ^ w[r]) & LBL_MASK);
        d = opq(d);
        const uint32_t sq = (uint32_t)(P.seen[q] - (int)(w[q] >> LBL_BITS));   // bit 31: lc > seen[q]
        acc |= ~(d - 1u) & (sq | ~itr);
    }
    return (acc >> 31) != 0u;
}

template <bool LIVE, bool SLAB = false>
__device__ __forceinline__ unsigned sp_mask(const SpParams &P, const unsigned long long *L, int i, int j, int k,
                                            size_t c, unsigned long long own, int (&lab)[7])
{
    uint32_t w[7];
    sp_nb_words<LIVE, SLAB>(P, L, i, j, k, c, w);
    return sp_mask_w(P, i, j, k, own, w, lab, LIVE);
}

// f(own, upwind labels) from the neighbours' low words
template <bool LIVE>
__device__ __forceinline__ unsigned long long sp_eval_w(const SpParams &P, int i, int j, int k,
                                                        unsigned long long own, const uint32_t (&w)[7])
{
    int lab[7];
    unsigned f = sp_mask_w(P, i, j, k, own, w, lab, LIVE);
    float phi = __uint_as_float((uint32_t)(own >> 32));
    int ct = lbl_of((uint32_t)own);
    bool changed = false;
    const f3 gx = mk3((float)i * P.dx + P.ox, (float)j * P.dx + P.oy, (float)k * P.dx + P.oz);
#ifdef SP_JACOBI_COUNT   // diagnostics only: candidates vs. packed slots the wave runs
    unsigned passes_ = 0;
    const unsigned cands_ = __builtin_popcount(f);
#endif
    // Candidates in increasing q, two per pass in packed FP32 (ptd_wave2): every lane walks
    // its own list, so a wave runs max(count)/2 passes instead of one divergent ptd per slot
    // q that any lane needs.  Distances do not depend on phi, so applying each pair in q
    // order right after it is evaluated is the reference's check order (:143-149).
    while (__any(f != 0u)) {
#ifdef SP_JACOBI_COUNT
        ++passes_;
#endif
        const bool has_a = f != 0u;
        const int qa = has_a ? __builtin_ctz(f) : 0;
        f &= f - 1u;
        const bool has_b = f != 0u;
        const int qb = has_b ? __builtin_ctz(f) : qa;
        f &= f - 1u;
        int ta = lab[0], tb = lab[0];
#pragma unroll
        for (int q = 1; q < 7; ++q) {   // static indices: no register-array indexing
            ta = (qa == q) ? lab[q] : ta;
            tb = (qb == q) ? lab[q] : tb;
        }
        const size_t ba = 3 * SDF_CHK(26, (has_a ? ta : 0), 0, P.ntri);
        const float4 a0 = P.soup[ba], a1 = P.soup[ba + 1], a2 = P.soup[ba + 2];
        float da, db = 0.f;
#if SP_SINGLE_PASS
        if (!__any(has_b)) {
            // no lane has a second candidate left: one distance per lane (ptd_wave, ~2/3 of a packed pass)
            da = ptd_wave(gx, mk3(a0.x, a0.y, a0.z), mk3(a1.x, a1.y, a1.z), mk3(a2.x, a2.y, a2.z), a2.w);
        } else
#endif
        {
            const size_t bb = 3 * SDF_CHK(26, (has_b ? tb : (has_a ? ta : 0)), 0, P.ntri);
            const float4 b0 = P.soup[bb], b1 = P.soup[bb + 1], b2 = P.soup[bb + 2];
            ptd_wave2(gx, mk3(a0.x, a0.y, a0.z), mk3(a1.x, a1.y, a1.z), mk3(a2.x, a2.y, a2.z), a2.w, gx,
                      mk3(b0.x, b0.y, b0.z), mk3(b1.x, b1.y, b1.z), mk3(b2.x, b2.y, b2.z), b2.w, da, db);
        }
        if (has_a && da < phi) {
            phi = da;
            ct = ta;
            changed = true;
        }
        if (has_b && db < phi) {
            phi = db;
            ct = tb;
            changed = true;
        }
    }
#ifdef SP_JACOBI_COUNT
    if (!LIVE) {
        atomicAdd(&P.ctl[SP_DIAG], (unsigned long long)cands_);
        atomicAdd(&P.ctl[SP_DIAG + 1], (unsigned long long)passes_);
    }
#endif
    if (!changed) return own;
    return ((unsigned long long)__float_as_uint(phi) << 32) | lo_word(ct, P.sweep + 1);
}

template <bool LIVE, bool SLAB = false>
__device__ __forceinline__ unsigned long long sp_eval(const SpParams &P, const unsigned long long *L, int i, int j,
                                                      int k, size_t c, unsigned long long own)
{
    uint32_t w[7];
    sp_nb_words<LIVE, SLAB>(P, L, i, j, k, c, w);
    return sp_eval_w<LIVE>(P, i, j, k, own, w);
}


// Request rechecks of the downstream neighbours of (i,j,k) (the cells whose upwind set
// contains it): the 7 request counters in one round trip.  The cells whose counter moved 0 -> 1
// are this lane's to queue: slot bits in *qmask, cells in tgt[].  With `claim`, the first of them
// is returned instead (the caller runs it itself, depth-first) and left out of *qmask.
// Only cells of planes [k_lo, k_hi) are requested (a Z-slab's own planes; for an upstream slab's
// cell -- an inbound entry -- that is the cells of this slab's first plane).
__device__ __forceinline__ size_t sp_request_collect(const SpParams &P, int i, int j, int k, size_t c, bool claim,
                                                     unsigned *qmask, size_t (&tgt)[7])
{
    const bool ii = P.di > 0 ? i + 1 <= P.ni - 1 : i - 1 >= 0;
    const bool jj = P.dj > 0 ? j + 1 <= P.nj - 1 : j - 1 >= 0;
    const bool kk = k + P.dk >= P.k_lo && k + P.dk < P.k_hi;
    const bool k0 = k >= P.k_lo && k < P.k_hi;   // targets in this cell's own plane
    const long long si = P.di, sj = (long long)P.dj * P.ni, sk = (long long)P.dk * P.ni * P.nj;
    const long long cc = (long long)c;
    unsigned old[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        // same order as the upwind list: (i), (j), (i,j), (k), (i,k), (j,k), (i,j,k)
        const int m = q + 1;
        const bool ui = m & 1, uj = m & 2, uk = m & 4;
        const bool ok = !((ui && !ii) || (uj && !jj) || (uk && !kk) || (!uk && !k0));
        tgt[q] = ok ? (size_t)(cc + (ui ? si : 0) + (uj ? sj : 0) + (uk ? sk : 0)) : ~(size_t)0;
        // branch-free: a slot with no target adds 0 to the range's first counter (not to c's own:
        // an inbound entry's c is the upstream slab's cell, outside this range).  (A conditional
        // atomic merged with a constant made hipcc wait for each of the 7 in turn: 7 round trips.)
#if SP_REQ_BRANCHFREE
        const unsigned r = atomicAdd(&P.req[SDF_CHK(24, ok ? tgt[q] : (size_t)P.c_lo, P.c_lo, P.c_lo + P.n)], ok ? 1u : 0u);
        old[q] = ok ? r : 1u;
#else
        old[q] = ok ? atomicAdd(&P.req[SDF_CHK(24, tgt[q], P.c_lo, P.c_lo + P.n)], 1u) : 1u;
#endif
    }
    size_t mine = ~(size_t)0;
    unsigned qm = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        if (old[q] != 0u) continue;
        if (claim && mine == ~(size_t)0) mine = tgt[q];
        else qm |= 1u << q;
    }
    *qmask = qm;
    return mine;
}

// Wave-level (every lane of the wave calls it, uniformly): queue the cells each lane collected
// (qmask / tgt of sp_request_collect) and retire `fin` lanes' work items, in ONE atomic on the
// shared queue word per wave.  Its low half is the ring tail, its high half the work items queued
// or running: new items count before this wave's finished ones stop counting, so the count cannot
// touch 0 while work remains.  (One atomic per lane saturated the word: ~100 returning atomics per
// microsecond on one address at 256^3 -- DESIGN.md §4.)
__device__ __forceinline__ void sp_append_wave(const SpParams &P, unsigned shard, unsigned qmask, const size_t (&tgt)[7],
                                               bool fin, unsigned nloc = 0)
{
    const unsigned lane = threadIdx.x & 63;
    const unsigned nq = __popc(qmask);
    const unsigned long long b0 = __ballot(nq & 1u), b1 = __ballot(nq & 2u), b2 = __ballot(nq & 4u),
                             bf = __ballot(fin);
    if (!(b0 | b1 | b2 | bf) && nloc == 0u) return;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned pre = (unsigned)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt));
    const unsigned long long tot = (unsigned long long)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    const unsigned long long nfin = (unsigned long long)__popcll(bf);
    unsigned long long t0 = 0;
    if (lane == 0) {
        // pending += tot - nfin, tail += tot (two's complement in the high half)
        const unsigned long long old_q = atomicAdd(&P.ctl[SP_SHARD0 + shard * SP_SHSTRIDE], (tot + nloc - nfin) * SP_PENDING_ONE + tot);
        t0 = old_q & 0xffffffffull;
        if (t0 + tot > SP_TAIL_LIMIT) atomicOr(&P.ctl[SP_ERR], 2ull);
    }
    t0 = ((unsigned long long)(unsigned)__shfl((int)(t0 >> 32), 0) << 32) | (unsigned)__shfl((int)t0, 0);
    unsigned long long t = t0 + pre;
#pragma unroll
    for (int q = 0; q < 7; ++q)
        if ((qmask >> q) & 1u) sp_st32(P.queue + (size_t)shard * P.cap + sp_slot(t++, P.cap), (unsigned)(tgt[q] + 1));
}

// sp_append_wave in two halves, so that the append's round trip overlaps the next iteration's
// first one (k_sp_recheck, SP_SPLIT_APPEND): sp_append_issue makes the wave's ONE atomic on the
// shard word (inline asm: the compiler's atomic optimiser would wait for it on the spot) and keeps
// what the stores need; sp_append_finish waits for the returned tail and stores the cells.  Until
// then the slots read 0 (a poller retries), while the items already count as pending.
struct SpAppend {
    unsigned long long old_q;   // lane 0: the shard word before the atomic (in flight until finish)
    unsigned long long tot;     // items appended by the wave
    unsigned pre;               // this lane's first item's offset
    unsigned qmask;             // this lane's items (slots of tgt)
    bool live;                  // wave-uniform: an atomic is in flight
};
__device__ __forceinline__ void sp_append_issue(const SpParams &P, unsigned shard, unsigned qmask, bool fin,
                                                unsigned nloc, SpAppend &A)
{
    const unsigned lane = threadIdx.x & 63;
    const unsigned nq = __popc(qmask);
    const unsigned long long b0 = __ballot(nq & 1u), b1 = __ballot(nq & 2u), b2 = __ballot(nq & 4u),
                             bf = __ballot(fin);
    A.live = (b0 | b1 | b2 | bf) != 0ull || nloc != 0u;
    if (!A.live) return;
    const unsigned long long lt = (1ull << lane) - 1ull;
    A.pre = (unsigned)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt));
    A.tot = (unsigned long long)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    A.qmask = qmask;
    const unsigned long long nfin = (unsigned long long)__popcll(bf);
    if (lane == 0) {
        // pending += tot + nloc - nfin, tail += tot (two's complement in the high half): the cells
        // handed to the wave's own lanes (sp_hand_local) run without passing through the ring
        unsigned long long *w = &P.ctl[SP_SHARD0 + shard * SP_SHSTRIDE];
        const unsigned long long d = (A.tot + nloc - nfin) * SP_PENDING_ONE + A.tot;
        // (s_nop 1: hipcc pads nothing inside asm -- the operand registers are rewritten right after)
        asm volatile("global_atomic_add_x2 %0, %1, %2, off sc0\n\ts_nop 1" : "=&v"(A.old_q) : "v"(w), "v"(d) : "memory");
    }
}
// The wait is unconditional (a scalar instruction every path from the loop top passes, live or
// not), so that the ISA check tools/check_split_append.py (run by tests/test_split_append_asm.py on
// every build) can prove statically that no instruction names the atomic's destination registers
// before it: the compiler's wait-count pass does not see the asm atomic.  Not live, it costs nothing
// extra -- by then every iteration's vector memory operations have been waited for by the returning
// atomics around it.
__device__ __forceinline__ void sp_append_finish(const SpParams &P, unsigned shard, const size_t (&tgt)[7], SpAppend &A)
{
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(A.old_q)::"memory");   // the returned word has landed
    if (!A.live) return;
    A.live = false;
    const unsigned lane = threadIdx.x & 63;
    unsigned long long t0 = 0;
    if (lane == 0) {
        t0 = A.old_q & 0xffffffffull;
        if (t0 + A.tot > SP_TAIL_LIMIT) atomicOr(&P.ctl[SP_ERR], 2ull);
    }
    t0 = ((unsigned long long)(unsigned)__shfl((int)(t0 >> 32), 0) << 32) | (unsigned)__shfl((int)t0, 0);
    unsigned long long t = t0 + A.pre;
#pragma unroll
    for (int q = 0; q < 7; ++q)
        if ((A.qmask >> q) & 1u) sp_st32(P.queue + (size_t)shard * P.cap + sp_slot(t++, P.cap), (unsigned)(tgt[q] + 1));
}

// wave-synchronous LDS hand-over between lanes of one wave
__device__ __forceinline__ void sp_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-level (uniform call): the cells the wave's lanes claimed this iteration (qmask / tgt of
// sp_request_collect) go first to the wave's own idle hand-off lanes (`free_lane`: lanes that take
// no ring tickets), in (lane, slot) order, through a 64-entry LDS array; only the rest is appended
// to the ring.  A chain link handed over this way costs no ring round trips (append atomic, slot
// store, the taker's tail read and slot poll): the taker evaluates it in the next iteration, like a
// depth-first claim.  Returns the number of cells handed over (wave-uniform); *got = the taken cell.
__device__ __forceinline__ unsigned sp_hand_local(unsigned *s_hand, unsigned *qmask, const size_t (&tgt)[7],
                                                  bool free_lane, size_t *got, unsigned long long *ipt = nullptr,
                                                  unsigned long long *ipd = nullptr)
{
#ifdef SP_ITER_PROF
#define SP_IPH(q) do { const unsigned long long t2_ = clock64(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); ipd[q] += t2_ - *ipt; *ipt = t2_; } while (0)
#else
#define SP_IPH(q) do { } while (0)
#endif
    const unsigned lane = threadIdx.x & 63;
    const unsigned nq = __popc(*qmask);
    const unsigned long long fm = __ballot(free_lane), b0 = __ballot(nq & 1u), b1 = __ballot(nq & 2u),
                             b2 = __ballot(nq & 4u);
    SP_IPH(9);
    if (!fm || !(b0 | b1 | b2)) return 0u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned tot = (unsigned)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    const unsigned nloc = tot < (unsigned)__popcll(fm) ? tot : (unsigned)__popcll(fm);
    unsigned x = (unsigned)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt));
    unsigned keep = *qmask;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        if ((*qmask >> q) & 1u) {
            if (x < nloc) {
                s_hand[x] = (unsigned)tgt[q];
                keep &= ~(1u << q);
            }
            ++x;
        }
    }
    SP_IPH(9);
    sp_wave_sync();
    const unsigned r = (unsigned)__popcll(fm & lt);
    if (free_lane && r < nloc) *got = s_hand[r];
    sp_wave_sync();   // every taker has read before the array is written again
    *qmask = keep;
    return nloc;
}

// Pass 1 of the sparse sweep: every cell against the labels of S, in two kernels.
// k_sp_jacobi streams the grid: a cell with no label left to examine (sp_mask == 0,
// ~90 % of them) is copied to X as is; the others are appended to a compact list that
// k_sp_jlist evaluates.  Evaluating in place would cost every wave as many ptd passes as
// its busiest lane needs while ~7 % of the packed lanes carry a candidate (measured,
// DESIGN.md §4); over the list nearly every lane has work.  Each wave gathers its list
// cells in LDS and appends them with one atomic per ~200 cells.
constexpr int SP_JWAVE = 256;   // LDS list entries per wave

// Z-slab: a cell of the slab's last plane (in the sweep's k direction) changed its label: write
// the new low word into the downstream slab's live halo, then -- once that store has completed --
// append the cell to the downstream slab's inbound ring (the slot is reserved locally; the
// downstream slab turns the entry into rechecks of its first plane).  A change on the first plane
// goes to the upstream slab's halo for its next sweep (no recheck there: it is downstream of it).
__device__ __forceinline__ void sp_push(const SpParams &P, int i, int j, int k, size_t c, uint32_t w)
{
    const size_t hp = (size_t)i + (size_t)P.ni * j;
    (void)SDF_CHK(27, hp, 0, (size_t)P.ni * P.nj);
    if (k == P.k_last && P.push_down_halo) {
        __hip_atomic_store(P.push_down_halo + hp, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long t = atomicAdd(&P.ctl[SP_OUTTAIL], 1ull);
        if (t < P.ring_cap)
            __hip_atomic_store(P.push_down_ring + t, (uint32_t)(c + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            atomicOr(&P.ctl[SP_ERR], 8ull);
    }
    if (k == P.k_first && P.push_up_halo)
        __hip_atomic_store(P.push_up_halo + hp, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// In place (P.sv != null, S == X) this reads the upwind neighbours' labels through P.S with plain
// loads while other lanes of the same launch store new labels into those cells: a neighbour may be
// seen before or after its own change in this pass.  Both are allowed -- the pass only has to give
// every cell whose upwind labels never change its final value; any cell that read a stale label has
// an upwind neighbour that relabelled, and every relabel requests its 7 downstream cells
// (sp_request_collect below) AFTER its store, so the repair pass re-evaluates them against the final
// labels.  This relies on the 8-byte cell stores never tearing (one global_store_dwordx2 per cell)
// and on S / X never being declared __restrict__ or read through the constant cache: the compiler must
// not assume the stores leave S unchanged.
// PAIR (one device): the cell and its 7 upwind low words from four 16-byte loads instead of eight narrow ones
// (the list pass ran at 56 % TA busy at C4, profiles/r06_limiter_c4.json): the pairs (c - 1, c) for di > 0 or
// (c, c + 1) for di < 0, at the cell and at its j-, k- and jk-upwind cells -- all inside the grid for a
// listed cell (it lies in the sweep's range, so every upwind neighbour exists).
template <bool SLAB = false, bool PAIR = false>
__device__ __forceinline__ void sp_jacobi_cell(const SpParams &P, unsigned c32, unsigned *qmask, size_t (&tgt)[7])
{
    const int i = (int)(c32 % (unsigned)P.ni);
    const unsigned r = c32 / (unsigned)P.ni;
    const int j = (int)(r % (unsigned)P.nj), k = (int)(r / (unsigned)P.nj);
    unsigned long long s, y;
    if constexpr (PAIR && !SLAB) {
        const long long dJ = -(long long)P.dj * P.ni, dK = -(long long)P.dk * P.ni * P.nj;
        const bool pos = P.di > 0;
        const unsigned long long *b = P.S + (long long)c32 - (pos ? 1 : 0);   // the pair holding the cell
        (void)SDF_CHK(22, (unsigned long long)((long long)c32 - (pos ? 1 : 0) + std::min(dJ, 0ll) + std::min(dK, 0ll)), 0, P.n);
        (void)SDF_CHK(22, (unsigned long long)((long long)c32 + (pos ? 0 : 1) + std::max(dJ, 0ll) + std::max(dK, 0ll)), 0, P.n);
        const sp_u32x4 O = *(const sp_u32x4 *)b, Jp = *(const sp_u32x4 *)(b + dJ), Kp = *(const sp_u32x4 *)(b + dK),
                       JK = *(const sp_u32x4 *)(b + dJ + dK);
        // the cell is element 1 of its pairs for di > 0 (element 0 its i-upwind neighbour), element 0 for di < 0
        s = pos ? (((unsigned long long)O.w << 32) | O.z) : (((unsigned long long)O.y << 32) | O.x);
        const uint32_t w[7] = {pos ? O.x : O.z, pos ? Jp.z : Jp.x, pos ? Jp.x : Jp.z, pos ? Kp.z : Kp.x,
                               pos ? Kp.x : Kp.z, pos ? JK.z : JK.x, pos ? JK.x : JK.z};
        y = sp_eval_w<false>(P, i, j, k, s, w);
    } else {
        s = P.S[SDF_CHK(20, c32, P.c_lo, P.c_lo + P.n)];
        y = sp_eval<false, SLAB>(P, P.S, i, j, k, c32, s);
    }
    if (!P.sv) {
        P.X[SDF_CHK(21, c32, P.c_lo, P.c_lo + P.n)] = y;
    } else if (y != s) {   // in place: keep the pre-sweep value, then change the cell
        P.sv[SDF_CHK(21, c32, P.c_lo, P.c_lo + P.n)] = s;
        P.X[c32] = y;
    }
    if (lbl_of((uint32_t)y) != lbl_of((uint32_t)s)) {
        if (SLAB) sp_push(P, i, j, k, c32, (uint32_t)y);
        sp_request_collect(P, i, j, k, c32, false, qmask, tgt);
    }
}

__device__ __forceinline__ void sp_jlist_flush(const SpParams &P, unsigned part, const unsigned *buf, unsigned cnt,
                                               unsigned lane)
{
    sp_wave_sync();
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(&P.ctl[SP_JLIST + part * SP_JSTRIDE], (unsigned long long)cnt);
    b = __shfl(b, 0);
    unsigned *list = P.jlist + (size_t)part * P.jcap;
    for (unsigned t = lane; t < cnt; t += 64) {
        const unsigned c32 = buf[t];
        if (b + t < P.jcap) list[b + t] = c32;
        else atomicOr(&P.ctl[SP_ERR], 4ull);   // cannot happen: a part holds every cell its blocks visit
    }
    sp_wave_sync();
}

// FAST (one device, c_lo = 0, n <= 2^29 so that byte offsets fit 32 bits): the same traversal, with
//   * the cell and its 7 upwind words loaded with ONE 32-bit byte offset from eight scalar bases (the
//     neighbours' displacements folded into the bases: no address arithmetic per neighbour; a base
//     may point outside the grid, but only cells inside the sweep's range -- whose upwind neighbours
//     all exist -- load through it);
//   * the mask reduced to sp_any_scan (the list decision needs no more).
// 178 -> ~130 VALU per 64 cells: C3 scan 89.5 -> 76.2 us, C4 639 -> 629 us (profiles/r05aq_jscan_kernel_stats.txt).
// C4's scan sat at 95 % VALU issue (SQ) and is no faster with fewer VALU, nor with the next cell's loads
// issued before this cell's mask (75 % VALU issue then), nor in a (j, k, i) plane-range order (which
// slowed the list pass: its cells lost their address order).
template <bool SLAB, bool FAST = false>
__global__ void __launch_bounds__(256) k_sp_jacobi(SpParams P)
{
    static_assert(!(SLAB && FAST), "the fast scan is for one device");
    __shared__ unsigned s_list[4][SP_JWAVE];
    const unsigned lane = threadIdx.x & 63;
    const unsigned part = blockIdx.x % SP_JPARTS;   // part % 8 = this block's XCD
    unsigned *buf = s_list[threadIdx.x >> 6];
    unsigned cnt = 0;   // wave-uniform
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so XCD x walks the x-th
    // contiguous eighth of the grid -- the neighbour planes a cell reads sit in its own L2.
    const bool xcd = gridDim.x % 8 == 0;
    const unsigned long long span = xcd ? (P.n + 7) / 8 : P.n;
    const unsigned long long base = xcd ? (unsigned long long)(blockIdx.x % 8) * span : 0ull;
#if SP_JACOBI_CHUNK
    // Each block scans one contiguous chunk of its XCD's eighth, so blocks are dispatched in
    // address order and the upwind plane a cell reads was just read by the blocks before it: still
    // in the XCD's L2.  (A grid-stride loop over 2,048 blocks per XCD jumped 8 planes per step and
    // fetched S twice from HBM: 268 MB per launch at 256^3, PMC.)
    const unsigned long long nb = xcd ? gridDim.x / 8 : gridDim.x;
    const unsigned long long chunk = (span + nb * blockDim.x - 1) / (nb * blockDim.x) * blockDim.x;   // = per_block of sp_reserve
    const unsigned long long c_beg = (unsigned long long)(xcd ? blockIdx.x / 8 : blockIdx.x) * chunk;
    const unsigned long long c_end = std::min(span, c_beg + chunk);
    const unsigned long long first = c_beg + threadIdx.x;
    const unsigned long long step = blockDim.x;
#else
    const unsigned long long c_end = span;
    const unsigned long long first = (unsigned long long)(xcd ? blockIdx.x / 8 : blockIdx.x) * blockDim.x + threadIdx.x;
    const unsigned long long step = (unsigned long long)(xcd ? gridDim.x / 8 : gridDim.x) * blockDim.x;
#endif
    // (i, j, k) of the lane's cell: divided out once, then advanced by the stride's own
    // (si, sj, sk) with carries (two integer divisions per cell cost ~30 instructions)
    int i, j, k, si, sj, sk;
    {
        const unsigned c0 = (unsigned)(P.c_lo + base + first), r0 = c0 / (unsigned)P.ni;
        i = (int)(c0 % (unsigned)P.ni);
        j = (int)(r0 % (unsigned)P.nj);
        k = (int)(r0 / (unsigned)P.nj);
        const unsigned st = (unsigned)step, rs = st / (unsigned)P.ni;
        si = (int)(st % (unsigned)P.ni);
        sj = (int)(rs % (unsigned)P.nj);
        sk = (int)(rs / (unsigned)P.nj);
    }
    const char *nbase[7];   // FAST: the 7 upwind words' scalar bases
    long long off[7];
    if (FAST) {
        const long long di = P.di, dj = (long long)P.dj * P.ni, dk = (long long)P.dk * P.ni * P.nj;
        off[0] = -di; off[1] = -dj; off[2] = -di - dj; off[3] = -dk; off[4] = -di - dk; off[5] = -dj - dk;
        off[6] = -di - dj - dk;
#pragma unroll
        for (int q = 0; q < 7; ++q) nbase[q] = (const char *)(P.S + off[q]);   // (global pointers: no FLAT)
    }
    for (unsigned long long it = first; it - lane < c_end; it += step) {   // wave-uniform trip count
        const bool valid = it < c_end && base + it < P.n;
        const unsigned long long c = P.c_lo + base + it;
        const unsigned c32 = (unsigned)c;   // cells < 2^32 (sparse_sweep_supported)
        unsigned f = 0;
        if (FAST && valid) {
            const uint32_t boff = c32 << 3;   // < 2^32 (c < 2^29)
            (void)SDF_CHK(20, c, 0, P.n);
            const unsigned long long s = *(const unsigned long long *)((const char *)P.S + boff);
            if (sp_in(P, i, j, k)) {
                uint32_t w[7];
                uint32_t bo = boff;
                asm volatile("" : "+v"(bo));   // zero-extended in this block: the loads take the scalar-base form
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    (void)SDF_CHK(22, (unsigned long long)((long long)c + off[q]), 0, P.n);
                    w[q] = *(const uint32_t *)(nbase[q] + bo);
                }
                const bool interior = i >= 1 && i <= P.ni - 2 && j >= 1 && j <= P.nj - 2 && k >= 1 && k <= P.nk - 2;
                f = sp_any_scan(P, (uint32_t)s, w, interior) ? 1u : 0u;
            }
            if (!f && !P.sv) P.X[c] = s;   // (in place the cell already holds it)
        } else if (valid) {
            const unsigned long long s = P.S[c];
            int lab[7];
            if (sp_in(P, i, j, k)) f = sp_mask<false, SLAB>(P, P.S, i, j, k, c, s, lab);
            if (!f && !P.sv) P.X[c] = s;   // (in place the cell already holds it)
        }
        const unsigned long long want = __ballot(f != 0u);
        if (f) buf[cnt + __builtin_popcountll(want & ((1ull << lane) - 1ull))] = c32;
        cnt += (unsigned)__builtin_popcountll(want);
        if (cnt > SP_JWAVE - 64) {
            sp_jlist_flush(P, part, buf, cnt, lane);
            cnt = 0;
        }
        i += si;
        const int ci = i >= P.ni;
        i -= ci ? P.ni : 0;
        j += sj + ci;
        const int cj = j >= P.nj;
        j -= cj ? P.nj : 0;
        k += sk + cj;
    }
    if (cnt) sp_jlist_flush(P, part, buf, cnt, lane);
}

// The fast scan with 16-byte loads (SP_JSCAN_PAIR).  The scan's limiter is the texture addresser: TA busy
// 82 % (average over the chip's TA units, 96 % at the busiest) of the C4 launch's cycles while HBM ran at
// 2.8 TB/s and VALU issue at ~18 % (profiles/r06_limiter_c4.json); a wave-wide load costs the TA about the same
// per lane whatever its width (MI355X_MICROARCH.md: 8-B accesses 0.54-0.70x the 16-B rate), and k_sp_jacobi
// issued 8 of them per 64 cells: the cell (8 B) and its 7 upwind low words (4 B each).  Here a lane holds
// two consecutive cells (c, c + 1) and loads four 16-byte pairs -- its own, the j-upwind row's, the
// k-upwind plane's and the jk-diagonal's -- which hold every upwind word of both cells except the
// i-direction ones of one cell: those are the neighbouring lane's pair elements, moved by DPP (wave_shr:1 for
// di > 0, wave_shl:1 for di < 0; the wave's edge lane loads its four words itself).  4 wide loads per 128
// cells instead of 16 narrow ones.  Lanes whose pairs would leave the grid (its first planes / rows, and the
// last for negative directions) fill the pair registers word by word with bounds checks instead, so the DPP
// sources are right for every cell that needs them (a cell of the sweep's range has all its upwind words
// in the grid).  Same traversal (XCD eighths, one contiguous chunk per block), same list order (cells in
// address order), same decision (sp_any_scan): the list equals k_sp_jacobi<false, true>'s.
constexpr unsigned long long SP_PAD = 4;   // cells of padding past n in the state buffers (sp_pad)
inline unsigned long long sp_pad(unsigned long long n) { return n + SP_PAD; }

template <int NP>   // pairs per lane: 2 * NP consecutive cells, 4 * NP 16-byte loads issued together
__global__ void __launch_bounds__(256, NP == 1 ? 1 : 6) k_sp_jscan2(SpParams P)
{
    static_assert(NP >= 1 && 2 * NP <= SP_PAD + 1, "the last pair may read 2 NP - 1 cells past the grid");
    __shared__ unsigned s_list[4][SP_JWAVE];
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned part = blockIdx.x % SP_JPARTS;   // part % 8 = this block's XCD
    unsigned *buf = s_list[wv];
    unsigned cnt = 0;   // wave-uniform
    const unsigned long long span = (P.n + 7) / 8;   // launched with gridDim.x % 8 == 0 (sp_launch_jacobi)
    const unsigned long long base = (unsigned long long)(blockIdx.x % 8) * span;
    const unsigned long long nb = gridDim.x / 8;
    const unsigned long long chunk = (span + nb * blockDim.x - 1) / (nb * blockDim.x) * blockDim.x;
    const unsigned long long c_beg = (unsigned long long)(blockIdx.x / 8) * chunk;
    const unsigned long long c_end = std::min(span, c_beg + chunk);
    // an iteration covers 512 NP cells of the chunk: wave wv the 128 NP from wv * 128 NP, lane L 2 NP of them
    constexpr unsigned CL = 2 * NP, STEP = 512 * NP;
    const unsigned long long first = c_beg + wv * (128u * NP) + CL * lane;
    int i, j, k, si, sj, sk;
    {
        const unsigned c0 = (unsigned)(base + first), r0 = c0 / (unsigned)P.ni;
        i = (int)(c0 % (unsigned)P.ni);
        j = (int)(r0 % (unsigned)P.nj);
        k = (int)(r0 / (unsigned)P.nj);
        const unsigned rs = STEP / (unsigned)P.ni;
        si = (int)(STEP % (unsigned)P.ni);
        sj = (int)(rs % (unsigned)P.nj);
        sk = (int)(rs / (unsigned)P.nj);
    }
    const long long dJ = -(long long)P.dj * P.ni, dK = -(long long)P.dk * P.ni * P.nj;   // pair offsets (cells)
    const long long dlo = std::min(dJ, 0ll) + std::min(dK, 0ll), dhi = std::max(dJ, 0ll) + std::max(dK, 0ll);
    const char *bS = (const char *)P.S, *bJ = (const char *)(P.S + dJ), *bK = (const char *)(P.S + dK),
               *bJK = (const char *)(P.S + dJ + dK);   // (scalar bases; a base may lie outside the buffer)
    const bool pos = P.di > 0;
    const long long dI = pos ? -1ll : (long long)CL;   // (both signed: -1 : CL would be unsigned) the edge lane's own fetch: cell c + dI (+ the pair offsets)
    for (unsigned long long rel = first; rel - CL * lane < c_end; rel += STEP) {   // wave-uniform trip count
        const unsigned long long c = base + rel;
        sp_u32x4 O[NP], Jp[NP], Kp[NP], JK[NP];
        // every pair [x, x + 1] for x = c + 2p + {0, dJ, dK, dJ + dK} inside [0, n + SP_PAD)
        if ((long long)c + dlo >= 0 && (long long)c + CL - 1 + dhi <= (long long)(P.n + SP_PAD - 1)) {
            const uint32_t boff = (uint32_t)c << 3;   // c < 2^29
            (void)SDF_CHK(20, c, 0, P.n + SP_PAD);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                O[p] = *(const sp_u32x4 *)(bS + boff + 16 * p);
                Jp[p] = *(const sp_u32x4 *)(bJ + boff + 16 * p);
                Kp[p] = *(const sp_u32x4 *)(bK + boff + 16 * p);
                JK[p] = *(const sp_u32x4 *)(bJK + boff + 16 * p);
            }
        } else {   // the grid's edge: word by word, out-of-grid words 0 (no cell of the sweep's range reads them)
            auto ld = [&](long long x) -> unsigned long long {
                return (x >= 0 && x < (long long)P.n) ? P.S[SDF_CHK(22, x, 0, P.n)] : 0ull;
            };
            auto pair = [&](long long x) {
                const unsigned long long a = ld(x), b = ld(x + 1);
                return sp_u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
            };
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const long long cc = (long long)c + 2 * p;
                O[p] = pair(cc);
                Jp[p] = pair(cc + dJ);
                Kp[p] = pair(cc + dK);
                JK[p] = pair(cc + dJ + dK);
            }
        }
        // the i-upwind words of the lane's first cell (di > 0: cell c - 1) or last (di < 0: cell c + 2 NP) come
        // from the neighbouring lane by DPP; the wave's edge lane fetches its own
        uint32_t e0 = 0u, e1 = 0u, e2 = 0u, e3 = 0u;
        if (lane == (pos ? 0u : 63u)) {
            const long long x = (long long)c + dI;
            auto ld1 = [&](long long y) -> uint32_t {
                return (y >= 0 && y < (long long)P.n) ? (uint32_t)P.S[SDF_CHK(22, y, 0, P.n)] : 0u;
            };
            e0 = ld1(x);
            e1 = ld1(x + dJ);
            e2 = ld1(x + dK);
            e3 = ld1(x + dJ + dK);
        }
        uint32_t t0, t1, t2, t3;
        if (pos) {   // wave_shr:1 -- lane L takes lane L - 1's last cell; lane 0 keeps its own fetch
            t0 = (uint32_t)__builtin_amdgcn_update_dpp((int)e0, (int)O[NP - 1].z, 0x138, 0xf, 0xf, false);
            t1 = (uint32_t)__builtin_amdgcn_update_dpp((int)e1, (int)Jp[NP - 1].z, 0x138, 0xf, 0xf, false);
            t2 = (uint32_t)__builtin_amdgcn_update_dpp((int)e2, (int)Kp[NP - 1].z, 0x138, 0xf, 0xf, false);
            t3 = (uint32_t)__builtin_amdgcn_update_dpp((int)e3, (int)JK[NP - 1].z, 0x138, 0xf, 0xf, false);
        } else {     // wave_shl:1 -- lane L takes lane L + 1's first cell; lane 63 keeps its own fetch
            t0 = (uint32_t)__builtin_amdgcn_update_dpp((int)e0, (int)O[0].x, 0x130, 0xf, 0xf, false);
            t1 = (uint32_t)__builtin_amdgcn_update_dpp((int)e1, (int)Jp[0].x, 0x130, 0xf, 0xf, false);
            t2 = (uint32_t)__builtin_amdgcn_update_dpp((int)e2, (int)Kp[0].x, 0x130, 0xf, 0xf, false);
            t3 = (uint32_t)__builtin_amdgcn_update_dpp((int)e3, (int)JK[0].x, 0x130, 0xf, 0xf, false);
        }
        unsigned f[CL];
        int ic = i, jc = j, kc = k;   // coordinates of cell c + m, advanced along the row
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            const int p = m >> 1;
            const bool hi = m & 1;
            // this cell's words and its i-upwind cell's (q: i, j, ij, k, ik, jk, ijk; k_sp_jacobi's off[])
            const uint32_t wo = hi ? O[p].z : O[p].x, wj = hi ? Jp[p].z : Jp[p].x, wk = hi ? Kp[p].z : Kp[p].x,
                           wjk = hi ? JK[p].z : JK[p].x;
            uint32_t ui, uj, uk, ujk;   // the i-upwind cell's words
            if (pos) {
                if (m == 0) { ui = t0; uj = t1; uk = t2; ujk = t3; }
                else if (hi) { ui = O[p].x; uj = Jp[p].x; uk = Kp[p].x; ujk = JK[p].x; }
                else { ui = O[p - 1].z; uj = Jp[p - 1].z; uk = Kp[p - 1].z; ujk = JK[p - 1].z; }
            } else {
                if (m == CL - 1) { ui = t0; uj = t1; uk = t2; ujk = t3; }
                else if (!hi) { ui = O[p].z; uj = Jp[p].z; uk = Kp[p].z; ujk = JK[p].z; }
                else { ui = O[p + 1].x; uj = Jp[p + 1].x; uk = Kp[p + 1].x; ujk = JK[p + 1].x; }
            }
            const bool v = rel + m < c_end && c + m < P.n;
            f[m] = 0u;
            if (v && sp_in(P, ic, jc, kc)) {
                const uint32_t w[7] = {ui, wj, uj, wk, uk, wjk, ujk};
                const bool interior = ic >= 1 && ic <= P.ni - 2 && jc >= 1 && jc <= P.nj - 2 && kc >= 1 && kc <= P.nk - 2;
                f[m] = sp_any_scan(P, wo, w, interior) ? 1u : 0u;
            }
            if (!P.sv && v && !f[m])   // two buffers: cells that keep their value are copied (in place they hold it)
                P.X[c + m] = ((unsigned long long)(hi ? O[p].w : O[p].y) << 32) | wo;
            if (++ic == P.ni) {
                ic = 0;
                if (++jc == P.nj) { jc = 0; ++kc; }
            }
        }
        // the list in address order: lane L's cells after those of lanes < L
        const unsigned long long lt = (1ull << lane) - 1ull;
        unsigned at = cnt, tot = 0;
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            const unsigned long long bm = __ballot(f[m] != 0u);
            at += (unsigned)__builtin_popcountll(bm & lt);
            tot += (unsigned)__builtin_popcountll(bm);
        }
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            if (f[m]) buf[at] = (unsigned)(c + m);
            at += f[m];
        }
        cnt += tot;
        if (cnt > SP_JWAVE - 64 * CL) {
            sp_jlist_flush(P, part, buf, cnt, lane);
            cnt = 0;
        }
        i += si;
        const int ci = i >= P.ni;
        i -= ci ? P.ni : 0;
        j += sj + ci;
        const int cj = j >= P.nj;
        j -= cj ? P.nj : 0;
        k += sk + cj;
    }
    if (cnt) sp_jlist_flush(P, part, buf, cnt, lane);
}

// The pair scan streaming along k (SP_JSCAN_K).  k_sp_jscan2 loads four pair streams per lane: its own, the
// j-upwind row's, the k-upwind plane's and the jk diagonal's; the last two are the first two of the plane
// before.  Here a wave owns one row segment of 64 x 2 NP cells (i) and walks a chunk of KC planes in the
// sweep's k order, upwind first, so the plane it needs as k-upwind is the one it held in the previous
// iteration: its k and jk pairs are the previous O and Jp (registers), and a plane costs two pair loads per
// lane instead of four (the chunk's first plane: four).  The j-upwind row is the block's next wave's own row
// (a workgroup is 4 consecutive rows), loaded again from L1 / L2.  Blocks: XCD x = blockIdx % 8 takes the
// x-th eighth of the (k-chunk, row group, segment) items, so a block's neighbours are on its XCD.  Same
// decision (sp_any_scan) for the same cells, so the same list SET as k_sp_jacobi's; its order is per row
// segment and plane (k_sp_jlist evaluates each listed cell independently, and the repair's result does not
// depend on the order of its requests: the header's uniqueness argument).
struct SpKGeom {
    unsigned nseg, nrg, kc, items, per_xcd;   // row segments per row, row groups (4 rows), planes per chunk, items
};
inline SpKGeom sp_kgeom(int ni, int nj, int nk, int np)
{
    SpKGeom G;
    const unsigned rw = 128u * (unsigned)np;
    G.nseg = ((unsigned)ni + rw - 1) / rw;
    G.nrg = ((unsigned)nj + 3) / 4;
    // about 16,384 items, 4..64 planes each: at C4 8 planes per chunk (scan + list pass per sweep, rocprof:
    // 4 planes 453 + 336, 8 planes 435 + 338, 32 planes 444 + 340, 128 planes 557 + 393 us; k_sp_jscan2 521 + 309,
    // profiles/r06o_kc_c4.txt); C3 takes the minimum, 4
    const unsigned long long cols = (unsigned long long)G.nseg * G.nrg;
    G.kc = (unsigned)std::max<unsigned long long>(4, std::min<unsigned long long>(64, cols * (unsigned long long)nk / 16384));
    if (const char *e = getenv("SDFGEN_JSCAN_KC")) G.kc = (unsigned)std::max(1, std::min(nk, atoi(e)));   // (diagnostics)
    G.items = (unsigned)(((unsigned long long)nk + G.kc - 1) / G.kc * cols);
    G.per_xcd = (G.items + 7) / 8;
    return G;
}
inline unsigned long long sp_kgeom_cells_per_block(const SpKGeom &G, int np) { return (unsigned long long)G.kc * 4 * 128 * np; }
// the k-streaming scan runs on a whole grid on one device whose cell indices fit the list's 32 bits
inline bool sp_kscan_ok(unsigned long long c_lo, unsigned long long n, int ni, int nj, int nk)
{
    return SP_JSCAN_FAST && c_lo == 0 && n == (unsigned long long)ni * nj * nk && n + SP_PAD < (1ull << 32);
}

template <int NP, bool WIDE>   // WIDE: 64-bit byte offsets (grids above 2^29 cells: C5)
__global__ void __launch_bounds__(256, NP == 1 ? 1 : 6) k_sp_jscan3(SpParams P, SpKGeom G)
{
    __shared__ unsigned s_list[4][SP_JWAVE];
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned part = blockIdx.x % SP_JPARTS;   // part % 8 = this block's XCD (k_sp_jlist's blocks of the part run there)
    unsigned *buf = s_list[wv];
    unsigned cnt = 0;   // wave-uniform
    constexpr unsigned CL = 2 * NP, RW = 64 * CL;
    const unsigned item = (blockIdx.x % 8) * G.per_xcd + blockIdx.x / 8;
    const int j = (int)((item / G.nseg) % G.nrg) * 4 + (int)wv;   // this wave's row
    if (item >= G.items || j >= P.nj) return;   // (no workgroup barrier below: a wave may leave)
    const unsigned seg = item % G.nseg, kch = item / (G.nseg * G.nrg);
    const int i0 = (int)(seg * RW + CL * lane);   // the lane's first cell in the row
    const bool lane_in = i0 < P.ni;                // lanes past the row end load the wave's first pair (never used)
    const long long dJ = -(long long)P.dj * P.ni, dK = -(long long)P.dk * P.ni * P.nj;   // pair offsets (cells)
    const bool hasJ = (unsigned)(j - P.dj) < (unsigned)P.nj;   // the j-upwind row exists (else no cell of it is in range)
    const char *bS = (const char *)P.S, *bJ = (const char *)(P.S + dJ), *bK = (const char *)(P.S + dK),
               *bJK = (const char *)(P.S + dJ + dK);   // (scalar bases; a base may lie outside the buffer)
    const bool pos = P.di > 0;
    const long long dI = pos ? -1ll : (long long)CL;   // the edge lane's own fetch: cell c + dI
    const unsigned ip = (unsigned)(pos ? i0 : i0 + CL - 1);   // (unused: keeps the edge cell's row test cheap)
    (void)ip;
    sp_u32x4 O[NP], Jp[NP], Kp[NP], JK[NP];
    uint32_t e0 = 0u, e1 = 0u, e2 = 0u, e3 = 0u;   // the edge lane's i-upwind words (O, J, K, JK)
    const int kk0 = (int)(kch * G.kc), kk1 = min(P.nk, kk0 + (int)G.kc);
    for (int kk = kk0; kk < kk1; ++kk) {   // wave-uniform
        const int k = P.dk > 0 ? kk : P.nk - 1 - kk;   // planes in the sweep's order: upwind first
        const long long crow = (long long)P.ni * (j + (long long)P.nj * k);   // the row's first cell
        const unsigned long long c = (unsigned long long)(crow + (lane_in ? i0 : (int)(seg * RW)));
        const uint32_t boff32 = (uint32_t)c << 3;   // (c < 2^29 unless WIDE)
        const unsigned long long boff = WIDE ? c << 3 : (unsigned long long)boff32;
        (void)SDF_CHK(20, c, 0, P.n + SP_PAD);
        const bool first = kk == kk0;
        const bool hasK = (unsigned)(k - P.dk) < (unsigned)P.nk;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (!first) { Kp[p] = O[p]; JK[p] = Jp[p]; }
            O[p] = *(const sp_u32x4 *)(bS + boff + 16 * p);
            Jp[p] = hasJ ? *(const sp_u32x4 *)(bJ + boff + 16 * p) : sp_u32x4{0u, 0u, 0u, 0u};
            if (first) {
                Kp[p] = hasK ? *(const sp_u32x4 *)(bK + boff + 16 * p) : sp_u32x4{0u, 0u, 0u, 0u};
                JK[p] = (hasK && hasJ) ? *(const sp_u32x4 *)(bJK + boff + 16 * p) : sp_u32x4{0u, 0u, 0u, 0u};
            }
        }
        if (lane == (pos ? 0u : 63u)) {
            const long long x = (long long)c + dI;
            auto ld1 = [&](long long y) -> uint32_t {
                return (y >= 0 && y < (long long)P.n) ? (uint32_t)P.S[SDF_CHK(22, y, 0, P.n)] : 0u;
            };
            if (!first) { e2 = e0; e3 = e1; }
            e0 = ld1(x);
            e1 = hasJ ? ld1(x + dJ) : 0u;
            if (first) {
                e2 = hasK ? ld1(x + dK) : 0u;
                e3 = (hasK && hasJ) ? ld1(x + dJ + dK) : 0u;
            }
        }
        uint32_t t0, t1, t2, t3;
        if (pos) {   // wave_shr:1 -- lane L takes lane L - 1's last cell; lane 0 keeps its own fetch
            t0 = (uint32_t)__builtin_amdgcn_update_dpp((int)e0, (int)O[NP - 1].z, 0x138, 0xf, 0xf, false);
            t1 = (uint32_t)__builtin_amdgcn_update_dpp((int)e1, (int)Jp[NP - 1].z, 0x138, 0xf, 0xf, false);
            t2 = (uint32_t)__builtin_amdgcn_update_dpp((int)e2, (int)Kp[NP - 1].z, 0x138, 0xf, 0xf, false);
            t3 = (uint32_t)__builtin_amdgcn_update_dpp((int)e3, (int)JK[NP - 1].z, 0x138, 0xf, 0xf, false);
        } else {     // wave_shl:1 -- lane L takes lane L + 1's first cell; lane 63 keeps its own fetch
            t0 = (uint32_t)__builtin_amdgcn_update_dpp((int)e0, (int)O[0].x, 0x130, 0xf, 0xf, false);
            t1 = (uint32_t)__builtin_amdgcn_update_dpp((int)e1, (int)Jp[0].x, 0x130, 0xf, 0xf, false);
            t2 = (uint32_t)__builtin_amdgcn_update_dpp((int)e2, (int)Kp[0].x, 0x130, 0xf, 0xf, false);
            t3 = (uint32_t)__builtin_amdgcn_update_dpp((int)e3, (int)JK[0].x, 0x130, 0xf, 0xf, false);
        }
        unsigned f[CL];
        const bool jk_in = (P.dj > 0 ? j >= 1 : j <= P.nj - 2) && (P.dk > 0 ? k >= 1 : k <= P.nk - 2);
        const bool jk_interior = j >= 1 && j <= P.nj - 2 && k >= 1 && k <= P.nk - 2;
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            const int p = m >> 1;
            const bool hi = m & 1;
            const int ic = i0 + m;
            const uint32_t wo = hi ? O[p].z : O[p].x, wj = hi ? Jp[p].z : Jp[p].x, wk = hi ? Kp[p].z : Kp[p].x,
                           wjk = hi ? JK[p].z : JK[p].x;
            uint32_t ui, uj, uk, ujk;   // the i-upwind cell's words
            if (pos) {
                if (m == 0) { ui = t0; uj = t1; uk = t2; ujk = t3; }
                else if (hi) { ui = O[p].x; uj = Jp[p].x; uk = Kp[p].x; ujk = JK[p].x; }
                else { ui = O[p - 1].z; uj = Jp[p - 1].z; uk = Kp[p - 1].z; ujk = JK[p - 1].z; }
            } else {
                if (m == CL - 1) { ui = t0; uj = t1; uk = t2; ujk = t3; }
                else if (!hi) { ui = O[p].z; uj = Jp[p].z; uk = Kp[p].z; ujk = JK[p].z; }
                else { ui = O[p + 1].x; uj = Jp[p + 1].x; uk = Kp[p + 1].x; ujk = JK[p + 1].x; }
            }
            const bool v = lane_in && ic < P.ni;
            f[m] = 0u;
            if (v && jk_in && (pos ? ic >= 1 : ic <= P.ni - 2)) {
                const uint32_t w[7] = {ui, wj, uj, wk, uk, wjk, ujk};
                const bool interior = jk_interior && ic >= 1 && ic <= P.ni - 2;
                f[m] = sp_any_scan(P, wo, w, interior) ? 1u : 0u;
            }
            if (!P.sv && v && !f[m])   // two buffers: cells that keep their value are copied (in place they hold it)
                P.X[c + m] = ((unsigned long long)(hi ? O[p].w : O[p].y) << 32) | wo;
        }
        // the list: lane L's cells after those of lanes < L (the row segment in address order)
        const unsigned long long lt = (1ull << lane) - 1ull;
        unsigned at = cnt, tot = 0;
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            const unsigned long long bm = __ballot(f[m] != 0u);
            at += (unsigned)__builtin_popcountll(bm & lt);
            tot += (unsigned)__builtin_popcountll(bm);
        }
#pragma unroll
        for (int m = 0; m < CL; ++m) {
            if (f[m]) buf[at] = (unsigned)(c + m);
            at += f[m];
        }
        cnt += tot;
        if (cnt > SP_JWAVE - 64 * CL) {
            sp_jlist_flush(P, part, buf, cnt, lane);
            cnt = 0;
        }
    }
    if (cnt) sp_jlist_flush(P, part, buf, cnt, lane);
}

// Pass 1b: the listed cells, each exactly as in place (sp_eval against S).
// Z-slab: it pushes into the neighbours' live halos, so it runs after k_sp_slab_wait saw both
// neighbours READY.
template <bool SLAB, bool PAIR = false>
__global__ void __launch_bounds__(256) k_sp_jlist(SpParams P)
{
    const unsigned part = blockIdx.x % SP_JPARTS;
    const unsigned long long cnt0 = P.ctl[SP_JLIST + part * SP_JSTRIDE];
    const unsigned long long cnt = cnt0 < P.jcap ? cnt0 : P.jcap;
    const unsigned *list = P.jlist + (size_t)part * P.jcap;
    const unsigned lane = threadIdx.x & 63;
    // wave-uniform trip count: the queue appends are wave-level (sp_append_wave)
    for (unsigned long long x = (unsigned long long)(blockIdx.x / SP_JPARTS) * blockDim.x + threadIdx.x; x - lane < cnt;
         x += (unsigned long long)(gridDim.x / SP_JPARTS) * blockDim.x) {
        unsigned qmask = 0;
        size_t tgt[7];
        if (x < cnt) sp_jacobi_cell<SLAB, PAIR>(P, list[x], &qmask, tgt);
        sp_append_wave(P, (unsigned)(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) & (P.nq - 1u)), qmask, tgt, false);
    }
}

// Pass 2: drain the recheck work list.  One lane = one worker; chains are followed depth-first by
// the lane that changed the upstream cell.  Written as a flat loop in which every lane does at
// most one poll or one evaluation per iteration: a lane spinning on an empty slot must never hold
// back (SIMT reconvergence) lanes of its own wave whose work would fill that slot.  Queue traffic
// is per wave: one ticket atomic for all lanes that need work, one read of the shard's tail word
// (lanes poll their slot only once the tail has passed it, and the same word says when the shard
// has drained), one append atomic for all lanes' new items and finished ones.
//
// Z-slab: the lanes of workgroup 0 also drain the inbound ring (cells of the upstream slab's last
// plane that changed label; their live halo words are already in place): each entry becomes
// requests for this slab's first-plane cells downstream of it.  A lane's inbound part is finished
// once the upstream slab's repair has ended (its DONE flag) and every entry it appended (its
// COUNT) is taken; local lanes stop only after all SP_INLANES inbound lanes finished and nothing is
// queued or running.  The last wave to leave tells the downstream slab (COUNT, then DONE) and the
// upstream slab (DONE: our pushes into its halo for its next sweep are in place).
template <bool SLAB>
__global__ void __launch_bounds__(64) k_sp_recheck(SpParams P)
{
    constexpr size_t NONE = ~(size_t)0;
    __shared__ unsigned s_hand[64];   // sp_hand_local
    unsigned long long runs = 0, claims = 0, h = 0, h_in = 0;
    size_t e = NONE, next = NONE;
    unsigned rq = 1;
    bool done = false, waiting = false, in_wait = false;
    bool in_role = SLAB && P.in_ring != nullptr && blockIdx.x == 0;   // still draining the inbound ring
    unsigned spins = 0, in_spins = 0;
    const unsigned lane = threadIdx.x & 63;
    const unsigned long long lane_lt = (1ull << lane) - 1ull;
    // hand-off lanes take work only from their own wave (sp_hand_local), never ring tickets: a
    // ticket holder is bound to its ring slot.  They leave with the wave once its ring lanes saw the
    // shard drain (their cells count as pending there, so a drained shard has none running).
    const bool local = lane >= 64u - (unsigned)SP_LOCAL_LANES;
    const unsigned shard = blockIdx.x & (P.nq - 1u);   // this wave's home work-list shard
    unsigned long long *const q_tail = &P.ctl[SP_SHARD0 + shard * SP_SHSTRIDE];   // pending << 32 | tail
    unsigned long long *const q_head = q_tail + 16;
    unsigned *const ring = P.queue + (size_t)shard * P.cap;
    unsigned long long t_start = 0, n_in = 0;   // Z-slab phase timers (TM_*)
    if (SLAB && P.tm) {
        t_start = wall_clock64();
        if (blockIdx.x == 0 && lane == 0) P.tm[TM_REPAIR_T0 + P.tm_m] = t_start;
    }
#if SP_SPLIT_APPEND
    SpAppend app;
    app.live = false;
    app.old_q = 0;   // read by the unconditional wait of sp_append_finish before the first issue
    size_t tgt_app[7];   // the cells of the append in flight
#endif
#ifdef SP_ITER_PROF   // diagnostics: cycles per phase of an iteration, busy (>= 1 lane evaluates) or idle
    unsigned long long ip_b[12] = {}, ip_i[12] = {}, ip_d[12], ip_t = 0, ip_nb = 0, ip_ni = 0;
#define SP_IP(q) do { const unsigned long long t2_ = clock64(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); ip_d[q] = t2_ - ip_t; ip_t = t2_; } while (0)
#else
#define SP_IP(q) do { } while (0)
#endif
    for (;;) {
        unsigned qmask = 0;   // cells this lane queues this iteration (sp_append_wave below)
        size_t tgt[7];
        bool fin = false;     // this lane's work item ended this iteration
#ifdef SP_ITER_PROF
        for (int q = 0; q < 12; ++q) ip_d[q] = 0;
        ip_t = clock64();
#endif
        {
            // queue tickets for every lane that needs one: ONE atomic on the head word per wave
            const bool busy_wave = SP_BUSY_NO_TICKET && __any(e != NONE);   // (wave-uniform, all lanes)
            const bool want = !done && e == NONE && !waiting && !(SLAB && in_role) && !local && !busy_wave;
            const unsigned long long wm = __ballot(want);
            if (wm) {
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(q_head, (unsigned long long)__popcll(wm));
                base = ((unsigned long long)(unsigned)__shfl((int)(base >> 32), 0) << 32) | (unsigned)__shfl((int)base, 0);
                if (want) {
                    h = base + (unsigned long long)__popcll(wm & lane_lt);
                    waiting = true;
                }
            }
        }
        SP_IP(0);
        // SP_DIRECT_POLL: a waiting ring lane's slot poll is issued first, so that it and the tail read
        // below share one round trip (the tail then only decides the shard's drain)
        unsigned vpoll = 0u;
        if (SP_DIRECT_POLL && !done && e == NONE && waiting && !local && !(SLAB && in_role))
            vpoll = sp_ld32(ring + sp_slot(h, P.cap));
        // the shard's tail word, read once for the wave's waiting lanes
        unsigned long long qw = 0;
        bool tail_read = false;   // wave-uniform
        if (__any(!done && e == NONE && waiting && !(SLAB && in_role)) && !(SP_BUSY_NO_TAIL && __any(e != NONE))) {
            if (lane == 0) qw = sp_ld64(q_tail);
            qw = ((unsigned long long)(unsigned)__shfl((int)(qw >> 32), 0) << 32) | (unsigned)__shfl((int)qw, 0);
            tail_read = true;
        }
        SP_IP(1);
#if SP_SPLIT_APPEND && !SP_LATE_APPEND
        sp_append_finish(P, shard, tgt_app, app);   // last iteration's append (its atomic overlapped the above)
#endif
        SP_IP(2);
        if (SLAB && in_role && e == NONE) {
            if (!in_wait) {
                h_in = atomicAdd(&P.ctl[SP_INHEAD], 1ull);
                in_wait = true;
            }
            const unsigned v = h_in < P.ring_cap ? __hip_atomic_load(P.in_ring + h_in, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            if (v) {
                __hip_atomic_store(P.in_ring + h_in, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                in_wait = false;
                in_spins = 0;
                ++n_in;
                const unsigned u = v - 1;   // an upstream cell: its downstream cells here are queued
                const int iu = (int)(u % (unsigned)P.ni);
                const unsigned ru = u / (unsigned)P.ni;
                sp_request_collect(P, iu, (int)(ru % (unsigned)P.nj), (int)(ru / (unsigned)P.nj), u, false, &qmask, tgt);
            } else if (__hip_atomic_load(P.flags + (SP_FL_DONE + P.up_side) * SP_FL_STRIDE, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) >= P.epoch &&
                       h_in >= __hip_atomic_load(P.flags + (SP_FL_COUNT + P.up_side) * SP_FL_STRIDE,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                in_role = false;   // DONE is written after COUNT: nothing more can come
                sp_order();
                atomicAdd(&P.ctl[SP_INDONE], 1ull);
                if (P.tm) {
                    atomicMax(P.tm + TM_INBOUND + P.tm_m, wall_clock64() - t_start);
                    if (n_in) atomicAdd(P.tm + TM_INBOUND_N + P.tm_m, n_in);
                }
            } else if (++in_spins > SP_WATCHDOG || ((in_spins & 255u) == 255u && (sp_ld64(&P.ctl[SP_ERR]) & 16ull))) {
                atomicOr(&P.ctl[SP_ERR], 16ull);
                in_role = false;
                atomicAdd(&P.ctl[SP_INDONE], 1ull);
            }
        } else if (!done && e == NONE && !local) {   // a ring lane: its ticket's slot
            // SP_DIRECT_POLL: the slot is polled every iteration, in the same round trip as the tail read
            // (a slot not yet appended, or appended but not yet stored, reads 0: every slot a sweep uses is
            // zeroed by its taker, and positions restart at 0 each sweep); otherwise only once the tail has
            // passed it (appended; its store may still land) -- a second round trip per pick-up
            const unsigned v = SP_DIRECT_POLL ? vpoll : (h < (qw & 0xffffffffull) ? sp_ld32(ring + sp_slot(h, P.cap)) : 0u);
            if (v) {
                sp_st32(ring + sp_slot(h, P.cap), 0u);
                e = SDF_CHK(28, v - 1, P.c_lo, P.c_lo + P.n);
                next = NONE;
                rq = 1;
                waiting = false;
                spins = 0;
            } else if (tail_read && (qw >> 32) == 0ull &&
                       (!SLAB || !P.in_ring || sp_ld64(&P.ctl[SP_INDONE]) >= (unsigned long long)SP_INLANES)) {
                done = true;   // nothing queued or running in this shard (nor to come): no slot can fill any more
            } else if (++spins > SP_WATCHDOG) {
                atomicOr(&P.ctl[SP_ERR], 1ull);
                done = true;
            }
        }
        SP_IP(3);
        // (profile: the stamps are per lane -- a lane outside the busy block keeps its last stamp --
        // so a busy iteration is reported from its first busy lane)
        const unsigned long long ip_bm = __ballot(e != NONE);
        const bool ip_busy = ip_bm != 0ull;
        (void)ip_busy;
        if (e != NONE) {
            // one evaluation of cell e, retiring `rq` requests
            const int i = (int)((unsigned)e % (unsigned)P.ni);
            const unsigned r0 = (unsigned)e / (unsigned)P.ni;
            const int j = (int)(r0 % (unsigned)P.nj), k = (int)(r0 / (unsigned)P.nj);
            // The upwind words, the cell's current value and its pre-sweep copy are issued together:
            // ONE round trip (the cell's current value used to be waited for first, then its copy with
            // the neighbours: two).  Reading sv before knowing the cell moved is safe: whoever changed
            // the cell stored sv, then X, then fenced before retiring the request we observed.
            uint32_t w[7];
            sp_nb_words<true, SLAB>(P, P.X, i, j, k, e, w);
            const unsigned long long cur = sp_ld64(P.X + SDF_CHK(25, e, P.c_lo, P.c_lo + P.n));
            const unsigned long long pre = P.sv ? sp_ld64(P.sv + e) : P.S[e];
            // f's own input is the cell's pre-sweep value: in place, a cell stamped with this sweep
            // has changed already and keeps it in sv
            const bool moved = P.sv && lc_of((uint32_t)cur) == P.sweep + 1;
#ifdef SP_NOEVAL_RECHECK   // diagnostics: the work list's own cost (no evaluation, no relabel)
            const unsigned long long y = cur;
            (void)w;
            (void)pre;
#else
            const unsigned long long own = !P.sv ? pre : moved ? pre : cur;
            const unsigned long long y = sp_eval_w<true>(P, i, j, k, own, w);
#endif
            ++runs;
            const bool relabel = y != cur && lbl_of((uint32_t)y) != lbl_of((uint32_t)cur);
            SP_IP(4);
            if (y != cur) {
                if (P.sv && !moved) sp_st64(P.sv + e, cur);   // its first change in this sweep
                sp_st64(P.X + e, y);
                if (relabel || P.sv) sp_order();   // the new label (and sv) are visible before anyone reads them
            }
            if (SLAB && relabel) sp_push(P, i, j, k, e, (uint32_t)y);
            SP_IP(5);
            // retire e's requests and ask for the downstream rechecks in one round trip
            const unsigned old = atomicSub(P.req + e, rq);
            if (relabel) {
                const size_t m = sp_request_collect(P, i, j, k, e, next == NONE, &qmask, tgt);
                if (m != NONE) next = m;
            }
            if (old == rq) {   // no request arrived meanwhile: e is settled
                if (next != NONE) {
                    e = next;   // the work item's pending count carries over to the claimed cell
                    next = NONE;
                    rq = 1;
                    ++claims;
                } else {
                    e = NONE;
                    fin = true;   // retired in sp_append_wave, in the same atomic as the wave's new items
                }
            } else {
                rq = old - rq;   // evaluate again for the requests that arrived meanwhile
                sp_order();
            }
#ifdef SP_ITER_PROF
            sp_order();   // (profile only: the request atomics' returns land inside phase 6)
#endif
            SP_IP(6);
        }
#ifdef SP_ITER_PROF
        { const unsigned long long t2_ = clock64(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); ip_d[11] += t2_ - ip_t; ip_t = t2_; }   // (join)
#endif
        unsigned nloc = 0;
        if (SP_LOCAL_LANES) {
            size_t got = NONE;
#ifdef SP_ITER_PROF
            nloc = sp_hand_local(s_hand, &qmask, tgt, local && !done && e == NONE && !(SLAB && in_role), &got, &ip_t, ip_d);
#else
            nloc = sp_hand_local(s_hand, &qmask, tgt, local && !done && e == NONE && !(SLAB && in_role), &got);
#endif
            if (got != NONE) {
                e = SDF_CHK(28, got, P.c_lo, P.c_lo + P.n);   // owned: its counter moved 0 -> 1 for the requester
                next = NONE;
                rq = 1;
            }
        }
        const bool idle_local = local && e == NONE && !(SLAB && in_role);
        SP_IP(7);
#if SP_SPLIT_APPEND
#if SP_LATE_APPEND
        sp_append_finish(P, shard, tgt_app, app);   // last iteration's append: its atomic overlapped this whole iteration
#endif
        sp_append_issue(P, shard, qmask, fin, nloc, app);
        SP_IP(8);
        if (app.live) {
#pragma unroll
            for (int q = 0; q < 7; ++q) tgt_app[q] = tgt[q];
        }
        if (__all(done || idle_local)) {
            sp_append_finish(P, shard, tgt_app, app);
            break;
        }
#else
        sp_append_wave(P, shard, qmask, tgt, fin, nloc);
        if (__all(done || idle_local)) break;
#endif
        if (SP_IDLE_SLEEP && !__any(e != NONE)) __builtin_amdgcn_s_sleep(SP_IDLE_SLEEP);
#ifdef SP_ITER_PROF
        SP_IP(10);   // (phase 9: hand-off ballots, 11: hand-off slot writes; 7: the rest of the hand-off)
        {
            const int src = ip_busy ? __ffsll((long long)ip_bm) - 1 : 0;
            for (int q = 0; q < 12; ++q) {
                const unsigned long long v = ((unsigned long long)(unsigned)__shfl((int)(ip_d[q] >> 32), src) << 32) |
                                             (unsigned)__shfl((int)ip_d[q], src);
                if (ip_busy) ip_b[q] += v;
                else ip_i[q] += v;
            }
        }
        if (ip_busy) ++ip_nb;
        else ++ip_ni;
#endif
    }
#ifdef SP_ITER_PROF
    if (lane == 0) {
        for (int q = 0; q < 12; ++q) {
            atomicAdd(&P.ctl[SP_DIAGX + q], ip_b[q]);
            atomicAdd(&P.ctl[SP_DIAGX + 12 + q], ip_i[q]);
        }
        atomicAdd(&P.ctl[SP_DIAGX + 24], ip_nb);
        atomicAdd(&P.ctl[SP_DIAGX + 25], ip_ni);
    }
#endif
    if (runs) atomicAdd(&P.ctl[SP_RUNS], runs);
    if (claims) atomicAdd(&P.ctl[SP_ENQ], claims);
    if (SLAB) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every push of this wave has landed
        if ((threadIdx.x & 63) == 0 && atomicAdd(&P.ctl[SP_EXIT], 1ull) == gridDim.x - 1ull) {
            if (P.tm) P.tm[TM_REPAIR + P.tm_m] = wall_clock64() - sp_ld64(P.tm + TM_REPAIR_T0 + P.tm_m);
            if (P.down_flags) {
                __hip_atomic_store(P.down_flags + (SP_FL_COUNT + P.up_side) * SP_FL_STRIDE, sp_ld64(&P.ctl[SP_OUTTAIL]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(P.down_flags + (SP_FL_DONE + P.up_side) * SP_FL_STRIDE, P.epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (P.up_flags)
                __hip_atomic_store(P.up_flags + (SP_FL_DONE + 1 - P.up_side) * SP_FL_STRIDE, P.epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Z-slab, around each sparse sweep:
//   k_sp_slab_wait(DONE, previous epoch)  both neighbours finished the previous sweep: their pushes
//                                         into our halo planes are in place;
//   k_sp_slab_halo                        the live halos start as copies of the pre-sweep ones, then
//                                         the neighbours are told they may push (READY);
//   k_sp_jacobi                           (no pushes)
//   k_sp_slab_wait(READY, this epoch)     both neighbours' live halos are initialised;
//   k_sp_jlist, k_sp_recheck              (push).
// The waits are one-workgroup launches: a wide launch whose blocks spin could starve a neighbour
// slab sharing the device (the one-GPU tests) of the slots it needs to make progress.
struct SpHaloParams {
    const uint32_t *hS[2];                     // [side] pre-sweep halo planes (ni*nj low words)
    uint32_t *hX[2];                           // [side] live halo planes
    unsigned long long plane;
    unsigned long long *flags;                 // ours (written by the neighbours)
    unsigned long long *nb_flags[2];           // the lower / upper neighbour's (null: none)
    unsigned long long epoch;
    int word;                                  // k_sp_slab_wait: SP_FL_DONE or SP_FL_READY
    unsigned long long *ctl;                   // sparse control words (error bits)
    unsigned *arrive;                          // zeroed before k_sp_slab_halo
    unsigned long long *tm;                    // Z-slab phase timers (TM_*; null: not recorded)
    int tm_m;                                  // second-pass sweep index 0..7
};

__global__ void __launch_bounds__(64) k_sp_slab_wait(SpHaloParams H)
{
    if (threadIdx.x >= 2 || !H.nb_flags[threadIdx.x]) return;
    const unsigned long long *f = H.flags + (H.word + threadIdx.x) * SP_FL_STRIDE;
    const unsigned long long t0 = wall_clock64();
    for (unsigned spins = 0;; ++spins) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= H.epoch) break;
        // fail fast once a handshake of this call has already failed (the neighbour is not coming)
        if (spins > SP_WATCHDOG || ((spins & 255u) == 255u && (sp_ld64(&H.ctl[SP_ERR]) & 16ull))) {
            atomicOr(&H.ctl[SP_ERR], 16ull);
            break;
        }
        if (spins < 64) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(16);
    }
    if (H.tm) atomicMax(H.tm + (H.word == SP_FL_DONE ? TM_WAIT_DONE : TM_WAIT_READY) + H.tm_m, wall_clock64() - t0);
}

__global__ void __launch_bounds__(256) k_sp_slab_halo(SpHaloParams H)
{
    for (int side = 0; side < 2; ++side) {
        if (!H.nb_flags[side]) continue;
        for (unsigned long long p = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; p < H.plane;
             p += (unsigned long long)gridDim.x * blockDim.x)
            __hip_atomic_store(H.hX[side] + p, __hip_atomic_load(H.hS[side] + p, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_SYSTEM),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(H.arrive, 1u) == gridDim.x - 1u) {
        // the side-s neighbour sees us from its side 1 - s
        if (H.nb_flags[0])
            __hip_atomic_store(H.nb_flags[0] + (SP_FL_READY + 1) * SP_FL_STRIDE, H.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        if (H.nb_flags[1])
            __hip_atomic_store(H.nb_flags[1] + (SP_FL_READY + 0) * SP_FL_STRIDE, H.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Z-slab, after the tile sweeps of the first pass: our first and last planes' low words go into
// the neighbours' pre-sweep halo planes of the first sparse sweep (parity 0), then DONE(epoch).
struct SpExportParams {
    const unsigned long long *cell;            // global cell index
    unsigned long long plane;
    unsigned long long c_first, c_last;        // first cell of plane k_lo / k_hi - 1
    uint32_t *nb_hS[2];                        // lower neighbour's upper halo, upper neighbour's lower halo
    unsigned long long *nb_flags[2];
    unsigned long long epoch;
    unsigned *arrive;
};

__global__ void __launch_bounds__(256) k_sp_slab_export(SpExportParams E)
{
    for (unsigned long long p = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; p < E.plane;
         p += (unsigned long long)gridDim.x * blockDim.x) {
        if (E.nb_hS[0])
            __hip_atomic_store(E.nb_hS[0] + p, (uint32_t)E.cell[E.c_first + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (E.nb_hS[1])
            __hip_atomic_store(E.nb_hS[1] + p, (uint32_t)E.cell[E.c_last + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(E.arrive, 1u) == gridDim.x - 1u) {
        if (E.nb_flags[0])
            __hip_atomic_store(E.nb_flags[0] + (SP_FL_DONE + 1) * SP_FL_STRIDE, E.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        if (E.nb_flags[1])
            __hip_atomic_store(E.nb_flags[1] + (SP_FL_DONE + 0) * SP_FL_STRIDE, E.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// Brick-owned repair (one GPU).  The grid is cut into 8x8x8 bricks.  A repair
// request names a cell; it sets the cell's bit in its brick's request bits and counts in the
// brick's request counter; the request that moves the counter 0 -> 1 queues the BRICK.  A wave
// that takes a brick owns it -- only the owner writes the brick's cells -- and repairs it in LDS:
// the brick's cells, their pre-sweep values and the upwind halo's labels are loaded once, and the
// requested cells and everything downstream of a relabel inside the brick are evaluated in one
// pass over the brick's anti-diagonals in the sweep's order (a cell's upwind neighbours lie on
// earlier diagonals, so each is final when the cell is evaluated).  A chain link inside a brick
// then costs an LDS read instead of the cell protocol's device round trips (label loads, the
// label store's wait, the request counters, the work list).  Relabelled cells are written back,
// and only cells on the brick's downstream faces request cells of the next bricks.  The owner
// retires the requests it saw; if more came meanwhile (an upwind brick changed a halo label) it
// reloads the halo and runs again.  Exact for the same reason as the cell protocol: when the work
// list drains, every cell satisfies x_c = f(S_c, labels(x_upwind)).
// ---------------------------------------------------------------------------
constexpr int SPB = 8;                     // brick edge (cells)
constexpr int SPB_CELLS = SPB * SPB * SPB;
constexpr int SPB_WORDS = SPB_CELLS / 32;  // request-bit words per brick
constexpr int SPB_H = SPB + 1;             // LDS label block edge: the upwind halo layer at 0

struct SpBrick {
    unsigned *breq;                        // per brick: outstanding requests (zero between sweeps)
    unsigned *bits;                        // per brick: SPB_WORDS request-bit words (zero between sweeps)
    int nbi, nbj, nbk;                     // bricks per axis
    unsigned long long nbricks;
};

// brick of global cell (i, j, k) and the cell's bit there, in the sweep's orientation (a grows
// downstream along i whatever the sign of di; the same for b, c)
__device__ __forceinline__ void spb_locate(const SpParams &P, const SpBrick &B, int i, int j, int k, unsigned *brick,
                                           unsigned *bit)
{
    const int bi = i / SPB, bj = j / SPB, bk = k / SPB;
    const int ei = min(SPB, P.ni - bi * SPB), ej = min(SPB, P.nj - bj * SPB), ek = min(SPB, P.nk - bk * SPB);
    const int a = P.di > 0 ? i - bi * SPB : ei - 1 - (i - bi * SPB);
    const int b = P.dj > 0 ? j - bj * SPB : ej - 1 - (j - bj * SPB);
    const int c = P.dk > 0 ? k - bk * SPB : ek - 1 - (k - bk * SPB);
    *brick = (unsigned)(bi + B.nbi * (bj + B.nbj * bk));
    *bit = (unsigned)(a + SPB * (b + SPB * c));
}

// Request the cells tgt[q] (slots with no target: ~0): bits first, and only once they are in
// place the counters -- an owner that counted a request finds its bit.  Bricks whose counter this
// lane moved 0 -> 1 are this lane's to queue: slot bits in *qmask, brick ids in bq[].
__device__ __forceinline__ void spb_request(const SpParams &P, const SpBrick &B, const size_t (&tgt)[7], unsigned *qmask,
                                            size_t (&bq)[7])
{
    unsigned br[7], bt[7];
    *qmask = 0;
    int fq = -1;   // first slot with a target
#pragma unroll
    for (int q = 6; q >= 0; --q)
        if (tgt[q] != ~(size_t)0) fq = q;
    if (fq < 0) return;   // (a lane with no target must not touch any counter: see below)
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        br[q] = 0;
        bt[q] = 0;
        if (tgt[q] != ~(size_t)0) {
            const unsigned t = (unsigned)tgt[q];
            const int i = (int)(t % (unsigned)P.ni);
            const unsigned r = t / (unsigned)P.ni;
            spb_locate(P, B, i, (int)(r % (unsigned)P.nj), (int)(r / (unsigned)P.nj), &br[q], &bt[q]);
            atomicOr(&B.bits[SDF_CHK(29, (size_t)br[q] * SPB_WORDS + (bt[q] >> 5), 0, B.nbricks * SPB_WORDS)],
                     1u << (bt[q] & 31u));
        }
    }
    sp_order();   // the bits are in place before any counter moves
    unsigned br0 = br[0];
#pragma unroll
    for (int q = 1; q < 7; ++q) br0 = fq == q ? br[q] : br0;
    unsigned old[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const bool ok = tgt[q] != ~(size_t)0;
        // branch-free (a conditional returning atomic costs a round trip each): a slot with no
        // target adds 0 to the lane's first target brick -- never to one shared word, which every
        // lane of every wave would hammer (a first version's 0-adds to brick 0 cost 20 ms per sweep)
        const unsigned r = atomicAdd(&B.breq[SDF_CHK(30, ok ? br[q] : br0, 0, B.nbricks)], ok ? 1u : 0u);
        old[q] = ok ? r : 1u;
    }
    unsigned qm = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        if (old[q] != 0u) continue;
        qm |= 1u << q;
        bq[q] = br[q];
    }
    *qmask = qm;
}

// the downstream neighbours of (i, j, k) in the grid (the cells whose upwind set contains it), ~0
// where there is none -- sp_request_collect's targets without its counters
__device__ __forceinline__ void spb_targets(const SpParams &P, int i, int j, int k, size_t c, size_t (&tgt)[7])
{
    const bool ii = P.di > 0 ? i + 1 <= P.ni - 1 : i - 1 >= 0;
    const bool jj = P.dj > 0 ? j + 1 <= P.nj - 1 : j - 1 >= 0;
    const bool kk = P.dk > 0 ? k + 1 <= P.nk - 1 : k - 1 >= 0;
    const long long si = P.di, sj = (long long)P.dj * P.ni, sk = (long long)P.dk * P.ni * P.nj;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int m = q + 1;
        const bool ui = m & 1, uj = m & 2, uk = m & 4;
        const bool ok = !((ui && !ii) || (uj && !jj) || (uk && !kk));
        tgt[q] = ok ? (size_t)((long long)c + (ui ? si : 0) + (uj ? sj : 0) + (uk ? sk : 0)) : ~(size_t)0;
    }
}

// Jacobi list pass, brick mode: the listed cells as in k_sp_jlist; a relabel requests its 7
// downstream cells from their bricks.
__global__ void __launch_bounds__(256) k_sp_jlist_brick(SpParams P, SpBrick B)
{
    const unsigned part = blockIdx.x % SP_JPARTS;
    const unsigned long long cnt0 = P.ctl[SP_JLIST + part * SP_JSTRIDE];
    const unsigned long long cnt = cnt0 < P.jcap ? cnt0 : P.jcap;
    const unsigned *list = P.jlist + (size_t)part * P.jcap;
    const unsigned lane = threadIdx.x & 63;
    for (unsigned long long x = (unsigned long long)(blockIdx.x / SP_JPARTS) * blockDim.x + threadIdx.x; x - lane < cnt;
         x += (unsigned long long)(gridDim.x / SP_JPARTS) * blockDim.x) {
        unsigned qmask = 0;
        size_t tgt[7], bq[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) tgt[q] = ~(size_t)0;
        if (x < cnt) {
            const unsigned c32 = list[x];
            const int i = (int)(c32 % (unsigned)P.ni);
            const unsigned r = c32 / (unsigned)P.ni;
            const int j = (int)(r % (unsigned)P.nj), k = (int)(r / (unsigned)P.nj);
            const unsigned long long s = P.S[SDF_CHK(20, c32, P.c_lo, P.c_lo + P.n)];
            const unsigned long long y = sp_eval<false>(P, P.S, i, j, k, c32, s);
            P.X[SDF_CHK(21, c32, P.c_lo, P.c_lo + P.n)] = y;
            if (lbl_of((uint32_t)y) != lbl_of((uint32_t)s)) spb_targets(P, i, j, k, c32, tgt);
        }
        // (the brick kernel reads the labels after this launch: no wait needed before the requests)
        spb_request(P, B, tgt, &qmask, bq);
        sp_append_wave(P, (unsigned)(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) & (P.nq - 1u)), qmask, bq, false);
    }
}

// The brick repair: one wave per workgroup, one brick at a time.  Lane (b, c) = (lane % 8,
// lane / 8) owns the brick's row (b, c): its 8 cells along a, their loads and write-backs; on
// anti-diagonal d it evaluates cell (d - b - c, b, c), so no lane needs a table to find its cell.
__global__ void __launch_bounds__(64) k_sp_brick(SpParams P, SpBrick B)
{
    __shared__ unsigned long long s_x[SPB_CELLS];      // the brick's cells (current), oriented index
    __shared__ unsigned long long s_s[SPB_CELLS];      // ... before the sweep
    __shared__ uint32_t s_w[SPB_H * SPB_H * SPB_H];    // low words with the upwind halo layer at 0
    __shared__ uint32_t s_f[SPB_WORDS];                // cells to evaluate
    const unsigned lane = threadIdx.x & 63;
    const int rb = (int)(lane % SPB), rc = (int)(lane / SPB);   // this lane's row
    const unsigned shard = blockIdx.x & (P.nq - 1u);
    unsigned long long *const q_tail = &P.ctl[SP_SHARD0 + shard * SP_SHSTRIDE];
    unsigned long long *const q_head = q_tail + 16;
    unsigned *const ring = P.queue + (size_t)shard * P.cap;
    unsigned long long runs = 0, h = 0;
    bool ticket = false;
    unsigned spins = 0;
#ifdef SP_ITER_PROF   // diagnostics: cycles per phase of a brick activation, activations, rounds
    unsigned long long bp[8] = {}, bp_t = 0, bp_act = 0, bp_rounds = 0;
#define SPB_P(q) do { const unsigned long long t2_ = clock64(); asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); bp[q] += t2_ - bp_t; bp_t = t2_; } while (0)
#else
#define SPB_P(q) do { } while (0)
#endif
    for (;;) {
        // ---- take a brick: one ticket per wave; the slot is read once the tail has passed it ----
        unsigned long long qw = 0, base = 0;
        unsigned v = 0;
        if (lane == 0) {
            if (!ticket) base = atomicAdd(q_head, 1ull);
            qw = sp_ld64(q_tail);
        }
        if (!ticket) {
            h = ((unsigned long long)(unsigned)__shfl((int)(base >> 32), 0) << 32) | (unsigned)__shfl((int)base, 0);
            ticket = true;
        }
        qw = ((unsigned long long)(unsigned)__shfl((int)(qw >> 32), 0) << 32) | (unsigned)__shfl((int)qw, 0);
        if (lane == 0 && h < (qw & 0xffffffffull)) v = sp_ld32(ring + sp_slot(h, P.cap));
        v = (unsigned)__shfl((int)v, 0);
        if (!v) {
            if ((qw >> 32) == 0ull) break;   // nothing queued or running in this shard: no slot can fill
            if (++spins > SP_WATCHDOG) {
                if (lane == 0) atomicOr(&P.ctl[SP_ERR], 1ull);
                break;
            }
            // back off: most waves are idle most of the time, and their polls of the shard words
            // slowed every other device access of the launch (a 4 us round trip at a 2 us poll)
            if (spins < 4) __builtin_amdgcn_s_sleep(1);
            else if (spins < 32) __builtin_amdgcn_s_sleep(4);
            else __builtin_amdgcn_s_sleep(16);
            continue;
        }
        if (lane == 0) sp_st32(ring + sp_slot(h, P.cap), 0u);
        ticket = false;
        spins = 0;
#ifdef SP_ITER_PROF
        bp_t = clock64();
        ++bp_act;
#endif
        const unsigned brick = SDF_CHK(31, v - 1, 0, B.nbricks);
        const int bi = (int)(brick % (unsigned)B.nbi), bt = (int)(brick / (unsigned)B.nbi);
        const int bj = bt % B.nbj, bk = bt / B.nbj;
        const int i0 = bi * SPB, j0 = bj * SPB, k0 = bk * SPB;
        const int ea = min(SPB, P.ni - i0), eb = min(SPB, P.nj - j0), ec = min(SPB, P.nk - k0);
        // oriented local (a, b, c) -> global: a grows in the sweep's i direction (-1: the upwind halo)
        const int ia0 = P.di > 0 ? i0 : i0 + ea - 1, sa = P.di;
        const int jb0 = P.dj > 0 ? j0 : j0 + eb - 1, sb = P.dj;
        const int kc0 = P.dk > 0 ? k0 : k0 + ec - 1, sc = P.dk;
        const long long rowstride = (long long)P.ni;
        const long long planestride = (long long)P.ni * P.nj;
        auto gidx = [&](int a, int b, int c) -> long long {
            return (long long)(ia0 + sa * a) + rowstride * (jb0 + sb * b) + planestride * (kc0 + sc * c);
        };
        auto ingrid = [&](int a, int b, int c) {
            const int i = ia0 + sa * a, j = jb0 + sb * b, k = kc0 + sc * c;
            return i >= 0 && i < P.ni && j >= 0 && j < P.nj && k >= 0 && k < P.nk;
        };
        const bool row_in = rb < eb && rc < ec;
        bool first = true;
        unsigned chg = 0, rel = 0;   // this lane's row: cells changed / relabelled (bit a)
        for (;;) {
            // requests so far, then their bits (requesters set the bit before counting)
            unsigned r = 0;
            if (lane == 0) r = sp_ld32(&B.breq[brick]);
            if (lane < SPB_WORDS) s_f[lane] = atomicExch(&B.bits[(size_t)brick * SPB_WORDS + lane], 0u);
            r = (unsigned)__shfl((int)r, 0);
            sp_order();   // the cells and halo are read after the requests were observed
            SPB_P(0);
#ifdef SP_ITER_PROF
            ++bp_rounds;
#endif
            // loads, all issued before the first is used: the row's cells (first round only -- the
            // owner is their only writer) and the upwind halo: the row's a = -1 cell, and 3 more
            // positions per lane for the b = -1 and c = -1 faces (9 x 9 + 9 x 8 = 153)
            unsigned long long xr[SPB], sr[SPB];
            uint32_t hr = 0, hf[3] = {0u, 0u, 0u};
            if (first && row_in) {
#pragma unroll
                for (int a = 0; a < SPB; ++a) {
                    if (a < ea) {
                        const size_t g = SDF_CHK(32, gidx(a, rb, rc), 0, P.n);
                        xr[a] = sp_ld64(P.X + g);
                        sr[a] = P.S[g];
                    }
                }
            }
            if (row_in && ingrid(-1, rb, rc))
                hr = sp_ld32(reinterpret_cast<const uint32_t *>(P.X + SDF_CHK(32, gidx(-1, rb, rc), 0, P.n)));
            int fa[3], fb[3], fc[3];
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int t = (int)lane + 64 * u;   // 0..152: (a, -1, c) for c = -1..7, then (a, b, -1) for b = 0..7
                fa[u] = t % SPB_H - 1;
                fb[u] = t < 81 ? -1 : (t - 81) / SPB_H;
                fc[u] = t < 81 ? t / SPB_H - 1 : -1;
                if (t < 153 && fa[u] < ea && fb[u] < eb && fc[u] < ec && ingrid(fa[u], fb[u], fc[u]))
                    hf[u] = sp_ld32(reinterpret_cast<const uint32_t *>(P.X + SDF_CHK(32, gidx(fa[u], fb[u], fc[u]), 0, P.n)));
            }
            if (first && row_in) {
#pragma unroll
                for (int a = 0; a < SPB; ++a) {
                    if (a < ea) {
                        const int o = a + SPB * (rb + SPB * rc);
                        s_x[o] = xr[a];
                        s_s[o] = sr[a];
                        s_w[(a + 1) + SPB_H * ((rb + 1) + SPB_H * (rc + 1))] = (uint32_t)xr[a];
                    }
                }
            }
            if (row_in) s_w[0 + SPB_H * ((rb + 1) + SPB_H * (rc + 1))] = hr;
#pragma unroll
            for (int u = 0; u < 3; ++u)
                if ((int)lane + 64 * u < 153) s_w[(fa[u] + 1) + SPB_H * ((fb[u] + 1) + SPB_H * (fc[u] + 1))] = hf[u];
            first = false;
            sp_wave_sync();
            SPB_P(1);
            // one pass over the anti-diagonals in the sweep's order
            const int dmax = ea + eb + ec - 3;
            for (int d = 0; d <= dmax; ++d) {
                const int a = d - rb - rc;
                const int o = a + SPB * (rb + SPB * rc);
                const bool act = row_in && a >= 0 && a < ea && ((s_f[o >> 5] >> (o & 31)) & 1u);
                if (!__any(act)) continue;
                if (act) {
                    const int i = ia0 + sa * a, j = jb0 + sb * rb, k = kc0 + sc * rc;
                    if (sp_in(P, i, j, k)) {
                        uint32_t w[7];
#pragma unroll
                        for (int q = 0; q < 7; ++q) {
                            const int m = q + 1;
                            w[q] = s_w[(a + 1 - (m & 1)) + SPB_H * ((rb + 1 - ((m >> 1) & 1)) + SPB_H * (rc + 1 - ((m >> 2) & 1)))];
                        }
                        const unsigned long long cur = s_x[o];
                        const unsigned long long y = sp_eval_w<true>(P, i, j, k, s_s[o], w);
                        ++runs;
                        if (y != cur) {
                            s_x[o] = y;
                            s_w[(a + 1) + SPB_H * ((rb + 1) + SPB_H * (rc + 1))] = (uint32_t)y;
                            chg |= 1u << a;
                            if (lbl_of((uint32_t)y) != lbl_of((uint32_t)cur)) {
                                // downstream cells inside the brick: later diagonals of this pass
#pragma unroll
                                for (int m = 1; m < 8; ++m) {
                                    const int a2 = a + (m & 1), b2 = rb + ((m >> 1) & 1), c2 = rc + ((m >> 2) & 1);
                                    if (a2 < ea && b2 < eb && c2 < ec) {
                                        const int o2 = a2 + SPB * (b2 + SPB * c2);
                                        atomicOr(&s_f[o2 >> 5], 1u << (o2 & 31));
                                    }
                                }
                                if (a == ea - 1 || rb == eb - 1 || rc == ec - 1) rel |= 1u << a;
                            }
                        }
                    }
                }
                sp_wave_sync();
            }
            SPB_P(2);
            // write back what changed, then (once it is visible) request the next bricks' cells
#pragma unroll
            for (int a = 0; a < SPB; ++a)
                if ((chg >> a) & 1u)
                    sp_st64(P.X + SDF_CHK(33, gidx(a, rb, rc), 0, P.n), s_x[a + SPB * (rb + SPB * rc)]);
            chg = 0;
            sp_order();
            SPB_P(3);
            while (__any(rel != 0u)) {
                size_t tgt[7], bq[7];
                unsigned qmask = 0;
#pragma unroll
                for (int q = 0; q < 7; ++q) tgt[q] = ~(size_t)0;
                if (rel) {
                    const int a = __builtin_ctz(rel);
                    rel &= rel - 1u;
                    size_t all[7];
                    spb_targets(P, ia0 + sa * a, jb0 + sb * rb, kc0 + sc * rc, (size_t)gidx(a, rb, rc), all);
#pragma unroll
                    for (int q = 0; q < 7; ++q) {   // only the targets outside this brick
                        const int m = q + 1;
                        const bool out = a + (m & 1) >= ea || rb + ((m >> 1) & 1) >= eb || rc + ((m >> 2) & 1) >= ec;
                        tgt[q] = out ? all[q] : ~(size_t)0;
                    }
                }
                spb_request(P, B, tgt, &qmask, bq);
                sp_append_wave(P, shard, qmask, bq, false);
            }
            SPB_P(4);
            // retire the requests this round saw; more arrived meanwhile: run again
            unsigned old = 0;
            if (lane == 0) old = atomicSub(&B.breq[brick], r);
            old = (unsigned)__shfl((int)old, 0);
            sp_wave_sync();
            if (old == r) break;
        }
        size_t none[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) none[q] = 0;
        sp_append_wave(P, shard, 0u, none, lane == 0);   // the brick's work item ends
        SPB_P(5);
    }
    if (runs) atomicAdd(&P.ctl[SP_RUNS], runs);
#ifdef SP_ITER_PROF
    if (lane == 0) {
        for (int q = 0; q < 6; ++q) atomicAdd(&P.ctl[SP_DIAGX + q], bp[q]);
        atomicAdd(&P.ctl[SP_DIAGX + 24], bp_act);
        atomicAdd(&P.ctl[SP_DIAGX + 25], bp_rounds);
    }
#endif
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct SparseSweepWorkspace {
    int workers = SP_WORKERS_DEFAULT;            // repair-kernel workgroups (diagnostics may lower it)
    bool brick = false;                          // one GPU: brick-owned repair (k_sp_brick) instead of per cell
    bool inplace = true;                         // one GPU, per-cell repair: sweep in place (SpParams::sv)
    unsigned *breq = nullptr, *bbits = nullptr;  // brick request counters and bits (zero between sweeps)
    size_t cap_breq = 0, cap_bbits = 0;
    unsigned long long ntri = ~0ull;             // soup size for bounds-checked builds
    unsigned long long *alt = nullptr;   // the second state buffer
    unsigned *req = nullptr, *queue = nullptr, *jlist = nullptr;
    unsigned long long *ctl = nullptr;
    size_t cap_alt = 0, cap_req = 0, cap_queue = 0, cap_jlist = 0;
};

inline bool sparse_sweep_supported(unsigned long long n, int ni, int nj, int nk)
{
    return ni >= 2 && nj >= 2 && nk >= 2 && n + SP_WORKERS * 64ull + 1024ull < 0xffffffffull;
}

template <class T>
inline int sp_grow(T **p, size_t *cap, size_t need, bool zero, hipStream_t st)
{
    if (*p && *cap >= need) return 0;
    if (*p) {
        const hipError_t e = hipFree(*p);
        *p = nullptr;
        *cap = 0;
        if (e != hipSuccess) return sdf_hip_rc(e);   // (a sticky fault of an earlier kernel: see st_grow)
    }
    *p = nullptr;
    *cap = 0;
    if (hipError_t e = hipMalloc((void **)p, need * sizeof(T)); e != hipSuccess) {
        *p = nullptr;
        return sdf_hip_rc(e);
    }
    if (zero) {
        if (hipError_t e = hipMemsetAsync(*p, 0, need * sizeof(T), st); e != hipSuccess) return sdf_hip_rc(e);
    }
    *cap = need;
    return 0;
}

// Workgroups of the Jacobi scan over n cells: about 8 cells per thread (a workgroup's set-up and list flush
// amortised: C3 scan 76.5 -> 71.2 us per sweep against 4 cells per thread, profiles/r05ba_jblocks.txt), but
// at least one round of the chip's 2,048 resident workgroups, at most SP_JBLOCKS (C4: 32 cells per thread,
// as fast as 16, faster than 64), and a multiple of the 8 XCDs (k_sp_jacobi's traversal).
inline unsigned long long sp_jblocks(unsigned long long n)
{
    unsigned long long b = std::max<unsigned long long>((n + 2047) / 2048, 2048);
    b = std::min<unsigned long long>(b, (n + 255) / 256);
    b = std::min<unsigned long long>(b, SP_JBLOCKS);
    return (b + 7) / 8 * 8;
}

// Workspace for sparse sweeps over n cells (allocations only: a Z-slab grows it before it
// enqueues anything, since a later hipFree would synchronise the device mid-call).
inline int sp_reserve(SparseSweepWorkspace &W, unsigned long long n, hipStream_t st)
{
    const unsigned long long cap = n + SP_WORKERS * 64ull + 1024ull;
    if (int rc_ = sp_grow(&W.req, &W.cap_req, n, true, st)) return rc_;
    if (int rc_ = sp_grow(&W.queue, &W.cap_queue, sp_shards(n) * cap, true, st)) return rc_;
    if (!W.ctl) {
        if (hipError_t e = hipMalloc((void **)&W.ctl, SP_NCTL * sizeof(unsigned long long)); e != hipSuccess) return sdf_hip_rc(e);
        if (hipError_t e = hipMemsetAsync(W.ctl, 0, SP_NCTL * sizeof(unsigned long long), st); e != hipSuccess) return sdf_hip_rc(e);
    }
    const unsigned long long blocks = sp_jblocks(n);
    const unsigned long long per_block = ((n + 7) / 8 + blocks / 8 * 256 - 1) / (blocks / 8 * 256) * 256;
    const unsigned long long jcap = (blocks + SP_JPARTS - 1) / SP_JPARTS * per_block;
    if (int rc_ = sp_grow(&W.jlist, &W.cap_jlist, SP_JPARTS * jcap, false, st)) return rc_;
    return 0;
}

// Shared part of a sparse sweep's setup: workspace for n cells starting at c_lo (req indexed by
// global cell), per-sweep control reset, launch geometry and the parameter block.
inline int sp_setup(SparseSweepWorkspace &W, hipStream_t st, const float4 *soup, const float origin[3], float dx,
                    int ni, int nj, int nk, int sweep, unsigned long long c_lo, unsigned long long n, SpParams &P,
                    unsigned long long &blocks)
{
    const int di = SP_DIRS[sweep % 8][0], dj = SP_DIRS[sweep % 8][1], dk = SP_DIRS[sweep % 8][2];
    const unsigned long long cap = n + SP_WORKERS * 64ull + 1024ull;
    if (int rc_ = sp_grow(&W.req, &W.cap_req, n, true, st)) return rc_;      // stays all-zero between sweeps
    if (int rc_ = sp_grow(&W.queue, &W.cap_queue, sp_shards(n) * cap, true, st)) return rc_; // slots are reset when consumed
    if (!W.ctl) {
        if (hipError_t e = hipMalloc((void **)&W.ctl, SP_NCTL * sizeof(unsigned long long)); e != hipSuccess) return sdf_hip_rc(e);
        if (hipError_t e = hipMemsetAsync(W.ctl, 0, SP_NCTL * sizeof(unsigned long long), st); e != hipSuccess) return sdf_hip_rc(e);
    }
    // per sweep: reset the list counters; error bits and statistics accumulate over the call
    if (hipError_t e = zero_async(W.ctl + SP_QUEUE, (SP_DIAGX - SP_QUEUE) * sizeof(unsigned long long), st); e != hipSuccess)
        return sdf_hip_rc(e);
    blocks = sp_jblocks(n);
    // each list part holds every cell its blocks visit (~n/64), so it never overflows; sizing
    // it for the ~10 % that are listed would need an in-place fallback whose registers
    // (ptd) halve the scan's occupancy: 150 -> 108 us per sweep at 256^3 without it
    const unsigned long long per_block = ((n + 7) / 8 + blocks / 8 * 256 - 1) / (blocks / 8 * 256) * 256;
    unsigned long long jcap = (blocks + SP_JPARTS - 1) / SP_JPARTS * per_block;
    if (sp_kscan_ok(c_lo, n, ni, nj, nk)) {   // the k-streaming scan's blocks too
        for (int np = 1; np <= 2; ++np) {
            const SpKGeom G = sp_kgeom(ni, nj, nk, np);
            jcap = std::max(jcap, (8ull * G.per_xcd + SP_JPARTS - 1) / SP_JPARTS * sp_kgeom_cells_per_block(G, np));
        }
    }
    if (int rc_ = sp_grow(&W.jlist, &W.cap_jlist, SP_JPARTS * jcap, false, st)) return rc_;
    memset(&P, 0, sizeof(P));
    P.soup = soup;
    P.req = W.req - c_lo;
    P.queue = W.queue;
    P.jlist = W.jlist;
    P.jcap = jcap;
    P.ctl = W.ctl;
    P.cap = cap;
    P.nq = sp_shards(n);
    P.n = n;
    P.c_lo = c_lo;
    P.ox = origin[0];
    P.oy = origin[1];
    P.oz = origin[2];
    P.dx = dx;
    P.ni = ni;
    P.nj = nj;
    P.nk = nk;
    P.di = di;
    P.dj = dj;
    P.dk = dk;
    P.sweep = sweep;
    P.k_lo = 0;
    P.k_hi = nk;
    P.ntri = W.ntri;
    for (int q = 0; q < 7; ++q) {
        const int m = q + 1;   // neighbour slot q lies upwind along the axes in mask m
        P.seen[q] = -1;
        for (int s2 = sweep - 1; s2 >= 0; --s2) {
            const int *d = SP_DIRS[s2 % 8];
            if ((!(m & 1) || d[0] == di) && (!(m & 2) || d[1] == dj) && (!(m & 4) || d[2] == dk)) {
                P.seen[q] = s2 + 1;
                break;
            }
        }
    }
    return 0;
}

// the one-device scan: the k-streaming pair scan on a whole grid (64-bit offsets above 2^29 cells), the
// other fast forms where the byte offsets fit 32 bits
inline void sp_launch_jacobi(unsigned long long blocks, hipStream_t st, const SpParams &P)
{
    static const int np = getenv("SDFGEN_JSCAN_NP") ? atoi(getenv("SDFGEN_JSCAN_NP")) : SP_JSCAN_PAIR;
    static const bool ks = getenv("SDFGEN_JSCAN_K") ? atoi(getenv("SDFGEN_JSCAN_K")) != 0 : SP_JSCAN_K != 0;
    if (ks && (np == 1 || np == 2) && sp_kscan_ok(P.c_lo, P.n, P.ni, P.nj, P.nk) && P.k_lo == 0 && P.k_hi == P.nk) {
        const SpKGeom G = sp_kgeom(P.ni, P.nj, P.nk, np);
        const bool wide = P.n > (1ull << 29);
        if (np == 2) {
            if (wide) hipLaunchKernelGGL((k_sp_jscan3<2, true>), dim3(8 * G.per_xcd), dim3(256), 0, st, P, G);
            else hipLaunchKernelGGL((k_sp_jscan3<2, false>), dim3(8 * G.per_xcd), dim3(256), 0, st, P, G);
        } else {
            if (wide) hipLaunchKernelGGL((k_sp_jscan3<1, true>), dim3(8 * G.per_xcd), dim3(256), 0, st, P, G);
            else hipLaunchKernelGGL((k_sp_jscan3<1, false>), dim3(8 * G.per_xcd), dim3(256), 0, st, P, G);
        }
    } else if (SP_JSCAN_FAST && P.c_lo == 0 && P.n == (unsigned long long)P.ni * P.nj * P.nk && P.k_lo == 0 && P.k_hi == P.nk &&
        P.n <= (1ull << 29) && blocks % 8 == 0) {
        if (np == 2) hipLaunchKernelGGL(k_sp_jscan2<2>, dim3((unsigned)blocks), dim3(256), 0, st, P);
        else if (np == 1) hipLaunchKernelGGL(k_sp_jscan2<1>, dim3((unsigned)blocks), dim3(256), 0, st, P);
        else
            hipLaunchKernelGGL((k_sp_jacobi<false, true>), dim3((unsigned)blocks), dim3(256), 0, st, P);
    }
    else
        hipLaunchKernelGGL((k_sp_jacobi<false, false>), dim3((unsigned)blocks), dim3(256), 0, st, P);
}

// The one-device list pass: its cells' words by 16-byte pair loads (SP_JLIST_PAIR, A/B) or eight narrow loads
// (SDFGEN_JLIST_NARROW=1 forces those)
#ifndef SP_JLIST_PAIR
#define SP_JLIST_PAIR 0   // measured neutral at C3 (38.2 vs 37.9 us) and slower at C4 (275 vs 264 us per sweep): off
#endif
inline void sp_launch_jlist(unsigned long long blocks, hipStream_t st, const SpParams &P)
{
    static const bool narrow = !SP_JLIST_PAIR || getenv("SDFGEN_JLIST_NARROW") != nullptr;
    if (narrow) hipLaunchKernelGGL((k_sp_jlist<false, false>), dim3((unsigned)blocks), dim3(256), 0, st, P);
    else hipLaunchKernelGGL((k_sp_jlist<false, true>), dim3((unsigned)blocks), dim3(256), 0, st, P);
}

// Enqueue one sparse sweep on `st`: reads *cell, writes the other buffer, then swaps
// the two so *cell holds the result.  Returns 0 or a negative SDFGEN_HIP_E* code.
inline int sparse_sweep(SparseSweepWorkspace &W, hipStream_t st, const float4 *soup, unsigned long long **cell,
                        size_t *cap_cell, const float origin[3], float dx, int ni, int nj, int nk,
                        int sweep)
{
    const unsigned long long n = (unsigned long long)ni * nj * nk;
    const int nw = (W.workers > 0 && W.workers <= SP_WORKERS) ? W.workers : SP_WORKERS;
    // (the two state buffers swap: both carry k_sp_jscan2's padding)
    if (int rc_ = sp_grow(&W.alt, &W.cap_alt, sp_pad(n), false, st)) return rc_;
    SpParams P;
    unsigned long long blocks = 0;
    if (int rc = sp_setup(W, st, soup, origin, dx, ni, nj, nk, sweep, 0, n, P, blocks)) return rc;
    if (W.brick) {
        P.S = *cell;
        P.X = W.alt;
        SpBrick B;
        B.nbi = (ni + SPB - 1) / SPB;
        B.nbj = (nj + SPB - 1) / SPB;
        B.nbk = (nk + SPB - 1) / SPB;
        B.nbricks = (unsigned long long)B.nbi * B.nbj * B.nbk;
        if (int rc_ = sp_grow(&W.breq, &W.cap_breq, B.nbricks, true, st)) return rc_;
        if (int rc_ = sp_grow(&W.bbits, &W.cap_bbits, B.nbricks * SPB_WORDS, true, st)) return rc_;
        B.breq = W.breq;
        B.bits = W.bbits;
        sp_launch_jacobi(blocks, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        hipLaunchKernelGGL(k_sp_jlist_brick, dim3(32 * SP_JPARTS), dim3(256), 0, st, P, B);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        hipLaunchKernelGGL(k_sp_brick, dim3(nw), dim3(64), 0, st, P, B);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
    } else if (W.inplace) {
        // in place: the cells that keep their value (~99.9 %) are neither copied nor swapped
        P.S = *cell;
        P.X = *cell;
        P.sv = W.alt;
        sp_launch_jacobi(blocks, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        sp_launch_jlist(SP_JLIST_PER_PART * SP_JPARTS, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        hipLaunchKernelGGL(k_sp_recheck<false>, dim3(nw), dim3(64), 0, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        return 0;
    } else {
        P.S = *cell;
        P.X = W.alt;
        sp_launch_jacobi(blocks, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        const unsigned long long lblocks = SP_JLIST_PER_PART * SP_JPARTS;   // k_sp_jlist: part = blockIdx % SP_JPARTS
        sp_launch_jlist(lblocks, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
        hipLaunchKernelGGL(k_sp_recheck<false>, dim3(nw), dim3(64), 0, st, P);
        if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
    }
    // swap the state buffers (both hold n cells)
    unsigned long long *t = *cell;
    const size_t tc = *cap_cell;
    *cell = W.alt;
    *cap_cell = W.cap_alt;
    W.alt = t;
    W.cap_alt = tc;
    return 0;
}

// One sparse sweep of a Z-slab (planes [k_lo, k_hi) of the grid).  Sides: 0 = the
// lower neighbour (planes below k_lo), 1 = the upper one.
struct SpSlabSweep {
    const unsigned long long *S;       // pre-sweep state, global cell index (own planes only)
    unsigned long long *X;             // result, global cell index (== S: in place, with sv)
    unsigned long long *sv;            // in place: pre-sweep values of changed cells (SpParams::sv); else null
    int k_lo, k_hi;
    const uint32_t *hS[2];             // our pre-sweep halo planes
    uint32_t *hX[2];                   // our live halo planes
    uint32_t *nb_hX[2];                // the neighbour's live halo of OUR boundary plane (remote)
    uint32_t *nb_ring[2];              // the neighbour's inbound ring fed by us (remote)
    uint32_t *in_ring[2];              // our inbound ring fed by that neighbour
    unsigned long long ring_cap;
    unsigned long long *flags;         // ours
    unsigned long long *nb_flags[2];   // the neighbours' (null: no neighbour)
    unsigned long long prev_epoch, epoch;
    unsigned *arrive;                  // one local word (the halo kernel's arrival counter)
    unsigned long long *tm;            // phase timers (TM_*; null: none) and this sweep's index 0..7
    int tm_m;
};

inline int sparse_sweep_slab(SparseSweepWorkspace &W, hipStream_t st, const float4 *soup, const SpSlabSweep &L,
                             const float origin[3], float dx, int ni, int nj, int nk, int sweep)
{
    const unsigned long long plane = (unsigned long long)ni * nj;
    const unsigned long long c_lo = plane * L.k_lo, n = plane * (L.k_hi - L.k_lo);
    const int nw = (W.workers > 0 && W.workers <= SP_WORKERS) ? W.workers : SP_WORKERS;
    SpParams P;
    unsigned long long blocks = 0;
    if (int rc = sp_setup(W, st, soup, origin, dx, ni, nj, nk, sweep, c_lo, n, P, blocks)) return rc;
    SpHaloParams H;
    memset(&H, 0, sizeof(H));
    for (int side = 0; side < 2; ++side) {
        H.hS[side] = L.hS[side];
        H.hX[side] = L.hX[side];
        H.nb_flags[side] = L.nb_flags[side];
    }
    H.plane = plane;
    H.flags = L.flags;
    H.ctl = W.ctl;
    H.arrive = L.arrive;
    H.tm = L.tm;
    H.tm_m = L.tm_m;
    H.word = SP_FL_DONE;
    H.epoch = L.prev_epoch;
    hipLaunchKernelGGL(k_sp_slab_wait, dim3(1), dim3(64), 0, st, H);
    if (hipError_t e_ = hipMemsetAsync(L.arrive, 0, sizeof(unsigned), st); e_ != hipSuccess) return sdf_hip_rc(e_);
    H.epoch = L.epoch;
    hipLaunchKernelGGL(k_sp_slab_halo, dim3((unsigned)std::min<unsigned long long>((plane + 255) / 256, 256)),
                       dim3(256), 0, st, H);
    P.S = L.S;
    P.X = L.X;
    P.sv = L.sv;
    P.k_lo = L.k_lo;
    P.k_hi = L.k_hi;
    const int up = P.dk > 0 ? 0 : 1, down = 1 - up;
    P.up_side = up;
    P.k_first = P.dk > 0 ? L.k_lo : L.k_hi - 1;
    P.k_last = P.dk > 0 ? L.k_hi - 1 : L.k_lo;
    P.hS_up = L.hS[up];
    P.hX_up = L.hX[up];
    P.push_down_halo = L.nb_flags[down] ? L.nb_hX[down] : nullptr;
    P.push_down_ring = L.nb_flags[down] ? L.nb_ring[down] : nullptr;
    P.push_up_halo = L.nb_flags[up] ? L.nb_hX[up] : nullptr;
    P.in_ring = L.nb_flags[up] ? L.in_ring[up] : nullptr;
    P.ring_cap = L.ring_cap;
    P.flags = L.flags;
    P.up_flags = L.nb_flags[up];
    P.down_flags = L.nb_flags[down];
    P.epoch = L.epoch;
    P.tm = L.tm;
    P.tm_m = L.tm_m;
    const char *stg = getenv("SDFGEN_DEBUG_SPARSE_STAGE");   // diagnostics: stop after kernel n (1 halo .. 4 all)
    const int stage = stg ? atoi(stg) : 4;
    if (stage >= 2) hipLaunchKernelGGL(k_sp_jacobi<true>, dim3((unsigned)blocks), dim3(256), 0, st, P);
    H.word = SP_FL_READY;
    if (stage >= 3) hipLaunchKernelGGL(k_sp_slab_wait, dim3(1), dim3(64), 0, st, H);
    const unsigned long long lblocks = 32 * SP_JPARTS;
    if (stage >= 3) hipLaunchKernelGGL(k_sp_jlist<true>, dim3((unsigned)lblocks), dim3(256), 0, st, P);
    if (stage >= 4) hipLaunchKernelGGL(k_sp_recheck<true>, dim3(nw), dim3(64), 0, st, P);
    if (hipError_t e_ = hipGetLastError(); e_ != hipSuccess) return sdf_hip_rc(e_);
    return 0;
}

// Repair workgroups of one slab when `share` slab sessions run on the current device: a quarter of the
// chip's resident k_sp_recheck<true> workgroups split between them (share 8 at 171 VGPRs: 64 each;
// share 1 and 2 keep the default), so the slabs' repair kernels and the first-pass grids of slabs still
// in their first pass fit together with room for uneven placement.
inline int sp_share_workers(int share)
{
    if (share <= 1) return SP_WORKERS;
    int occ = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_sp_recheck<true>, 64, 0) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        occ = 8;
        cus = 256;
    }
    return std::max(16, occ * cus / (4 * share));
}

inline void sparse_sweep_release(SparseSweepWorkspace &W)
{
    (void)hipFree(W.alt);
    (void)hipFree(W.req);
    (void)hipFree(W.queue);
    (void)hipFree(W.jlist);
    (void)hipFree(W.ctl);
    (void)hipFree(W.breq);
    (void)hipFree(W.bbits);
    W = SparseSweepWorkspace();
}

}  // namespace sdfhip
