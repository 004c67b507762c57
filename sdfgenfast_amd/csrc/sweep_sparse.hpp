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
//   * the high half of ctl[SP_QUEUE] counts queued or running work items (it grows in
//     the same atomic as the ring tail); workers leave when it is 0.
// Every spin is bounded (watchdog -> error bit, reported by the host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geom.hpp"

namespace sdfhip {

// ctl[SP_QUEUE]: work items appended to the ring (low 32 bits) and work items queued or
// running (high 32 bits) in ONE word, so an append is one atomic round trip.
// ctl layout: words 0..7 accumulate over the call (error bits, statistics); from SP_QUEUE
// on everything is reset before each sweep: the work-list counters, then the Jacobi list
// counters of SP_JPARTS parts, one 128-byte line each (a shared line serialises the
// atomics of the whole grid: 1.4 ms per sweep at 256^3, measured).
enum { SP_ERR = 0, SP_ENQ = 1, SP_RUNS = 2, SP_DIAG = 4, SP_QUEUE = 8, SP_HEAD = 9,
       SP_JPARTS = 64, SP_JSTRIDE = 16, SP_JLIST = 16, SP_NCTL = SP_JLIST + SP_JPARTS * SP_JSTRIDE };
constexpr unsigned long long SP_PENDING_ONE = 1ull << 32;
constexpr unsigned long long SP_TAIL_LIMIT = 0xF0000000ull;   // appends per sweep (error beyond)
constexpr unsigned SP_WATCHDOG = 1u << 24;   // empty polls (~1 s) before giving up
constexpr int SP_WORKERS = 512;              // max one-wave workgroups of the repair kernel
constexpr int SP_WORKERS_DEFAULT = 128;

// the reference's 8 sweep directions in pass order (cpu_lib/makelevelset3.cpp:243-291)
constexpr int SP_DIRS[8][3] = {{+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
                               {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};

struct SpParams {
    const float4 *soup;                // 3 float4 per triangle
    const unsigned long long *S;       // (phi bits << 32) | label before the sweep, i-fastest
    unsigned long long *X;             // result of the sweep
    unsigned *req;                     // per-cell recheck requests (zero between sweeps)
    unsigned *queue;                   // ring of cell+1 (0 = empty)
    unsigned *jlist;                   // Jacobi list: SP_JPARTS parts of jcap cells
    unsigned long long jcap;
    unsigned long long *ctl;           // SP_* counters
    unsigned long long cap;            // ring slots
    unsigned long long n;              // cells
    float ox, oy, oz, dx;
    int ni, nj, nk;
    int di, dj, dk;
    int sweep;                         // index (0..15) of this sweep
    int seen[7];                       // per neighbour slot q: s'+1 of the last earlier sweep in which
                                       // an interior cell examined that neighbour (-1: none)
};

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
template <bool LIVE>
__device__ __forceinline__ unsigned sp_mask(const SpParams &P, const unsigned long long *L, int i, int j, int k,
                                            size_t c, unsigned long long own, int (&lab)[7])
{
    const long long si = P.di, sj = (long long)P.dj * P.ni, sk = (long long)P.dk * P.ni * P.nj;
    const long long cc = (long long)c;
    const long long nb[7] = {cc - si, cc - sj, cc - si - sj, cc - sk, cc - si - sk, cc - sj - sk, cc - si - sj - sk};
    int lcq[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        // the low word (label, stamp) only: half the bytes of the 8-byte cell (a 32-bit load of
        // a 64-bit atomically stored word sees one of its stored values' halves)
        const uint32_t *lw = reinterpret_cast<const uint32_t *>(L + nb[q]);
        const uint32_t w = LIVE ? sp_ld32(lw) : *lw;
        lab[q] = lbl_of(w);
        lcq[q] = lc_of(w);
    }
    const int ct0 = lbl_of((uint32_t)own);
    const bool interior = i >= 1 && i <= P.ni - 2 && j >= 1 && j <= P.nj - 2 && k >= 1 && k <= P.nk - 2;
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
#ifdef SP_JACOBI_NOEVAL   // diagnostics only: the Jacobi pass's memory floor (wrong results)
    if (!LIVE) f = 0;
#endif
    return f;
}

template <bool LIVE>
__device__ __forceinline__ unsigned long long sp_eval(const SpParams &P, const unsigned long long *L, int i, int j,
                                                      int k, size_t c, unsigned long long own)
{
    int lab[7];
    unsigned f = sp_mask<LIVE>(P, L, i, j, k, c, own, lab);
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
        const size_t ba = 3 * (size_t)(has_a ? ta : 0), bb = 3 * (size_t)(has_b ? tb : (has_a ? ta : 0));
        const float4 a0 = P.soup[ba], a1 = P.soup[ba + 1], a2 = P.soup[ba + 2];
        const float4 b0 = P.soup[bb], b1 = P.soup[bb + 1], b2 = P.soup[bb + 2];
        float da, db;
        ptd_wave2(gx, mk3(a0.x, a0.y, a0.z), mk3(a1.x, a1.y, a1.z), mk3(a2.x, a2.y, a2.z), a2.w, gx,
                  mk3(b0.x, b0.y, b0.z), mk3(b1.x, b1.y, b1.z), mk3(b2.x, b2.y, b2.z), b2.w, da, db);
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


// Request rechecks of the downstream neighbours of (i,j,k) (the cells whose upwind set
// contains it).  Returns the first cell this call took ownership of when `claim`, so
// the caller can run it itself; the others are queued.
__device__ __forceinline__ size_t sp_request_downstream(const SpParams &P, int i, int j, int k, size_t c, bool claim)
{
    const bool ii = P.di > 0 ? i + 1 <= P.ni - 1 : i - 1 >= 0;
    const bool jj = P.dj > 0 ? j + 1 <= P.nj - 1 : j - 1 >= 0;
    const bool kk = P.dk > 0 ? k + 1 <= P.nk - 1 : k - 1 >= 0;
    const long long si = P.di, sj = (long long)P.dj * P.ni, sk = (long long)P.dk * P.ni * P.nj;
    const long long cc = (long long)c;
    // all requests in flight at once, then one reservation for the cells to queue
    size_t tgt[7];
    unsigned old[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        // same order as the upwind list: (i), (j), (i,j), (k), (i,k), (j,k), (i,j,k)
        const int m = q + 1;
        const bool ui = m & 1, uj = m & 2, uk = m & 4;
        const bool ok = !((ui && !ii) || (uj && !jj) || (uk && !kk));
        tgt[q] = ok ? (size_t)(cc + (ui ? si : 0) + (uj ? sj : 0) + (uk ? sk : 0)) : ~(size_t)0;
        old[q] = ok ? atomicAdd(&P.req[tgt[q]], 1u) : 1u;
    }
    size_t mine = ~(size_t)0;
    unsigned nq = 0;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        if (old[q] != 0u) continue;
        if (claim && mine == ~(size_t)0) mine = tgt[q];
        else ++nq;
    }
    if (nq) {
        // pending and tail grow together, so no item is visible to a worker before it counts
        const unsigned long long old_q = atomicAdd(&P.ctl[SP_QUEUE], nq * SP_PENDING_ONE + nq);
        unsigned long long t = old_q & 0xffffffffull;
        if (t + nq > SP_TAIL_LIMIT) atomicOr(&P.ctl[SP_ERR], 2ull);
#pragma unroll
        for (int q = 0; q < 7; ++q)
            if (old[q] == 0u && tgt[q] != mine) sp_st32(P.queue + (t++) % P.cap, (unsigned)(tgt[q] + 1));
    }
    return mine;
}

// Pass 1 of the sparse sweep: every cell against the labels of S, in two kernels.
// k_sp_jacobi streams the grid: a cell with no label left to examine (sp_mask == 0,
// ~90 % of them) is copied to X as is; the others are appended to a compact list that
// k_sp_jlist evaluates.  Evaluating in place would cost every wave as many ptd passes as
// its busiest lane needs while ~7 % of the packed lanes carry a candidate (measured,
// DESIGN.md §4); over the list nearly every lane has work.  Each wave gathers its list
// cells in LDS and appends them with one atomic per ~200 cells.
constexpr int SP_JWAVE = 256;   // LDS list entries per wave

__device__ __forceinline__ void sp_jacobi_cell(const SpParams &P, unsigned c32)
{
    const int i = (int)(c32 % (unsigned)P.ni);
    const unsigned r = c32 / (unsigned)P.ni;
    const int j = (int)(r % (unsigned)P.nj), k = (int)(r / (unsigned)P.nj);
    const unsigned long long s = P.S[c32];
    const unsigned long long y = sp_eval<false>(P, P.S, i, j, k, c32, s);
    P.X[c32] = y;
    if (lbl_of((uint32_t)y) != lbl_of((uint32_t)s)) sp_request_downstream(P, i, j, k, c32, false);
}

// wave-synchronous LDS hand-over between lanes of one wave
__device__ __forceinline__ void sp_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

__global__ void __launch_bounds__(256) k_sp_jacobi(SpParams P)
{
    __shared__ unsigned s_list[4][SP_JWAVE];
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so XCD x walks the x-th
    // contiguous eighth of the grid -- the neighbour planes a cell reads sit in its own L2.
    const bool xcd = gridDim.x % 8 == 0;
    const unsigned long long span = xcd ? (P.n + 7) / 8 : P.n;
    const unsigned long long base = xcd ? (unsigned long long)(blockIdx.x % 8) * span : 0ull;
    const unsigned lane = threadIdx.x & 63;
    const unsigned part = blockIdx.x % SP_JPARTS;   // part % 8 = this block's XCD
    unsigned *buf = s_list[threadIdx.x >> 6];
    unsigned cnt = 0;   // wave-uniform
    const unsigned long long first = (unsigned long long)(xcd ? blockIdx.x / 8 : blockIdx.x) * blockDim.x + threadIdx.x;
    const unsigned long long step = (unsigned long long)(xcd ? gridDim.x / 8 : gridDim.x) * blockDim.x;
    // (i, j, k) of the lane's cell: divided out once, then advanced by the stride's own
    // (si, sj, sk) with carries (two integer divisions per cell cost ~30 instructions)
    int i, j, k, si, sj, sk;
    {
        const unsigned c0 = (unsigned)(base + first), r0 = c0 / (unsigned)P.ni;
        i = (int)(c0 % (unsigned)P.ni);
        j = (int)(r0 % (unsigned)P.nj);
        k = (int)(r0 / (unsigned)P.nj);
        const unsigned st = (unsigned)step, rs = st / (unsigned)P.ni;
        si = (int)(st % (unsigned)P.ni);
        sj = (int)(rs % (unsigned)P.nj);
        sk = (int)(rs / (unsigned)P.nj);
    }
    for (unsigned long long it = first; it - lane < span; it += step) {   // wave-uniform trip count
        const unsigned long long c = base + it;
        const bool valid = it < span && c < P.n;
        const unsigned c32 = (unsigned)c;   // n < 2^32 (sparse_sweep_supported)
        unsigned f = 0;
        if (valid) {
            const unsigned long long s = P.S[c];
            int lab[7];
            if (sp_in(P, i, j, k)) f = sp_mask<false>(P, P.S, i, j, k, c, s, lab);
            if (!f) P.X[c] = s;
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

// Pass 1b: the listed cells, each exactly as in place (sp_eval against S).
__global__ void __launch_bounds__(256) k_sp_jlist(SpParams P)
{
    const unsigned part = blockIdx.x % SP_JPARTS;
    const unsigned long long cnt0 = P.ctl[SP_JLIST + part * SP_JSTRIDE];
    const unsigned long long cnt = cnt0 < P.jcap ? cnt0 : P.jcap;
    const unsigned *list = P.jlist + (size_t)part * P.jcap;
    for (unsigned long long x = (unsigned long long)(blockIdx.x / SP_JPARTS) * blockDim.x + threadIdx.x; x < cnt;
         x += (unsigned long long)(gridDim.x / SP_JPARTS) * blockDim.x)
        sp_jacobi_cell(P, list[x]);
}

// Pass 2: drain the recheck work list.  One lane = one worker; chains are followed
// depth-first by the lane that changed the upstream cell.  Written as a flat loop in
// which every lane does at most one poll or one evaluation per iteration: a lane
// spinning on an empty slot must never hold back (SIMT reconvergence) lanes of its own
// wave whose work would fill that slot.
__global__ void __launch_bounds__(64) k_sp_recheck(SpParams P)
{
    constexpr size_t NONE = ~(size_t)0;
    unsigned long long runs = 0, claims = 0, h = 0;
    size_t e = NONE, next = NONE;
    unsigned rq = 1;
    bool done = false, waiting = false;
    unsigned spins = 0;
    for (;;) {
        if (!done && e == NONE) {
            if (!waiting) {
                h = atomicAdd(&P.ctl[SP_HEAD], 1ull);
                waiting = true;
            }
            unsigned *slot = P.queue + h % P.cap;
            const unsigned v = sp_ld32(slot);
            if (v) {
                sp_st32(slot, 0u);
                e = v - 1;
                next = NONE;
                rq = 1;
                waiting = false;
                spins = 0;
            } else if ((sp_ld64(&P.ctl[SP_QUEUE]) >> 32) == 0ull) {
                done = true;   // nothing queued or running anywhere: no slot can fill any more
            } else if (++spins > SP_WATCHDOG) {
                atomicOr(&P.ctl[SP_ERR], 1ull);
                done = true;
            }
        }
        if (e != NONE) {
            // one evaluation of cell e, retiring `rq` requests
            const int i = (int)((unsigned)e % (unsigned)P.ni);
            const unsigned r0 = (unsigned)e / (unsigned)P.ni;
            const int j = (int)(r0 % (unsigned)P.nj), k = (int)(r0 / (unsigned)P.nj);
#ifdef SP_RT_PROBE   // diagnostics: N extra dependent device-scope round trips per evaluation
            {
                size_t e2 = e;
#pragma unroll
                for (int i_ = 0; i_ < SP_RT_PROBE; ++i_) e2 += (size_t)(sp_ld64(P.X + e2) & 0ull);
                e = e2;
            }
#endif
            const unsigned long long cur = sp_ld64(P.X + e);
#ifdef SP_NOEVAL_RECHECK   // diagnostics: the work list's own cost (no evaluation, no relabel)
            const unsigned long long y = cur;
#else
            const unsigned long long y = sp_eval<true>(P, P.X, i, j, k, e, P.S[e]);
#endif
            ++runs;
            const bool relabel = y != cur && lbl_of((uint32_t)y) != lbl_of((uint32_t)cur);
            if (y != cur) {
                sp_st64(P.X + e, y);
                if (relabel) sp_order();   // the new label is visible before anyone is asked to read it
            }
            // retire e's requests and ask for the downstream rechecks in one round trip
            const unsigned old = atomicSub(P.req + e, rq);
            if (relabel) {
                const size_t m = sp_request_downstream(P, i, j, k, e, next == NONE);
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
                    sp_order();
                    atomicSub(&P.ctl[SP_QUEUE], SP_PENDING_ONE);
                }
            } else {
                rq = old - rq;   // evaluate again for the requests that arrived meanwhile
                sp_order();
            }
        }
        if (__all(done)) break;
        if (!__any(e != NONE)) __builtin_amdgcn_s_sleep(2);
    }
    if (runs) atomicAdd(&P.ctl[SP_RUNS], runs);
    if (claims) atomicAdd(&P.ctl[SP_ENQ], claims);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct SparseSweepWorkspace {
    int workers = SP_WORKERS_DEFAULT;            // repair-kernel workgroups (diagnostics may lower it)
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
inline int sp_grow(T **p, size_t *cap, size_t need, bool zero)
{
    if (*p && *cap >= need) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void **)p, need * sizeof(T)) != hipSuccess) return -5;
    if (zero && hipMemset(*p, 0, need * sizeof(T)) != hipSuccess) return -4;
    *cap = need;
    return 0;
}

// Enqueue one sparse sweep on `st`: reads *cell, writes the other buffer, then swaps
// the two so *cell holds the result.  Returns 0 or a negative SDFGEN_HIP_E* code.
inline int sparse_sweep(SparseSweepWorkspace &W, hipStream_t st, const float4 *soup, unsigned long long **cell,
                        size_t *cap_cell, const float origin[3], float dx, int ni, int nj, int nk,
                        int sweep)
{
    const int di = SP_DIRS[sweep % 8][0], dj = SP_DIRS[sweep % 8][1], dk = SP_DIRS[sweep % 8][2];
    const unsigned long long n = (unsigned long long)ni * nj * nk;
    const int nw = (W.workers > 0 && W.workers <= SP_WORKERS) ? W.workers : SP_WORKERS;
    const unsigned long long cap = n + SP_WORKERS * 64ull + 1024ull;
    if (sp_grow(&W.alt, &W.cap_alt, n, false)) return -5;
    if (sp_grow(&W.req, &W.cap_req, n, true)) return -5;      // stays all-zero between sweeps
    if (sp_grow(&W.queue, &W.cap_queue, cap, true)) return -5; // slots are reset when consumed
    if (!W.ctl) {
        if (hipMalloc((void **)&W.ctl, SP_NCTL * sizeof(unsigned long long)) != hipSuccess) return -5;
        if (hipMemset(W.ctl, 0, SP_NCTL * sizeof(unsigned long long)) != hipSuccess) return -4;
    }
    // per sweep: reset the list counters; error bits and statistics accumulate over the call
    if (hipMemsetAsync(W.ctl + SP_QUEUE, 0, (SP_NCTL - SP_QUEUE) * sizeof(unsigned long long), st) != hipSuccess)
        return -4;
    unsigned long long blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    blocks = (blocks + 7) / 8 * 8;   // a multiple of the 8 XCDs (k_sp_jacobi's traversal)
    // each list part holds every cell its blocks visit (~n/64), so it never overflows; sizing
    // it for the ~10 % that are listed would need an in-place fallback whose registers
    // (ptd) halve the scan's occupancy: 150 -> 108 us per sweep at 256^3 without it
    const unsigned long long per_block = ((n + 7) / 8 + blocks / 8 * 256 - 1) / (blocks / 8 * 256) * 256;
    const unsigned long long jcap = (blocks + SP_JPARTS - 1) / SP_JPARTS * per_block;
    if (sp_grow(&W.jlist, &W.cap_jlist, SP_JPARTS * jcap, false)) return -5;
    SpParams P;
    P.soup = soup;
    P.S = *cell;
    P.X = W.alt;
    P.req = W.req;
    P.queue = W.queue;
    P.jlist = W.jlist;
    P.jcap = jcap;
    P.ctl = W.ctl;
    P.cap = cap;
    P.n = n;
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
    hipLaunchKernelGGL(k_sp_jacobi, dim3((unsigned)blocks), dim3(256), 0, st, P);
    if (hipGetLastError() != hipSuccess) return -4;
    const unsigned long long lblocks = 32 * SP_JPARTS;   // k_sp_jlist: part = blockIdx % SP_JPARTS
    hipLaunchKernelGGL(k_sp_jlist, dim3((unsigned)lblocks), dim3(256), 0, st, P);
    if (hipGetLastError() != hipSuccess) return -4;
    hipLaunchKernelGGL(k_sp_recheck, dim3(nw), dim3(64), 0, st, P);
    if (hipGetLastError() != hipSuccess) return -4;
    // swap the state buffers (both hold n cells)
    unsigned long long *t = *cell;
    const size_t tc = *cap_cell;
    *cell = W.alt;
    *cap_cell = W.cap_alt;
    W.alt = t;
    W.cap_alt = tc;
    return 0;
}

inline void sparse_sweep_release(SparseSweepWorkspace &W)
{
    (void)hipFree(W.alt);
    (void)hipFree(W.req);
    (void)hipFree(W.queue);
    (void)hipFree(W.jlist);
    (void)hipFree(W.ctl);
    W = SparseSweepWorkspace();
}

}  // namespace sdfhip
