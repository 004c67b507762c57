// sweep_wavefront.hpp -- one Gauss-Seidel sweep direction as ONE persistent launch:
// a pipelined column wavefront over (j,k) tiles.
//
// The reference sweep (cpu_lib/makelevelset3.cpp:130-151) visits, for direction
// (di,dj,dk), k then j then i, and updates each cell from its 7 upwind neighbours
// (:143-149).  In oriented coordinates (a,b,c) (a = i-1 for di>0, ni-2-i for di<0,
// likewise b,c) every upwind neighbour has a strictly smaller a+b+c, and each cell
// is written once per sweep, so ANY order that finishes a cell's upwind
// neighbours first reproduces the sequential result bit-for-bit.
//
// Decomposition (KBA-style): the (b,c) plane is cut into TB x TC tiles; a tile is
// one workgroup task that streams along a (the contiguous i axis).  Compute lane
// (bl,cl) owns column (b,c) and at local step h updates cell a = h - bl - cl, so a
// workgroup advances one anti-diagonal per step (two LDS barriers).  Neighbour
// results -- closest-triangle label AND the triangle's vertices -- travel through an
// LDS ring (4 slots per column), so the critical path never waits on a global
// gather: a candidate's vertices are already in LDS when it is evaluated.
// Tile-to-tile hand-off: lanes on a tile's last row/column publish each new label
// as an 8-byte tagged granule {epoch, label} (one sc1 store, no fence: the data is
// the flag, cdna_hip_programming.md G16 R2); a dedicated halo wave of the consumer
// tile polls those granules non-blockingly, gathers the triangles' vertices from
// the read-only soup and fills a per-stream LDS ring ahead of use.  The tile steps
// only when every halo entry it needs has landed (`go` vote), so there is no
// blocking spin anywhere except a bounded stall counter.
// Tasks are dequeued in anti-diagonal order (J+K, then J) from an atomic counter,
// so every producer tile has been claimed by a running workgroup before any of its
// consumers: no residency assumption, no deadlock.
// Candidate skips are exact: a label equal to the cell's own original label or to an
// earlier candidate's label evaluates to the same float and cannot pass strict '<'.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "geom.hpp"

namespace sdfhip {

constexpr int WF_TB = 16;                        // tile extent in b (j)
constexpr int WF_TC = 16;                        // tile extent in c (k)
constexpr int WF_NCOMP = WF_TB * WF_TC;          // compute lanes = columns per tile
constexpr int WF_NSTREAM = WF_TB + WF_TC + 1;    // halo streams: b-edge, c-edge, corner
constexpr int WF_R = 8;                          // halo ring slots per stream
constexpr int WF_THREADS = WF_NCOMP + 64;        // + one halo wave
constexpr int WF_RING_ENTS = 4 * WF_NCOMP;
constexpr int WF_ENTS = WF_RING_ENTS + WF_NSTREAM * WF_R;

struct WfParams {
    const float4 *soup;           // 3 float4 per triangle (xyz, w unused)
    unsigned long long *cell;     // (phi bits << 32) | closest_tri, i-fastest
    unsigned long long *hb;       // granules of tile-row edges:  [nJ][C][A]
    unsigned long long *hc;       // granules of tile-col edges:  [nK][B][A]
    const int2 *tasks;            // (J,K) in dequeue order
    int *queue;                   // task counter (zeroed before launch)
    int *err;                     // bit 1: stall watchdog fired
    unsigned long long *stats;    // optional [evals, stall iterations]
    float ox, oy, oz, dx;
    int ni, nj, nk;
    int A, B, C, nJ, nK, ntasks;
    int di, dj, dk;
    unsigned epoch;
};

__device__ __forceinline__ size_t wf_phys(const WfParams &P, int a, int b, int c)
{
    const int i = P.di > 0 ? a + 1 : P.ni - 2 - a;
    const int j = P.dj > 0 ? b + 1 : P.nj - 2 - b;
    const int k = P.dk > 0 ? c + 1 : P.nk - 2 - c;
    return (size_t)i + (size_t)P.ni * ((size_t)j + (size_t)P.nj * (size_t)k);
}

__device__ __forceinline__ f3 wf_xyz(float4 v) { return mk3(v.x, v.y, v.z); }

__global__ void __launch_bounds__(WF_THREADS) k_sweep_wavefront(WfParams P)
{
    __shared__ float4 s_ent[WF_ENTS * 3];   // entry e: [3e] = (x1, label bits), [3e+1] = x2, [3e+2] = x3
    __shared__ int s_ready[WF_NSTREAM];     // halo entries < s_ready[s] are in LDS
    __shared__ int s_nogo[2];
    __shared__ int s_task;

    const int tid = threadIdx.x;
    const bool is_comp = tid < WF_NCOMP;
    const int bl = tid % WF_TB, cl = tid / WF_TB;
    const int hs = tid - WF_NCOMP;
    unsigned long long n_evals = 0, n_stall = 0;

    for (;;) {
        if (tid == 0) {
            s_task = atomicAdd(P.queue, 1);
            s_nogo[0] = 0;
            s_nogo[1] = 0;
        }
        __syncthreads();
        const int task = s_task;
        if (task >= P.ntasks) break;
        const int2 JK = P.tasks[task];
        const int J = JK.x, K = JK.y;
        const int b0 = J * WF_TB, c0 = K * WF_TC;
        const int nsteps = P.A + WF_TB + WF_TC - 2;

        // ---------------- compute-lane setup ----------------
        const int b = b0 + bl, c = c0 + cl;
        const bool col = is_comp && b < P.B && c < P.C;
        // LDS sources of the 6 in-ring neighbours n1..n6 (cpu_lib/makelevelset3.cpp:144-149);
        // n0 = (a-1, b, c) is the lane's own previous result (ring slot of its own column).
        int nb_base[7], nb_stride[7], nb_mask[7];
        {
            auto ring = [&](int q, int lbl, int lcl) {
                nb_base[q] = lcl * WF_TB + lbl;
                nb_stride[q] = WF_NCOMP;
                nb_mask[q] = 3;
            };
            auto halo = [&](int q, int s) {
                nb_base[q] = WF_RING_ENTS + s * WF_R;
                nb_stride[q] = 1;
                nb_mask[q] = WF_R - 1;
            };
            ring(0, bl, cl);
            // (b-1, c)
            if (bl > 0) { ring(1, bl - 1, cl); ring(2, bl - 1, cl); } else { halo(1, cl); halo(2, cl); }
            // (b, c-1)
            if (cl > 0) { ring(3, bl, cl - 1); ring(4, bl, cl - 1); } else { halo(3, WF_TC + bl); halo(4, WF_TC + bl); }
            // (b-1, c-1)
            if (bl > 0 && cl > 0) { ring(5, bl - 1, cl - 1); ring(6, bl - 1, cl - 1); }
            else if (bl == 0 && cl == 0) { halo(5, WF_TC + WF_TB); halo(6, WF_TC + WF_TB); }
            else if (bl == 0) { halo(5, cl - 1); halo(6, cl - 1); }
            else { halo(5, WF_TC + bl - 1); halo(6, WF_TC + bl - 1); }
        }
        // own-column prefetch queue: cells a, a+1, a+2 and the vertices of cell a's label
        unsigned long long q0 = 0, q1 = 0, q2 = 0;
        float4 ov0 = make_float4(0, 0, 0, 0), ov1 = ov0, ov2 = ov0;
        if (col) {
            // a = -1 entry (boundary plane, never updated in this sweep) -> ring slot 3
            const unsigned long long e = P.cell[wf_phys(P, -1, b, c)];
            const int t = (int)(uint32_t)e;
            float4 v0 = make_float4(0, 0, 0, 0), v1 = v0, v2 = v0;
            if (t >= 0) { v0 = P.soup[3 * (size_t)t]; v1 = P.soup[3 * (size_t)t + 1]; v2 = P.soup[3 * (size_t)t + 2]; }
            v0.w = __int_as_float(t);
            const int ent = 3 * WF_NCOMP + tid;
            s_ent[3 * ent] = v0;
            s_ent[3 * ent + 1] = v1;
            s_ent[3 * ent + 2] = v2;
            q0 = P.cell[wf_phys(P, 0, b, c)];
            if (1 < P.A) q1 = P.cell[wf_phys(P, 1, b, c)];
            if (2 < P.A) q2 = P.cell[wf_phys(P, 2, b, c)];
            const int t0 = (int)(uint32_t)q0;
            if (t0 >= 0) { ov0 = P.soup[3 * (size_t)t0]; ov1 = P.soup[3 * (size_t)t0 + 1]; ov2 = P.soup[3 * (size_t)t0 + 2]; }
        }

        // ---------------- halo-lane setup ----------------
        bool hvalid = false, hbound = false;
        int hbs = 0, hcs = 0, hoff = 0;
        const unsigned long long *hsrc = nullptr;
        if (!is_comp && hs < WF_NSTREAM) {
            if (hs < WF_TC) {                      // (b0-1, c0+hs): tile row J-1, last row
                hbs = b0 - 1; hcs = c0 + hs; hoff = hs;
                hvalid = hcs < P.C;
                hbound = (J == 0);
                if (!hbound) hsrc = P.hb + ((size_t)(J - 1) * P.C + hcs) * P.A;
            } else if (hs < WF_TC + WF_TB) {       // (b0+bl, c0-1): tile col K-1, last column
                hbs = b0 + (hs - WF_TC); hcs = c0 - 1; hoff = hs - WF_TC;
                hvalid = hbs < P.B;
                hbound = (K == 0);
                if (!hbound) hsrc = P.hc + ((size_t)(K - 1) * P.B + hbs) * P.A;
            } else {                                // corner (b0-1, c0-1)
                hbs = b0 - 1; hcs = c0 - 1; hoff = 0;
                hvalid = true;
                hbound = (J == 0 || K == 0);
                if (!hbound) hsrc = P.hb + ((size_t)(J - 1) * P.C + hcs) * P.A;
            }
            if (hvalid) {
                const unsigned long long e = P.cell[wf_phys(P, -1, hbs, hcs)];
                const int t = (int)(uint32_t)e;
                float4 v0 = make_float4(0, 0, 0, 0), v1 = v0, v2 = v0;
                if (t >= 0) { v0 = P.soup[3 * (size_t)t]; v1 = P.soup[3 * (size_t)t + 1]; v2 = P.soup[3 * (size_t)t + 2]; }
                v0.w = __int_as_float(t);
                const int ent = WF_RING_ENTS + hs * WF_R + (WF_R - 1);
                s_ent[3 * ent] = v0;
                s_ent[3 * ent + 1] = v1;
                s_ent[3 * ent + 2] = v2;
                s_ready[hs] = 0;
            } else {
                s_ready[hs] = P.A;
            }
        }
        __syncthreads();

        // halo pipeline state (granule -> gather -> LDS), one entry in each stage
        int h_next = 0;
        bool g_pend = false, v_pend = false;
        int g_a = 0, v_a = 0;
        unsigned long long g_val = 0;
        float4 hv0 = make_float4(0, 0, 0, 0), hv1 = hv0, hv2 = hv0;
        unsigned stalls = 0;   // consecutive stalled iterations (workgroup-uniform)

        int h = 0, it = 0;
        while (h < nsteps) {
            const int a = h - bl - cl;
            const bool act = col && a >= 0 && a < P.A;
            // ---- go vote: every halo entry this step reads must be in LDS ----
            if (act) {
                bool ok = true;
                if (bl == 0 && s_ready[cl] <= a) ok = false;
                if (cl == 0 && s_ready[WF_TC + bl] <= a) ok = false;
                if (bl == 0 && cl == 0 && s_ready[WF_TC + WF_TB] <= a) ok = false;
                if (!ok) s_nogo[it & 1] = 1;
            }
            __syncthreads();
            const bool go = s_nogo[it & 1] == 0;
            if (tid == 0) s_nogo[(it + 1) & 1] = 0;

            if (is_comp) {
                if (go && act) {
                    float phi = __uint_as_float((uint32_t)(q0 >> 32));
                    int ct = (int)(uint32_t)q0;
                    const int ct_orig = ct;
                    int win = -1;   // LDS entry of the winning candidate (-1: own label)
                    const f3 gx = mk3((float)(P.di > 0 ? a + 1 : P.ni - 2 - a) * P.dx + P.ox,
                                      (float)(P.dj > 0 ? b + 1 : P.nj - 2 - b) * P.dx + P.oy,
                                      (float)(P.dk > 0 ? c + 1 : P.nk - 2 - c) * P.dx + P.oz);
                    int ent[7], lab[7];
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
                        const int aq = (q == 0 || q == 2 || q == 4 || q == 6) ? a - 1 : a;
                        ent[q] = nb_base[q] + (aq & nb_mask[q]) * nb_stride[q];
                        lab[q] = __float_as_int(s_ent[3 * ent[q]].w);
                    }
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
                        const int t = lab[q];
                        bool skip = (t < 0) || (t == ct_orig);
#pragma unroll
                        for (int r = 0; r < q; ++r) skip = skip || (lab[r] == t);
                        if (!skip) {
                            const float4 x1 = s_ent[3 * ent[q]], x2 = s_ent[3 * ent[q] + 1], x3 = s_ent[3 * ent[q] + 2];
                            const float d = ptd(gx, wf_xyz(x1), wf_xyz(x2), wf_xyz(x3));
                            ++n_evals;
                            if (d < phi) {
                                phi = d;
                                ct = t;
                                win = ent[q];
                            }
                        }
                    }
                    float4 w0, w1, w2;
                    if (win < 0) { w0 = ov0; w1 = ov1; w2 = ov2; }
                    else { w0 = s_ent[3 * win]; w1 = s_ent[3 * win + 1]; w2 = s_ent[3 * win + 2]; }
                    w0.w = __int_as_float(ct);
                    const int slot = (a & 3) * WF_NCOMP + tid;
                    s_ent[3 * slot] = w0;
                    s_ent[3 * slot + 1] = w1;
                    s_ent[3 * slot + 2] = w2;
                    if (win >= 0) P.cell[wf_phys(P, a, b, c)] = ((unsigned long long)__float_as_uint(phi) << 32) | (uint32_t)ct;
                    const unsigned long long gran = ((unsigned long long)P.epoch << 32) | (uint32_t)ct;
                    if (bl == WF_TB - 1 && J < P.nJ - 1)
                        __hip_atomic_store(P.hb + ((size_t)J * P.C + c) * P.A + a, gran, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    if (cl == WF_TC - 1 && K < P.nK - 1)
                        __hip_atomic_store(P.hc + ((size_t)K * P.B + b) * P.A + a, gran, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    // advance the own-column queue (cells are only written by this lane)
                    q0 = q1;
                    q1 = q2;
                    if (a + 3 < P.A) q2 = P.cell[wf_phys(P, a + 3, b, c)];
                    const int tn = (int)(uint32_t)q0;
                    if (a + 1 < P.A && tn >= 0) {
                        ov0 = P.soup[3 * (size_t)tn];
                        ov1 = P.soup[3 * (size_t)tn + 1];
                        ov2 = P.soup[3 * (size_t)tn + 2];
                    }
                }
            } else if (hvalid) {
                // ---- halo lane: (1) publish the gathered entry, (2) check granule -> gather, (3) issue next ----
                if (v_pend) {
                    const int ent = WF_RING_ENTS + hs * WF_R + (v_a & (WF_R - 1));
                    s_ent[3 * ent] = hv0;
                    s_ent[3 * ent + 1] = hv1;
                    s_ent[3 * ent + 2] = hv2;
                    s_ready[hs] = v_a + 1;
                    v_pend = false;
                }
                if (g_pend) {
                    const bool okg = hbound || (uint32_t)(g_val >> 32) == P.epoch;
                    if (okg) {
                        const int t = (int)(uint32_t)g_val;
                        hv0 = make_float4(0, 0, 0, 0); hv1 = hv0; hv2 = hv0;
                        if (t >= 0) { hv0 = P.soup[3 * (size_t)t]; hv1 = P.soup[3 * (size_t)t + 1]; hv2 = P.soup[3 * (size_t)t + 2]; }
                        hv0.w = __int_as_float(t);
                        v_a = g_a;
                        v_pend = true;
                        g_pend = false;
                        h_next = g_a + 1;
                    } else {
                        g_val = __hip_atomic_load(hsrc + g_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                if (!g_pend && h_next < P.A && h_next < h - hoff - 2 + WF_R) {
                    g_a = h_next;
                    if (hbound) g_val = P.cell[wf_phys(P, g_a, hbs, hcs)];
                    else g_val = __hip_atomic_load(hsrc + g_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    g_pend = true;
                }
            }
            __syncthreads();
            ++it;
            if (go) {
                ++h;
                stalls = 0;
            } else {
                ++n_stall;
                // watchdog: ~2^22 consecutive stalled iterations (seconds) means a lost
                // hand-off -- flag it and give up on the tile rather than hang the GPU.
                if (++stalls > (1u << 22)) {
                    if (tid == 0) atomicOr(P.err, 2);
                    h = nsteps;
                }
            }
        }
        __syncthreads();
    }
    if (P.stats) {
        if (n_evals) atomicAdd(P.stats, n_evals);
        if (tid == 0 && n_stall) atomicAdd(P.stats + 1, n_stall);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct WavefrontWorkspace {
    unsigned long long *hb = nullptr, *hc = nullptr, *stats = nullptr;
    size_t cap_hb = 0, cap_hc = 0;
    int2 *tasks = nullptr;
    size_t cap_tasks = 0;
    int task_nJ = -1, task_nK = -1;
    int *ctrl = nullptr;      // [0] queue counter, [1] error
    unsigned epoch = 0;
    bool count_evals = false;
};

inline bool wavefront_supported(int ni, int nj, int nk) { return ni >= 2 && nj >= 2 && nk >= 2; }

inline int wf_grow(unsigned long long **p, size_t *cap, size_t need)
{
    if (*p && *cap >= need) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void **)p, need * sizeof(unsigned long long)) != hipSuccess) return -5;
    if (hipMemset(*p, 0, need * sizeof(unsigned long long)) != hipSuccess) return -4;   // tags never match epoch 0
    *cap = need;
    return 0;
}

// Returns 0 or a negative SDFGEN_HIP_E* code (message in err).
inline int wavefront_sweep(WavefrontWorkspace &W, hipStream_t st, const float4 *soup, unsigned long long *cell,
                           const float origin[3], float dx, int ni, int nj, int nk, int di, int dj, int dk,
                           char *err, size_t errlen)
{
    const int A = ni - 1, B = nj - 1, C = nk - 1;
    const int nJ = (B + WF_TB - 1) / WF_TB, nK = (C + WF_TC - 1) / WF_TC;
    const int ntasks = nJ * nK;
    auto fail = [&](int code, const char *msg) {
        if (err && errlen) snprintf(err, errlen, "wavefront sweep: %s", msg);
        return code;
    };
    if (wf_grow(&W.hb, &W.cap_hb, (size_t)nJ * C * A)) return fail(-5, "halo buffer allocation failed");
    if (wf_grow(&W.hc, &W.cap_hc, (size_t)nK * B * A)) return fail(-5, "halo buffer allocation failed");
    if (!W.ctrl) {
        if (hipMalloc((void **)&W.ctrl, 16 * sizeof(int)) != hipSuccess) return fail(-5, "control allocation failed");
        if (hipMalloc((void **)&W.stats, 2 * sizeof(unsigned long long)) != hipSuccess) return fail(-5, "stats alloc");
    }
    if (W.task_nJ != nJ || W.task_nK != nK) {
        std::vector<int2> t;
        t.reserve(ntasks);
        for (int d = 0; d <= nJ + nK - 2; ++d)
            for (int J = 0; J < nJ; ++J) {
                const int K = d - J;
                if (K >= 0 && K < nK) t.push_back(make_int2(J, K));
            }
        if ((size_t)ntasks > W.cap_tasks) {
            if (W.tasks) (void)hipFree(W.tasks);
            if (hipMalloc((void **)&W.tasks, ntasks * sizeof(int2)) != hipSuccess) return fail(-5, "task table");
            W.cap_tasks = ntasks;
        }
        if (hipMemcpy(W.tasks, t.data(), ntasks * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess)
            return fail(-4, "task table upload");
        W.task_nJ = nJ;
        W.task_nK = nK;
    }
    if (++W.epoch == 0) ++W.epoch;
    if (hipMemsetAsync(W.ctrl, 0, sizeof(int), st) != hipSuccess) return fail(-4, "memset");
    WfParams P;
    P.soup = soup;
    P.cell = cell;
    P.hb = W.hb;
    P.hc = W.hc;
    P.tasks = W.tasks;
    P.queue = W.ctrl;
    P.err = W.ctrl + 1;
    P.stats = W.count_evals ? W.stats : nullptr;
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
    const int grid = ntasks < 1024 ? ntasks : 1024;
    hipLaunchKernelGGL(k_sweep_wavefront, dim3(grid), dim3(WF_THREADS), 0, st, P);
    if (hipGetLastError() != hipSuccess) return fail(-4, "launch failed");
    return 0;
}

inline void wavefront_release(WavefrontWorkspace &W)
{
    (void)hipFree(W.hb);
    (void)hipFree(W.hc);
    (void)hipFree(W.tasks);
    (void)hipFree(W.ctrl);
    (void)hipFree(W.stats);
    W = WavefrontWorkspace();
}

}  // namespace sdfhip
