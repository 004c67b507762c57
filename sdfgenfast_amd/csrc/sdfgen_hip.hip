// sdfgen_hip.hip -- MI355X (gfx950) backend for make_level_set3 behind the C-ABI in
// include/sdfgen_hip.h.
//
// Pipeline (one HIP stream per call):
//   k_prep   : gather the indexed mesh into a per-triangle vertex soup (48 B/tri),
//              validate indices, initialise the cell state         (:196-199)
//   k_band_lds: batches of BAND_BT (64) consecutive triangles per workgroup -- exact distances over
//              the band boxes, merged per cell in LDS, then one global atomicMin on the
//              packed u64 key (f32bits(d)<<32 | t) that reproduces the CPU's
//              ascending-t strict-< rule; ray-parity counts (:203-236)
//   sweeps   : 2 passes x 8 directions of the Gauss-Seidel sweep (:238-292),
//              reproduced bit-exactly by a hyperplane-ordered wavefront
//   k_sign   : one wave per (j,k) row -- ballot prefix parity, sign flip, i-fastest output
//              (:294-303); k_sign_kfast the same through an LDS tile for k-fastest output
// Cell state is one u64 per cell: high word = phi bits, low word = closest_tri.
// Line references are to /root/reference/cpu_lib/makelevelset3.cpp unless noted.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <vector>

#include "geom.hpp"
#include "sdfgen_hip.h"
#include "sweep_tile.hpp"
#include "sweep_sparse.hpp"

using namespace sdfhip;

namespace {

typedef unsigned long long u64;

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
struct Err {
    char *buf;
    size_t len;
    int set(int code, const char *fmt, ...)
    {
        if (buf && len) {
            va_list ap;
            va_start(ap, fmt);
            vsnprintf(buf, len, fmt, ap);
            va_end(ap);
        }
        return code;
    }
};

// Every C-ABI entry point that selects a device restores the caller's current device on return
// (success or error): the reference runs on, and leaves, the current device
// (gpu_lib/makelevelset3_gpu.cu:600-603), so a later call on the current device must not land on
// whichever GPU an earlier multi-device call touched last.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return err.set(e_ == hipErrorOutOfMemory ? SDFGEN_HIP_ENOMEM : SDFGEN_HIP_ERUNTIME, \
                           "GPU (HIP) error %s at %s:%d: %s", hipGetErrorName(e_), __FILE__,    \
                           __LINE__, #expr);                                                    \
    } while (0)

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

// Gather the indexed mesh into 3 float4 per triangle; validate indices; init cells.
__global__ void k_prep_soup(const uint32_t *__restrict__ tri, uint64_t ntri, const float *__restrict__ xyz,
                            uint64_t nvert, float4 *__restrict__ soup, int *__restrict__ err_flag)
{
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < ntri;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t v[3] = {tri[3 * t + 0], tri[3 * t + 1], tri[3 * t + 2]};
        f3 x[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            uint64_t q = v[c];
            if (q >= nvert) {
                atomicOr(err_flag, 1);
                q = 0;
            }
            const uint64_t xq = SDF_CHK(40, 3 * q, 0, 3 * nvert);
            x[c] = mk3(xyz[xq + 0], xyz[xq + 1], xyz[xq + 2]);
        }
        // w of the third vertex: the triangle's tri_invdet (read by every ptd_wave / ptd_wave2)
        (void)SDF_CHK(41, 3 * t + 2, 0, 3 * ntri);
        soup[3 * t + 0] = make_float4(x[0].x, x[0].y, x[0].z, 0.0f);
        soup[3 * t + 1] = make_float4(x[1].x, x[1].y, x[1].z, 0.0f);
        soup[3 * t + 2] = make_float4(x[2].x, x[2].y, x[2].z, tri_invdet(x[0], x[1], x[2]));
    }
}

__global__ void k_init(u64 *__restrict__ cell, uint32_t *__restrict__ cnt, uint64_t n, u64 init_key)
{
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
        cell[q] = init_key;
        cnt[q] = 0u;
    }
}

struct Grid {
    float ox, oy, oz, dx;
    int ni, nj, nk;
};

__device__ __forceinline__ f3 load_vtx(const float4 *soup, uint64_t t, int c)
{
    float4 v = soup[3 * t + c];
    return mk3(v.x, v.y, v.z);
}

__device__ __forceinline__ size_t cidx(int i, int j, int k, int ni, int nj)
{
    return (size_t)i + (size_t)ni * ((size_t)j + (size_t)nj * (size_t)k);
}

// ---------------------------------------------------------------------------
// Narrow band + ray parity (:203-236).
//
// Two work classes, so that no workgroup ever holds more than a bounded amount of work and no
// count can wrap (triangle boxes reach 2^30 cells at 1024^3, and a batch of them 2^36):
//   * small triangles (band box <= BAND_BIG_VOL cells and ray lattice <= BAND_BIG_LAT points) --
//     the sub-cell triangles of a fine mesh -- in batches of BAND_BT consecutive triangles per
//     workgroup (k_band_lds): the batch's (triangle, cell) pairs flattened over 256 threads,
//     candidates merged per cell in LDS (ds_min_u64 on (f32bits(d) << 32 | t)) and one global
//     atomicMin per cell of the union box; the batch's ray-lattice points flattened the same way;
//   * big triangles -- coarse meshes, a wide exact_band, grid-spanning faces -- are appended to a
//     list by the batch kernel, a one-workgroup scan turns their chunk counts into 64-bit offsets
//     (k_band_big_scan), and k_band_big spreads the chunks (BAND_CH_PAIRS cells or BAND_CH_LAT
//     lattice points of one triangle) over every wave of the chip.
// min() and the parity counts are order-independent, so the result is the one-triangle-at-a-time
// result bit for bit whatever runs where.
// ---------------------------------------------------------------------------
#ifndef BAND_BT_DEF
#define BAND_BT_DEF 64   // 64 (with the 40 KB table): band 0.86 -> 0.81 ms at C3; 16: 0.99
#endif
#ifndef BAND_LDS_DEF
#define BAND_LDS_DEF 4000   // 31 KB: with BAND_WPE 4, four workgroups per CU (5120, 40 KB: three)
#endif
#ifndef BAND_FDIV
#define BAND_FDIV 1      // box coordinates by float reciprocal + one exact correction: band 0.797 -> 0.765 ms at C3
#endif
#ifndef BAND_WQ
#define BAND_WQ 1        // triangle of a pair by a wave-wide search (no binary search): with FDIV 0.797 -> 0.676 ms at C3, 1.30 -> 1.19 at C4
#endif
// diagnostics only (wrong results): BAND_DIAG_NOPTD (a pair's distance without the point-triangle
// evaluation), BAND_DIAG_NOFLUSH (no global atomics from the LDS table), BAND_DIAG_NOPAIR (no pairs:
// the batches' set-up, ray parity, table initialisation and barriers)
constexpr int BAND_BT = BAND_BT_DEF;    // triangles per batch (<= 64: one wave sets a batch up)
constexpr int BAND_LDS = BAND_LDS_DEF;  // u64 keys in the LDS table (31 KB)
static_assert(BAND_BT >= 1 && BAND_BT <= 64, "a batch's boxes are scanned by one wave");
// find_q's binary search halves from BAND_BT / 2: it reaches every triangle only for a power of two
// (BAND_BT_DEF=48 measured a digest mismatch at C3: triangle 47 of a batch was never paired)
static_assert((BAND_BT & (BAND_BT - 1)) == 0, "BAND_BT must be a power of two");
constexpr uint32_t BAND_BIG_VOL = 4096;    // band-box cells above which a triangle is "big"
constexpr uint32_t BAND_BIG_LAT = 1024;    // ray-lattice points above which a triangle is "big"
constexpr uint32_t BAND_CH_PAIRS = 1024;   // cells per big-triangle chunk (one wave: 16 per lane)
constexpr uint32_t BAND_CH_LAT = 256;      // lattice points per big-triangle chunk (4 per lane)
// a batch's flattened counts stay far inside 32 bits
static_assert((uint64_t)BAND_BT * BAND_BIG_VOL < (1ull << 31) && (uint64_t)BAND_BT * BAND_BIG_LAT < (1ull << 31), "");

struct BandBox {
    int i0, j0, k0, bi, bj, bk;         // clamped band box (bi*bj*bk cells; 0 = empty)
};
struct LatBox {
    int j0, k0, nj, nk;                 // clamped ray lattice (nj*nk (j,k) points; 0 = empty)
};

// Grid coordinates of the triangle's vertices (:206-208) and its band box (:210-212), cut to the
// slab's planes [k_lo, k_hi) AFTER the reference's whole-grid clamp.
__device__ __forceinline__ void band_box(const float4 *soup, uint64_t t, const Grid &g, int band, int k_lo, int k_hi,
                                         BandBox &B, double f[9])
{
    const f3 xp = load_vtx(soup, t, 0), xq = load_vtx(soup, t, 1), xr = load_vtx(soup, t, 2);
    const double ox = g.ox, oy = g.oy, oz = g.oz, ddx = g.dx;
    f[0] = ((double)xp.x - ox) / ddx; f[1] = ((double)xp.y - oy) / ddx; f[2] = ((double)xp.z - oz) / ddx;
    f[3] = ((double)xq.x - ox) / ddx; f[4] = ((double)xq.y - oy) / ddx; f[5] = ((double)xq.z - oz) / ddx;
    f[6] = ((double)xr.x - ox) / ddx; f[7] = ((double)xr.y - oy) / ddx; f[8] = ((double)xr.z - oz) / ddx;
    const int i0 = clampi(wrap_add(trunc_to_int(dmin3(f[0], f[3], f[6])), -band), 0, g.ni - 1);
    const int i1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(f[0], f[3], f[6])), band), 1), 0, g.ni - 1);
    const int j0 = clampi(wrap_add(trunc_to_int(dmin3(f[1], f[4], f[7])), -band), 0, g.nj - 1);
    const int j1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(f[1], f[4], f[7])), band), 1), 0, g.nj - 1);
    int k0 = clampi(wrap_add(trunc_to_int(dmin3(f[2], f[5], f[8])), -band), 0, g.nk - 1);
    int k1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(f[2], f[5], f[8])), band), 1), 0, g.nk - 1);
    k0 = max(k0, k_lo);
    k1 = min(k1, k_hi - 1);
    B.i0 = i0;
    B.j0 = j0;
    B.k0 = k0;
    const bool ok = i1 >= i0 && j1 >= j0 && k1 >= k0;
    B.bi = ok ? i1 - i0 + 1 : 0;
    B.bj = ok ? j1 - j0 + 1 : 0;
    B.bk = ok ? k1 - k0 + 1 : 0;
}

// The ray lattice of :222-225 (its own clamp, independent of the band box: for a NaN, infinite or
// far vertex the two boxes differ), cut to the slab's planes.
__device__ __forceinline__ void lat_box(const double f[9], const Grid &g, int k_lo, int k_hi, LatBox &L)
{
    const int j0 = clampi(trunc_to_int(ceil(dmin3(f[1], f[4], f[7]))), 0, g.nj - 1);
    const int j1 = clampi(trunc_to_int(floor(dmax3(f[1], f[4], f[7]))), 0, g.nj - 1);
    const int k0 = max(clampi(trunc_to_int(ceil(dmin3(f[2], f[5], f[8]))), 0, g.nk - 1), k_lo);
    const int k1 = min(clampi(trunc_to_int(floor(dmax3(f[2], f[5], f[8]))), 0, g.nk - 1), k_hi - 1);
    const bool ok = j1 >= j0 && k1 >= k0;
    L.j0 = j0;
    L.k0 = k0;
    L.nj = ok ? j1 - j0 + 1 : 0;
    L.nk = ok ? k1 - k0 + 1 : 0;
}

// One lattice point of the ray-parity test (:226-235).
__device__ __forceinline__ void parity_point(const double *f, int j, int k, const Grid &g, uint32_t *cnt, int k_lo, int k_hi)
{
    (void)k_lo;
    (void)k_hi;
    double a, b, cc;
    if (pit2d((double)j, (double)k, f[1], f[2], f[4], f[5], f[7], f[8], a, b, cc)) {
        const double fi = (a * f[0] + b * f[3]) + cc * f[6];
        const int ii = trunc_to_int(ceil(fi));
        // (bounds builds: k of a lattice point lies in the slab's planes; the range is the slab's cnt)
        [[maybe_unused]] const size_t plane = (size_t)g.ni * g.nj;
        if (ii < 0) atomicAdd(cnt + SDF_CHK(45, cidx(0, j, k, g.ni, g.nj), plane * k_lo, plane * k_hi), 1u);
        else if (ii < g.ni) atomicAdd(cnt + SDF_CHK(45, cidx(ii, j, k, g.ni, g.nj), plane * k_lo, plane * k_hi), 1u);
    }
}

// The big-triangle list of one call: appended by k_band_lds, offsets by k_band_big_scan.
struct BandBig {
    uint32_t *tri;      // [cap] triangle index
    uint32_t *chunks;   // [cap] chunk count (pair chunks, then lattice chunks)
    u64 *pre;           // [cap + 1] exclusive prefix of chunks; pre[n] = total
    uint32_t *n;        // entries appended (zeroed per call)
};

__device__ __forceinline__ uint32_t ceil_div64(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

// Last q in [0, nb) with pre[q] <= fl (pre ascending, pre[0] = 0).
__device__ __forceinline__ int find_q(const unsigned *pre, int nb, unsigned fl)
{
    int q = 0;
#pragma unroll
    for (int step = BAND_BT / 2; step >= 1; step >>= 1)
        if (q + step < nb && pre[q + step] <= fl) q += step;
    return q;
}

// The same q for a wave whose lanes carry consecutive flat indices F + lane: lane x holds pre[x]
// (lanes >= nb: UINT_MAX).  The offsets at or below F give lane 0's triangle; each offset inside
// (F, F + 63] -- usually none or one, a box holding ~90 cells -- moves the lanes at or past it on.
__device__ __forceinline__ int band_wq(unsigned pl, unsigned F, unsigned lane)
{
    int q = __popcll(__ballot(pl <= F)) - 1;
    unsigned long long m = __ballot(pl > F && pl - F <= 63u);
    const unsigned fl = F + lane;
    while (m) {
        const int b = __ffsll((long long)m) - 1;
        q += fl >= (unsigned)__builtin_amdgcn_readlane((int)pl, b) ? 1 : 0;
        m &= m - 1;
    }
    return q;
}

#ifndef BAND_WPE
#define BAND_WPE 4   // waves per SIMD the band kernel's register budget must allow: 128 VGPRs (166 unbounded; the
                     // spills stay in the batch set-up) and, with the 31 KB table, 4 workgroups per CU instead of 3:
                     // band C3 0.662 -> 0.629-0.635 ms, C4 1.18-1.19 -> 1.17-1.18 (profiles/r05aw_ab_band_c{3,4}.log);
                     // 5 waves (96 VGPRs) spill inside the pair loop
#endif
__global__ void __launch_bounds__(256, BAND_WPE) k_band_lds(const float4 *__restrict__ soup, uint64_t ntri, Grid g, int band,
                                                  float init, u64 *__restrict__ cell, uint32_t *__restrict__ cnt,
                                                  unsigned long long *__restrict__ eval_count, int k_lo, int k_hi,
                                                  BandBig big)
{
    __shared__ u64 s_key[BAND_LDS];
    __shared__ BandBox s_box[BAND_BT];
    __shared__ LatBox s_lat[BAND_BT];
    __shared__ double s_f[BAND_BT][9];        // grid coordinates of the batch's vertices (parity)
    __shared__ unsigned s_pre[BAND_BT + 1];   // prefix sums of the box volumes
    __shared__ unsigned s_lpre[BAND_BT + 1];  // prefix sums of the lattice sizes
    __shared__ int s_u[6];                    // union box: i0, j0, k0, ni, nj, nk
    const int tid = threadIdx.x;
    unsigned long long evals = 0;
    for (uint64_t t0 = (uint64_t)blockIdx.x * BAND_BT; t0 < ntri; t0 += (uint64_t)gridDim.x * BAND_BT) {
        const int nb = (int)min<uint64_t>(BAND_BT, ntri - t0);
        if (tid < 64) {
            // wave 0, lane q = triangle t0 + q (lanes >= nb carry empty boxes): boxes, the big-triangle
            // hand-off, prefix sums of the box and lattice sizes and the union box -- no single-thread loop
            BandBox B{0, 0, 0, 0, 0, 0};
            LatBox L{0, 0, 0, 0};
            double f[9];
            if (tid < nb) {
                band_box(soup, t0 + tid, g, band, k_lo, k_hi, B, f);
                lat_box(f, g, k_lo, k_hi, L);
            }
            const uint64_t vol = (uint64_t)B.bi * (uint64_t)B.bj * (uint64_t)B.bk;
            const uint64_t lat = (uint64_t)L.nj * (uint64_t)L.nk;
            const bool is_big = vol > BAND_BIG_VOL || lat > BAND_BIG_LAT;
            const u64 bm = __ballot(is_big);
            if (bm) {   // one append per wave
                uint32_t base = 0;
                if (tid == __ffsll((long long)bm) - 1) base = atomicAdd(big.n, (uint32_t)__popcll(bm));
                base = __shfl(base, __ffsll((long long)bm) - 1);
                if (is_big) {
                    const uint32_t slot = base + (uint32_t)__popcll(bm & ((1ull << tid) - 1ull));
                    big.tri[slot] = (uint32_t)(t0 + tid);
                    big.chunks[slot] = ceil_div64(vol, BAND_CH_PAIRS) + ceil_div64(lat, BAND_CH_LAT);
                    B = BandBox{0, 0, 0, 0, 0, 0};
                    L = LatBox{0, 0, 0, 0};
                }
            }
            if (tid < BAND_BT) {   // (lanes >= BAND_BT only exist in builds with smaller batches)
                s_box[tid] = B;
                s_lat[tid] = L;
            }
            if (tid < BAND_BT && L.nj) {
#pragma unroll
                for (int c = 0; c < 9; ++c) s_f[tid][c] = f[c];
            }
            const unsigned v32 = (unsigned)(B.bi * B.bj * B.bk), l32 = (unsigned)(L.nj * L.nk);
            unsigned incl = v32, lincl = l32;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const unsigned y = __shfl_up(incl, d), ly = __shfl_up(lincl, d);
                if (tid >= d) {
                    incl += y;
                    lincl += ly;
                }
            }
            if (tid < nb) {
                s_pre[tid] = incl - v32;
                s_lpre[tid] = lincl - l32;
            }
            if (tid == nb - 1) {
                s_pre[nb] = incl;
                s_lpre[nb] = lincl;
            }
            int ui0 = B.bi ? B.i0 : INT_MAX, uj0 = B.bi ? B.j0 : INT_MAX, uk0 = B.bi ? B.k0 : INT_MAX;
            int ui1 = B.bi ? B.i0 + B.bi - 1 : -1, uj1 = B.bi ? B.j0 + B.bj - 1 : -1, uk1 = B.bi ? B.k0 + B.bk - 1 : -1;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                ui0 = min(ui0, __shfl_xor(ui0, d)); uj0 = min(uj0, __shfl_xor(uj0, d)); uk0 = min(uk0, __shfl_xor(uk0, d));
                ui1 = max(ui1, __shfl_xor(ui1, d)); uj1 = max(uj1, __shfl_xor(uj1, d)); uk1 = max(uk1, __shfl_xor(uk1, d));
            }
            if (tid == 0) {
                s_u[0] = ui0; s_u[1] = uj0; s_u[2] = uk0;
                s_u[3] = ui1 >= ui0 ? ui1 - ui0 + 1 : 0;
                s_u[4] = uj1 >= uj0 ? uj1 - uj0 + 1 : 0;
                s_u[5] = uk1 >= uk0 ? uk1 - uk0 + 1 : 0;
            }
        }
        __syncthreads();
        const unsigned total = s_pre[nb], ltotal = s_lpre[nb];
        evals += tid == 0 ? total : 0;
        const int ui0 = s_u[0], uj0 = s_u[1], uk0 = s_u[2], uni = s_u[3], unj = s_u[4];
        const unsigned long long uvol = (unsigned long long)uni * unj * (unsigned)s_u[5];
        const bool merge = uvol > 0 && uvol <= BAND_LDS;
        if (merge)
            for (unsigned c = tid; c < uvol; c += 256) s_key[c] = ~0ull;
        // the batch's ray-lattice points over all 256 threads (:222-235)
        for (unsigned fl = tid; fl < ltotal; fl += 256) {
            const int q = (int)SDF_CHK(42, find_q(s_lpre, nb, fl), 0, nb);
            const LatBox L = s_lat[q];
            const unsigned r = fl - s_lpre[q], kk = r / (unsigned)L.nj;
            parity_point(s_f[q], L.j0 + (int)(r - kk * (unsigned)L.nj), L.k0 + (int)kk, g, cnt, k_lo, k_hi);
        }
        __syncthreads();
        // (triangle, cell) pair of flat index fl (triangle q of the batch)
        auto pair_in = [&](int q, unsigned fl, int &i, int &j, int &k) {
            // bounds builds: the pair's triangle is one of the batch's, and a live pair's fl lies in its box
            // (lanes past the batch's last pair decode one too, never emitted)
            q = (int)SDF_CHK(42, q, 0, nb);
            if (fl < total) (void)SDF_CHK(43, fl, s_pre[q], s_pre[q + 1]);
            const BandBox B = s_box[q];
            const unsigned r = fl - s_pre[q], bij = (unsigned)(B.bi * B.bj);
#if BAND_FDIV
            // r < bi*bj*bk <= BAND_BIG_VOL (a small triangle's box): the float quotient is within 1 of
            // the exact one (|error| < 4096 * 2^-22), and one signed correction makes it exact
            auto qdiv = [](unsigned x, unsigned d, unsigned &rm) {
                int qq = (int)((float)x * __builtin_amdgcn_rcpf((float)d));
                int rr = (int)x - qq * (int)d;
                qq = rr < 0 ? qq - 1 : (rr >= (int)d ? qq + 1 : qq);
                rr = rr < 0 ? rr + (int)d : (rr >= (int)d ? rr - (int)d : rr);
                rm = (unsigned)rr;
                return (unsigned)qq;
            };
            unsigned rem, ii;
            const unsigned kk = qdiv(r, bij, rem), jj = qdiv(rem, (unsigned)B.bi, ii);
            i = B.i0 + (int)ii;
#else
            const unsigned kk = r / bij, rem = r - kk * bij, jj = rem / (unsigned)B.bi;
            i = B.i0 + (int)(rem - jj * (unsigned)B.bi);
#endif
            j = B.j0 + (int)jj;
            k = B.k0 + (int)kk;
        };
        auto emit = [&](float d, int i, int j, int k, uint64_t t) {
            if (d < init) {   // also rejects NaN
                const u64 key = ((u64)__float_as_uint(d) << 32) | (u64)(uint32_t)t;
                if (merge) {
                    atomicMin(&s_key[SDF_CHK(46, (unsigned)((k - uk0) * unj + (j - uj0)) * (unsigned)uni + (unsigned)(i - ui0), 0,
                                             uvol)], key);
                } else {
                    u64 *p = cell + SDF_CHK(44, cidx(i, j, k, g.ni, g.nj), (size_t)g.ni * g.nj * k_lo, (size_t)g.ni * g.nj * k_hi);
                    if (key < *p) atomicMin(p, key);
                }
            }
        };
        // two pairs per lane (F + L and F + 256 + L for lane L of a wave at F, a wave-uniform loop),
        // evaluated together in packed FP32 (ptd_wave2)
        {
            const unsigned lane = (unsigned)tid & 63u;
#if BAND_WQ
            const unsigned pl = lane < (unsigned)nb ? s_pre[lane] : 0xffffffffu;
#endif
#if BAND_DIAG_NOPAIR
            if (false)
#endif
            for (unsigned F = (unsigned)tid - lane; F < total; F += 512) {
                const unsigned fa = F + lane, fb = fa + 256;
                const bool one = fa < total, two = fb < total;
#if BAND_WQ
                // both searches by the whole wave (their ballots need every lane), then selected
                const int qa = band_wq(pl, F, lane), qb0 = band_wq(pl, F + 256, lane);
                const int qb = two ? qb0 : qa;
#else
                const int qa = find_q(s_pre, nb, fa), qb = two ? find_q(s_pre, nb, fb) : qa;
#endif
                int i, j, k, i2, j2, k2;
                pair_in(qa, fa, i, j, k);
                pair_in(qb, two ? fb : fa, i2, j2, k2);
                const f3 gx = mk3((float)i * g.dx + g.ox, (float)j * g.dx + g.oy, (float)k * g.dx + g.oz);
                const f3 gx2 = mk3((float)i2 * g.dx + g.ox, (float)j2 * g.dx + g.oy, (float)k2 * g.dx + g.oz);
                const float4 *sa = soup + 3 * SDF_CHK(47, t0 + qa, 0, ntri), *sb = soup + 3 * SDF_CHK(47, t0 + qb, 0, ntri);
                const float4 a0 = sa[0], a1 = sa[1], a2 = sa[2], b0 = sb[0], b1 = sb[1], b2 = sb[2];
                float d, d2 = 0.0f;
#if BAND_DIAG_NOPTD
                d = (float)(i + j + k) * g.dx + a0.x * 0.0f;
                d2 = (float)(i2 + j2 + k2) * g.dx + b0.x * 0.0f;
#else
                if (__any(two)) {
                    ptd_wave2(gx, mk3(a0.x, a0.y, a0.z), mk3(a1.x, a1.y, a1.z), mk3(a2.x, a2.y, a2.z), a2.w, gx2,
                              mk3(b0.x, b0.y, b0.z), mk3(b1.x, b1.y, b1.z), mk3(b2.x, b2.y, b2.z), b2.w, d, d2);
                } else {
                    d = ptd_wave(gx, mk3(a0.x, a0.y, a0.z), mk3(a1.x, a1.y, a1.z), mk3(a2.x, a2.y, a2.z), a2.w);
                }
#endif
                if (one) emit(d, i, j, k, t0 + qa);
                if (two) emit(d2, i2, j2, k2, t0 + qb);
            }
        }
        __syncthreads();
#if BAND_DIAG_NOFLUSH
        if (false)
#endif
        if (merge)
            for (unsigned c = tid; c < uvol; c += 256) {
                const u64 key = s_key[c];
                if (key == ~0ull) continue;
                const unsigned ij = (unsigned)(uni * unj), kk = c / ij, rem = c - kk * ij, jj = rem / (unsigned)uni;
                u64 *p = cell + SDF_CHK(44, cidx(ui0 + (int)(rem - jj * (unsigned)uni), uj0 + (int)jj, uk0 + (int)kk, g.ni, g.nj),
                                        (size_t)g.ni * g.nj * k_lo, (size_t)g.ni * g.nj * k_hi);
                atomicMin(p, key);   // no load-compare first: 0.81 -> 0.78 ms at C3 (no return to wait for)
            }
        __syncthreads();
    }
    if (eval_count && tid == 0 && evals) atomicAdd(eval_count, evals);
}

// Exclusive prefix of the big triangles' chunk counts in 64 bits (one workgroup; the list holds at
// most one entry per BAND_BIG_VOL cells or BAND_BIG_LAT lattice points of band work, so this scan
// is small against the work it dispatches, and empty -- one wave reading one word -- for fine meshes).
__global__ void __launch_bounds__(1024) k_band_big_scan(BandBig big)
{
    __shared__ u64 s_w[16];
    __shared__ u64 s_carry;
    const uint32_t n = *big.n;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < n; b += 1024) {
        const uint32_t e = b + tid;
        const u64 v = e < n ? big.chunks[e] : 0;
        u64 incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u64 y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        u64 wbase = s_carry;
        for (int q = 0; q < w; ++q) wbase += s_w[q];
        if (e < n) big.pre[e] = wbase + incl - v;
        __syncthreads();
        if (tid == 1023) s_carry = wbase + incl;
        __syncthreads();
    }
    if (tid == 0) big.pre[n] = s_carry;
}

// The big triangles' chunks, one per wave at a time over the whole chip: chunk c of entry e is
// BAND_CH_PAIRS consecutive cells of the triangle's band box (c < its pair chunks) or BAND_CH_LAT
// consecutive points of its ray lattice.  No LDS merge: a big triangle's cells are distinct, and
// the load-compare keeps the atomics to the cells it improves.
__global__ void __launch_bounds__(256) k_band_big(const float4 *__restrict__ soup, Grid g, int band, float init,
                                                  u64 *__restrict__ cell, uint32_t *__restrict__ cnt,
                                                  unsigned long long *__restrict__ eval_count, int k_lo, int k_hi,
                                                  BandBig big)
{
    const uint32_t n = *big.n;
    if (n == 0) return;
    const u64 total = big.pre[n];
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    unsigned long long evals = 0;
    for (uint64_t q = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); q < total; q += nw) {
        // entry: the last e with pre[e] <= q, by a 64-ary search across the wave's lanes
        uint32_t lo = 0, hi = n;
        while (hi - lo > 1) {
            const uint32_t step = (hi - lo + 63) / 64, x = lo + (uint32_t)lane * step;
            const u64 m = __ballot(x < hi && big.pre[x] <= q);   // lanes 0 .. c-1 (pre ascending; lane 0 always)
            const uint32_t c = (uint32_t)__popcll(m);
            lo += (c - 1) * step;
            hi = min(hi, lo + step);
        }
        const uint32_t e = (uint32_t)SDF_CHK(48, lo, 0, n);
        const uint64_t t = big.tri[e];
        BandBox B;
        LatBox L;
        double f[9];
        band_box(soup, t, g, band, k_lo, k_hi, B, f);
        lat_box(f, g, k_lo, k_hi, L);
        const uint64_t vol = (uint64_t)B.bi * (uint64_t)B.bj * (uint64_t)B.bk;
        const uint64_t lat = (uint64_t)L.nj * (uint64_t)L.nk;
        const uint64_t c = q - big.pre[e];
        const uint64_t npc = (vol + BAND_CH_PAIRS - 1) / BAND_CH_PAIRS;
        if (c < npc) {
            // cells [c * CH, c * CH + CH) of the box, i fastest: decode the chunk start once (64-bit),
            // then each cell as a small offset from it (32-bit)
            const uint64_t b0 = c * BAND_CH_PAIRS, bij = (uint64_t)B.bi * (uint64_t)B.bj;
            const uint32_t rk = (uint32_t)(b0 / bij);
            const uint64_t rem = b0 - (uint64_t)rk * bij;   // < bi * bj, which may pass 2^32
            const uint32_t rj = (uint32_t)(rem / (uint64_t)B.bi), ri = (uint32_t)(rem - (uint64_t)rj * B.bi);
            const uint32_t nvalid = (uint32_t)min<uint64_t>(BAND_CH_PAIRS, vol - b0);
            evals += lane == 0 ? nvalid : 0;
            const f3 x1 = load_vtx(soup, t, 0), x2 = load_vtx(soup, t, 1), x3 = load_vtx(soup, t, 2);
            const float inv = soup[3 * t + 2].w;
            auto cell_of = [&](uint32_t r, int &i, int &j, int &k) {
                const uint32_t ii = ri + r, cj = ii / (uint32_t)B.bi;
                const uint32_t jj = rj + cj, ck = jj / (uint32_t)B.bj;
                i = B.i0 + (int)(ii - cj * (uint32_t)B.bi);
                j = B.j0 + (int)(jj - ck * (uint32_t)B.bj);
                k = B.k0 + (int)(rk + ck);
            };
            auto emit = [&](float d, int i, int j, int k) {
                if (d < init) {   // also rejects NaN
                    const u64 key = ((u64)__float_as_uint(d) << 32) | (u64)(uint32_t)t;
                    u64 *p = cell + SDF_CHK(44, cidx(i, j, k, g.ni, g.nj), (size_t)g.ni * g.nj * k_lo, (size_t)g.ni * g.nj * k_hi);
                    if (key < *p) atomicMin(p, key);
                }
            };
            for (uint32_t r = lane; r < nvalid; r += 128) {   // two cells per lane in packed FP32
                const bool two = r + 64 < nvalid;
                int i, j, k, i2, j2, k2;
                cell_of(r, i, j, k);
                cell_of(two ? r + 64 : r, i2, j2, k2);
                const f3 gx = mk3((float)i * g.dx + g.ox, (float)j * g.dx + g.oy, (float)k * g.dx + g.oz);
                const f3 gx2 = mk3((float)i2 * g.dx + g.ox, (float)j2 * g.dx + g.oy, (float)k2 * g.dx + g.oz);
                float d, d2 = 0.0f;
                if (__any(two)) ptd_wave2(gx, x1, x2, x3, inv, gx2, x1, x2, x3, inv, d, d2);
                else d = ptd_wave(gx, x1, x2, x3, inv);
                emit(d, i, j, k);
                if (two) emit(d2, i2, j2, k2);
            }
        } else {
            const uint64_t b0 = (c - npc) * BAND_CH_LAT;
            const uint32_t rk = (uint32_t)(b0 / (uint64_t)L.nj), rj = (uint32_t)(b0 - (uint64_t)rk * L.nj);
            const uint32_t nvalid = (uint32_t)min<uint64_t>(BAND_CH_LAT, lat - b0);
            for (uint32_t r = lane; r < nvalid; r += 64) {
                const uint32_t jj = rj + r, ck = jj / (uint32_t)L.nj;
                parity_point(f, L.j0 + (int)(jj - ck * (uint32_t)L.nj), L.k0 + (int)(rk + ck), g, cnt, k_lo, k_hi);
            }
        }
    }
    if (eval_count && lane == 0 && evals) atomicAdd(eval_count, evals);
}

// Buffers of the big-triangle list (grow-only, one entry per triangle at most).
struct BandWork {
    BandBig big{nullptr, nullptr, nullptr, nullptr};
    size_t cap = 0;
};

int band_reserve(BandWork &bw, uint64_t ntri, Err &err)
{
    if (!bw.big.n) HIPCHK(hipMalloc((void **)&bw.big.n, 64));
    if (bw.cap >= ntri && bw.big.tri) return 0;
    (void)hipFree(bw.big.tri);
    (void)hipFree(bw.big.chunks);
    (void)hipFree(bw.big.pre);
    bw.big.tri = bw.big.chunks = nullptr;
    bw.big.pre = nullptr;
    bw.cap = 0;
    const size_t c = std::max<uint64_t>(ntri, 1);
    HIPCHK(hipMalloc((void **)&bw.big.tri, c * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void **)&bw.big.chunks, c * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void **)&bw.big.pre, (c + 1) * sizeof(u64)));
    bw.cap = c;
    return 0;
}

void band_release(BandWork &bw)
{
    (void)hipFree(bw.big.tri);
    (void)hipFree(bw.big.chunks);
    (void)hipFree(bw.big.pre);
    (void)hipFree(bw.big.n);
    bw = BandWork{};
}

// One sweep cell update: the CPU's sequential check_neighbour chain (:90-102, :143-149)
// with the exact skips (a candidate equal to the cell's own original label, or to an
// earlier candidate's label, evaluates to the same float and can never pass strict <).
__device__ __forceinline__ void sweep_cell(const float4 *__restrict__ soup, u64 *__restrict__ cell, const Grid &g,
                                           int i, int j, int k, int di, int dj, int dk)
{
    const size_t c0 = cidx(i, j, k, g.ni, g.nj);
    const u64 own = cell[c0];
    float phi = __uint_as_float((uint32_t)(own >> 32));
    int32_t ct = lbl_of((uint32_t)own);
    const int32_t ct_orig = ct;
    int32_t nb[7];
    nb[0] = lbl_of((uint32_t)cell[cidx(i - di, j, k, g.ni, g.nj)]);
    nb[1] = lbl_of((uint32_t)cell[cidx(i, j - dj, k, g.ni, g.nj)]);
    nb[2] = lbl_of((uint32_t)cell[cidx(i - di, j - dj, k, g.ni, g.nj)]);
    nb[3] = lbl_of((uint32_t)cell[cidx(i, j, k - dk, g.ni, g.nj)]);
    nb[4] = lbl_of((uint32_t)cell[cidx(i - di, j, k - dk, g.ni, g.nj)]);
    nb[5] = lbl_of((uint32_t)cell[cidx(i, j - dj, k - dk, g.ni, g.nj)]);
    nb[6] = lbl_of((uint32_t)cell[cidx(i - di, j - dj, k - dk, g.ni, g.nj)]);
    const f3 gx = mk3((float)i * g.dx + g.ox, (float)j * g.dx + g.oy, (float)k * g.dx + g.oz);
    bool changed = false;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int32_t t = nb[q];
        bool skip = (t < 0) || (t == ct_orig);
#pragma unroll
        for (int r = 0; r < q; ++r) skip = skip || (nb[r] == t);
        if (!skip) {
            float d = ptd(gx, load_vtx(soup, (uint64_t)t, 0), load_vtx(soup, (uint64_t)t, 1),
                          load_vtx(soup, (uint64_t)t, 2));
            if (d < phi) {
                phi = d;
                ct = t;
                changed = true;
            }
        }
    }
    if (changed) cell[c0] = ((u64)__float_as_uint(phi) << 32) | lo_word(ct, 0);
}

// Reference-order sweep, one launch per oriented hyperplane s = a+b+c:
// every upwind neighbour of a cell lies on hyperplane s-1..s-3, finished by earlier launches.
__global__ void __launch_bounds__(256) k_sweep_plane(const float4 *__restrict__ soup, u64 *__restrict__ cell, Grid g,
                                                     int di, int dj, int dk, int s, int a_lo, int b_lo, int b_cnt,
                                                     int n_threads)
{
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_threads) return;
    const int a = a_lo + idx / b_cnt;
    const int b = b_lo + idx % b_cnt;
    const int c = s - a - b;
    if (c < 0 || c >= g.nk - 1) return;
    if (b >= g.nj - 1) return;
    const int i = di > 0 ? a + 1 : g.ni - 2 - a;
    const int j = dj > 0 ? b + 1 : g.nj - 2 - b;
    const int k = dk > 0 ? c + 1 : g.nk - 2 - c;
    sweep_cell(soup, cell, g, i, j, k, di, dj, dk);
}

// Sign pass: one wave per (j,k) row; prefix parity by ballot, sign flip (-0.0 kept),
// output in Array3f (i-fastest) or k-fastest layout.   :294-303
// Rows k in [k_lo, k_lo + k_cnt); the output holds just those planes.
__global__ void __launch_bounds__(256) k_sign(const u64 *__restrict__ cell, const uint32_t *__restrict__ cnt, Grid g,
                                              int layout, float *__restrict__ out, int k_lo, int k_cnt)
{
    const int lane = threadIdx.x & 63;
    const uint64_t nrows = (uint64_t)g.nj * k_cnt;
    const uint64_t rstep = ((uint64_t)gridDim.x * blockDim.x) >> 6;   // grid-stride over rows (capped grid)
    for (uint64_t row = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6; row < nrows; row += rstep) {
        const int j = (int)(row % g.nj), k = k_lo + (int)(row / g.nj);
        const size_t base = SDF_CHK(49, cidx(0, j, k, g.ni, g.nj), (size_t)g.ni * g.nj * k_lo,
                                    (size_t)g.ni * g.nj * (k_lo + k_cnt));
        uint32_t carry = 0;
        for (int i0 = 0; i0 < g.ni; i0 += 64) {
            const int i = i0 + lane;
            const bool ok = i < g.ni;
            uint32_t par = ok ? (cnt[base + i] & 1u) : 0u;
            const u64 mask = __ballot(par);
            const u64 below = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);  // lanes 0..lane
            const uint32_t pre = (carry + (uint32_t)__popcll(mask & below)) & 1u;
            if (ok) {
                uint32_t bits = (uint32_t)(cell[base + i] >> 32);
                if (pre) bits ^= 0x80000000u;
                float v = __uint_as_float(bits);
                const size_t nout = (size_t)g.ni * g.nj * k_cnt;
                if (layout == SDFGEN_LAYOUT_ARRAY3) out[SDF_CHK(50, cidx(i, j, k - k_lo, g.ni, g.nj), 0, nout)] = v;
                else out[SDF_CHK(50, ((size_t)i * g.nj + j) * k_cnt + (k - k_lo), 0, nout)] = v;
                (void)nout;
            }
            carry = (carry + (uint32_t)__popcll(mask)) & 1u;
        }
    }
}

// The sign pass with k-fastest output (SDFGEN_LAYOUT_KFAST: numpy (ni,nj,nk) C-order, the .sdf body):
// k_sign's row walk along i would write every lane to its own line (stride nj*nk floats) -- 3.7 ms
// at 512^3 against 0.4 for i-fastest.  Here a workgroup owns 64 rows (j, k0..k0+63) and walks i in
// chunks of 64: each wave signs 16 of the rows (prefix parity along i by ballot, carries kept per
// row) into an LDS tile [k][i], then the tile is written transposed -- for each i, 64 consecutive k:
// one 256-byte run per wave store.
__global__ void __launch_bounds__(256) k_sign_kfast(const u64 *__restrict__ cell, const uint32_t *__restrict__ cnt,
                                                    Grid g, float *__restrict__ out, int k_lo, int k_cnt)
{
    __shared__ float s_t[64][65];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int kblocks = (k_cnt + 63) / 64;
    const uint64_t ntile = (uint64_t)g.nj * kblocks;
    const u64 below = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);   // lanes 0..lane
    for (uint64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const int j = (int)(tile % g.nj), kb = (int)(tile / g.nj) * 64;
        uint32_t carry[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) carry[r] = 0;
        for (int i0 = 0; i0 < g.ni; i0 += 64) {
            const int i = i0 + lane;
            const bool ok = i < g.ni;
#pragma unroll
            for (int r = 0; r < 16; ++r) {   // rows kb + 16 w + r (wave-uniform)
                const int kr = kb + 16 * w + r;
                if (kr < k_cnt) {
                    const size_t base = SDF_CHK(49, cidx(0, j, k_lo + kr, g.ni, g.nj), (size_t)g.ni * g.nj * k_lo,
                                                (size_t)g.ni * g.nj * (k_lo + k_cnt));
                    const uint32_t par = ok ? (cnt[base + i] & 1u) : 0u;
                    const u64 mask = __ballot(par);
                    const uint32_t pre = (carry[r] + (uint32_t)__popcll(mask & below)) & 1u;
                    uint32_t bits = ok ? (uint32_t)(cell[base + i] >> 32) : 0u;
                    if (pre) bits ^= 0x80000000u;
                    s_t[16 * w + r][lane] = __uint_as_float(bits);
                    carry[r] = (carry[r] + (uint32_t)__popcll(mask)) & 1u;
                }
            }
            __syncthreads();
            const int kk = kb + lane;
            for (int ii = w; ii < 64 && i0 + ii < g.ni; ii += 4)
                if (kk < k_cnt) out[SDF_CHK(50, ((size_t)(i0 + ii) * g.nj + j) * k_cnt + kk, 0, (size_t)g.ni * g.nj * k_cnt)] = s_t[lane][ii];
            __syncthreads();
        }
    }
}

// Diagnostics kernels (the parity tests' geometry entry points).
__global__ void k_debug_ptd(uint64_t n, const float *__restrict__ pts, float *__restrict__ out, int variant)
{
    uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (q >= n) return;
    const float *p = pts + 12 * q;
    const f3 x0 = mk3(p[0], p[1], p[2]), x1 = mk3(p[3], p[4], p[5]), x2 = mk3(p[6], p[7], p[8]),
             x3 = mk3(p[9], p[10], p[11]);
    if (variant == 3) {   // packed pair: this lane's point against its own and its neighbour's triangle
        const uint64_t q2 = (q ^ 1) < n ? (q ^ 1) : q;
        const float *r = pts + 12 * q2;
        float da, db;
        const f3 y1 = mk3(r[3], r[4], r[5]), y2 = mk3(r[6], r[7], r[8]), y3 = mk3(r[9], r[10], r[11]);
        ptd_wave2(x0, x1, x2, x3, tri_invdet(x1, x2, x3), x0, y1, y2, y3, tri_invdet(y1, y2, y3), da, db);
        out[q] = da;
        (void)db;
        return;
    }
    if (variant == 4) {   // packed pair, second half: the neighbour's point against this lane's triangle
        const uint64_t q2 = (q ^ 1) < n ? (q ^ 1) : q;
        const float *r = pts + 12 * q2;
        float da, db;
        const f3 y1 = mk3(r[3], r[4], r[5]), y2 = mk3(r[6], r[7], r[8]), y3 = mk3(r[9], r[10], r[11]);
        ptd_wave2(mk3(r[0], r[1], r[2]), y1, y2, y3, tri_invdet(y1, y2, y3), x0, x1, x2, x3, tri_invdet(x1, x2, x3),
                  da, db);
        out[q] = db;
        (void)da;
        return;
    }
    out[q] = variant == 0 ? ptd(x0, x1, x2, x3) : (variant == 1 ? ptd_nb(x0, x1, x2, x3) : ptd_wave(x0, x1, x2, x3, tri_invdet(x1, x2, x3)));
}

__global__ void k_debug_pit2d(uint64_t n, const double *__restrict__ in, double *__restrict__ out)
{
    uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *p = in + 8 * q;
    double a = 0, b = 0, c = 0;
    bool r = pit2d(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], a, b, c);
    out[4 * q] = r ? 1.0 : 0.0;
    out[4 * q + 1] = a;
    out[4 * q + 2] = b;
    out[4 * q + 3] = c;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
const int SWEEP_DIRS[8][3] = {{+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
                              {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};

// Status words of one call (run_pipeline): [0] prep error flag, [1] tile sweep error bits, [2] band
// evaluations, [3, 3 + ST_NSTATS) tile sweep statistics, then SP_NCTL sparse sweep control words.
constexpr int STATUS_SP = 3 + ST_NSTATS;
constexpr int STATUS_N = STATUS_SP + SP_NCTL;
__global__ void k_status(unsigned long long *__restrict__ out, const int *flag, const int *wf_err,
                         const unsigned long long *evals, const unsigned long long *wf_stats,
                         const unsigned long long *sp_ctl)
{
    for (int t = threadIdx.x; t < STATUS_N; t += blockDim.x) {
        unsigned long long v = 0;
        if (t == 0) v = (unsigned)*flag;
        else if (t == 1) v = wf_err ? (unsigned)*wf_err : 0u;
        else if (t == 2) v = *evals;
        else if (t < STATUS_SP) v = wf_stats ? wf_stats[t - 3] : 0ull;
        else v = sp_ctl ? sp_ctl[t - STATUS_SP] : 0ull;
        out[t] = v;
    }
}

struct Workspace {
    int device = -1;
    hipStream_t stream = nullptr;
    u64 *cell = nullptr;
    uint32_t *cnt = nullptr;
    float4 *soup = nullptr;
    uint32_t *tri = nullptr;
    float *xyz = nullptr;
    int *err_flag = nullptr;
    unsigned long long *evals = nullptr;
    unsigned long long *status = nullptr;   // STATUS_N words gathered by k_status, read back in one copy
    size_t cap_cell = 0, cap_cnt = 0, cap_soup = 0, cap_tri = 0, cap_xyz = 0;
    hipEvent_t ev[40] = {};
    bool ev_ok = false;
    std::mutex mu;
    TileSweepWorkspace wf;
    SparseSweepWorkspace sp;
    BandWork band;                      // the big-triangle list of the band phase
    float *out = nullptr;               // phi of the host-buffer entry point before its copy-out
    size_t cap_out = 0;
};

std::mutex g_mu;
std::vector<Workspace *> g_ws;
sdfgen_hip_profile g_prof;
std::mutex g_prof_mu;

template <class T>
int grow(T **p, size_t *cap, size_t need, Err &err)
{
    if (need <= *cap && *p) return 0;
    if (*p) {
        HIPCHK(hipFree(*p));
        *p = nullptr;
        *cap = 0;
    }
    size_t n = std::max<size_t>(need, 1);
    HIPCHK(hipMalloc((void **)p, n * sizeof(T)));
    *cap = n;
    return 0;
}

int get_ws(int device, Workspace **out, Err &err)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (Workspace *w : g_ws)
        if (w->device == device) {
            *out = w;
            return 0;
        }
    Workspace *w = new Workspace();
    w->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
    for (auto &e : w->ev) HIPCHK(hipEventCreate(&e));
    w->ev_ok = true;
    g_ws.push_back(w);
    *out = w;
    return 0;
}

int validate(uint64_t ntri, uint64_t nvert, float dx, int ni, int nj, int nk, int layout, Err &err)
{
    if (ni <= 0 || nj <= 0 || nk <= 0)
        return err.set(SDFGEN_HIP_EINVAL, "Grid dimensions must be positive (nx, ny, nz > 0)");
    if (!(dx > 0.0f) || !std::isfinite(dx)) return err.set(SDFGEN_HIP_EINVAL, "Cell spacing dx must be positive");
    if (layout != SDFGEN_LAYOUT_ARRAY3 && layout != SDFGEN_LAYOUT_KFAST)
        return err.set(SDFGEN_HIP_EINVAL, "out_layout must be 0 (Array3f) or 1 (k-fastest)");
    if ((uint64_t)ni * nj * nk >= (1ull << 40)) return err.set(SDFGEN_HIP_EINVAL, "grid too large");
    if (ntri >= (uint64_t)LBL_MASK)
        return err.set(SDFGEN_HIP_EINVAL, "too many triangles (the GPU backend supports up to %u)", LBL_MASK - 1u);
    (void)nvert;
    return 0;
}

inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap)
{
    uint64_t b = (n + block - 1) / block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

// Waves of k_band_big: 8 per CU (its chunks are independent; an empty list exits at once).
constexpr unsigned BAND_BIG_WG = 512;

// The band phase of one call (or one Z-slab's planes [k_lo, k_hi)) on stream st.
int band_enqueue(BandWork &bw, hipStream_t st, const float4 *soup, uint64_t ntri, const Grid &g, int band, float init,
                 u64 *cell, uint32_t *cnt, unsigned long long *evals, int k_lo, int k_hi, Err &err)
{
    if (!ntri) return 0;
    if (int rc = band_reserve(bw, ntri, err)) return rc;
    HIPCHK(zero_async(bw.big.n, sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_band_lds, dim3(grid_for((ntri + BAND_BT - 1) / BAND_BT, 1, 8192)), dim3(256), 0, st, soup, ntri,
                       g, band, init, cell, cnt, evals, k_lo, k_hi, bw.big);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_band_big_scan, dim3(1), dim3(1024), 0, st, bw.big);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_band_big, dim3(BAND_BIG_WG), dim3(256), 0, st, soup, g, band, init, cell, cnt, evals, k_lo, k_hi,
                       bw.big);
    HIPCHK(hipGetLastError());
    return 0;
}

// Bounds-checked builds (make BOUNDS=1): report the first out-of-range index a kernel formed.
int check_oob(Err &err, const char *where)
{
#ifdef SDFGEN_BOUNDS
    unsigned long long v = 0, z = 0;
    HIPCHK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(sdf_oob), sizeof(v)));
    if (v) {
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(sdf_oob), &z, sizeof(z)));
        return err.set(SDFGEN_HIP_ERUNTIME, "%s: out-of-range index at site %llu: %llu", where, v >> 48,
                       v & 0xffffffffffffull);
    }
#else
    (void)err;
    (void)where;
#endif
    return 0;
}

// The whole pipeline on device buffers already resident on ws->device.
int run_pipeline(Workspace *ws, hipStream_t st, const uint32_t *d_tri, uint64_t ntri, const float *d_xyz,
                 uint64_t nvert, const float origin[3], float dx, int ni, int nj, int nk, int band, int layout,
                 float *d_out, Err &err)
{
    const uint64_t n = (uint64_t)ni * nj * nk;
    int rc;
    if ((rc = grow(&ws->cell, &ws->cap_cell, sp_pad(n), err))) return rc;   // (k_sp_jscan2 reads past the last cell)
    if ((rc = grow(&ws->cnt, &ws->cap_cnt, n, err))) return rc;
    if ((rc = grow(&ws->soup, &ws->cap_soup, 3 * std::max<uint64_t>(ntri, 1), err))) return rc;
    if (!ws->err_flag) {
        HIPCHK(hipMalloc((void **)&ws->err_flag, sizeof(int)));
        HIPCHK(hipMalloc((void **)&ws->evals, sizeof(unsigned long long)));
        HIPCHK(hipMalloc((void **)&ws->status, STATUS_N * sizeof(unsigned long long)));
    }
    Grid g{origin[0], origin[1], origin[2], dx, ni, nj, nk};
    const float init = (float)(ni + nj + nk) * dx;  // :197
    const u64 init_key = ((u64)__builtin_bit_cast(uint32_t, init) << 32) | 0xffffffffull;

    hipEvent_t *ev = ws->ev;
    HIPCHK(hipEventRecord(ev[0], st));
    HIPCHK(zero_async(ws->err_flag, sizeof(int), st));
    HIPCHK(zero_async(ws->evals, sizeof(unsigned long long), st));
    if (ntri) {
        hipLaunchKernelGGL(k_prep_soup, dim3(grid_for(ntri, 256, 8192)), dim3(256), 0, st, d_tri, ntri, d_xyz, nvert,
                           ws->soup, ws->err_flag);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_init, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, ws->cell, ws->cnt, n, init_key);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev[1], st));
    if ((rc = band_enqueue(ws->band, st, ws->soup, ntri, g, band, init, ws->cell, ws->cnt, ws->evals, 0, nk, err)))
        return rc;
    HIPCHK(hipEventRecord(ev[2], st));

    // ---- sweeps ----
    int launches = 0;
    const int A = ni - 1, B = nj - 1, C = nk - 1;
    const bool do_sweep = (A > 0 && B > 0 && C > 0 && ntri > 0);
    int impl = 0;
    if (do_sweep && tile_sweep_supported(ni, nj, nk)) impl = 1;
    {
        const char *e = getenv("SDFGEN_SWEEP");  // diagnostics: "plane" forces the hyperplane launches
        if (e && strcmp(e, "plane") == 0) impl = 0;
        ws->wf.count = getenv("SDFGEN_COUNT_EVALS") != nullptr;
        const char *tr = getenv("SDFGEN_TRACE_SWEEP");   // diagnostics: per-task timing of one sweep
        ws->wf.trace_sweep = tr ? atoi(tr) : -1;
        ws->wf.trace_multi = getenv("SDFGEN_TRACE_MULTI") != nullptr;   // diagnostics: the whole first pass
        const char *gr = getenv("SDFGEN_TILE_GRID");     // diagnostics: cap on resident workgroups
        ws->wf.grid_override = gr ? atoi(gr) : 0;
        const char *ld = getenv("SDFGEN_TILE_LEAD");      // diagnostics: inter-wave lead
        ws->wf.lead_override = ld ? atoi(ld) : -1;
        if (ws->wf.count && ws->wf.stats) HIPCHK(hipMemsetAsync(ws->wf.stats, 0, ST_NSTATS * sizeof(u64), st));
    }
    const char *nsw_env = getenv("SDFGEN_DEBUG_NSWEEPS");   // diagnostics: stop after n sweeps
    const int nsweeps = nsw_env ? atoi(nsw_env) : 16;
    // Sweeps from `sparse_first` on run as Jacobi + repair (sweep_sparse.hpp): in the second
    // pass only ~0.05 % of the labels change.  SDFGEN_SPARSE_FROM overrides (16 = never).
    int sparse_first = 16;
    if (impl == 1 && sparse_sweep_supported(n, ni, nj, nk)) {
        const char *e = getenv("SDFGEN_SPARSE_FROM");
        sparse_first = e ? std::max(0, std::min(16, atoi(e))) : 8;
    }
    int sparse_sweeps = 0;
    {
        const char *e = getenv("SDFGEN_SPARSE_WORKERS");   // diagnostics: repair-kernel workgroups
        // repair workgroups: fewer on small grids (256^3: 64 beat 128 by 0.25 ms; 512^3: 128
        // beat 64 by 2.2 ms -- more concurrent chains there)
        ws->sp.workers = e ? atoi(e) : sp_workers_for((unsigned long long)ni * nj * nk);
        const char *b = getenv("SDFGEN_SPARSE_BRICK");    // 1 = the brick-owned repair (measured slower)
        ws->sp.brick = b && atoi(b) == 1;
        const char *ip = getenv("SDFGEN_SPARSE_INPLACE");  // diagnostics: 0 = two buffers, swapped per sweep
        ws->sp.inplace = !(ip && atoi(ip) == 0);
    }
    ws->wf.skip_seen = getenv("SDFGEN_NO_SEEN_SKIP") == nullptr;   // diagnostics
    ws->wf.clo = 0;
    ws->wf.chi = n;
    ws->wf.ntri = ntri;
    ws->sp.ntri = ntri;
    if (ws->wf.ctrl) HIPCHK(zero_async(ws->wf.ctrl + 1, 15 * sizeof(int), st));   // error bits / report of this call
    if (sparse_first < 16 && ws->sp.ctl) HIPCHK(zero_async(ws->sp.ctl, SP_NCTL * sizeof(u64), st));
    // The first pass's tile sweeps as ONE launch whose sweeps overlap (tile_sweep_multi) unless
    // SDFGEN_TILE_MULTI=0, tracing is on, or the per-sweep halo buffers (17 GB at 1024^3) would
    // take more than half of the free device memory; its time is then reported as sweep 0's
    // (the other first-pass entries are ~0).
    int multi_n = 0;
    if (impl == 1 && ws->wf.trace_sweep < 0) {
        const char *e = getenv("SDFGEN_TILE_MULTI");
        const int want = std::min(std::min(sparse_first, nsweeps), ST_MAXSW);
        const double bytes = 8.0 * want * (((nj - 1 + 7) / 8) * (double)(nk - 1) + ((nk - 1 + 7) / 8) * (double)(nj - 1)) *
                             (double)(ni - 1);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        const double have = (double)free_b + (double)ws->wf.cap_mhb * 8.0 + (double)ws->wf.cap_mhc * 8.0;
        if (!(e && atoi(e) == 0) && want > 1 && bytes <= 0.5 * have) multi_n = want;
    }
    // sweeps 1..multi_n-1 run inside sweep 0's launch: no event of their own (back-to-back event
    // records cost ~5 us of stream time each: a 37 us gap after the first pass in the kernel trace)
    // Likewise the second pass's sweeps after the first are timed together (in sweep sparse_first's
    // slot) unless SDFGEN_SWEEP_EVENTS asks for per-sweep times (diagnostics: ~6 us of stream time
    // per event between two kernels).
    static const bool per_sweep_events = getenv("SDFGEN_SWEEP_EVENTS") != nullptr;
    auto evrec = [&](int s) {
        return !(multi_n > 1 && s >= 1 && s < multi_n) && (per_sweep_events || s <= sparse_first || s >= nsweeps);
    };
    for (int s = 0; s < 16; ++s) {
        if (evrec(s)) HIPCHK(hipEventRecord(ev[3 + s], st));
        if (!do_sweep || s >= nsweeps) continue;
        const int di = SWEEP_DIRS[s % 8][0], dj = SWEEP_DIRS[s % 8][1], dk = SWEEP_DIRS[s % 8][2];
        if (impl == 1 && s >= sparse_first) {
            sdf_last_hip = hipSuccess;
            if ((rc = sparse_sweep(ws->sp, st, ws->soup, &ws->cell, &ws->cap_cell, origin, dx, ni, nj, nk, s)))
                return err.set(rc == -5 ? SDFGEN_HIP_ENOMEM : SDFGEN_HIP_ERUNTIME, "GPU sparse sweep setup failed: %s", sdf_last_hip_name());
            launches += 2;
            ++sparse_sweeps;
            continue;
        }
        if (impl == 1 && multi_n > 1 && s < multi_n) {   // the first pass as one overlapped launch
            if (s == 0) {
                if ((rc = tile_sweep_multi(ws->wf, st, ws->soup, ws->cell, origin, dx, ni, nj, nk, 0, multi_n,
                                           SWEEP_DIRS, err.buf, err.len)))
                    return rc;
                ++launches;
            }
            continue;
        }
        if (impl == 1) {
            ws->wf.cur_sweep = s;
            if ((rc = tile_sweep(ws->wf, st, ws->soup, ws->cell, origin, dx, ni, nj, nk, di, dj, dk, err.buf,
                                      err.len)))
                return rc;
            ++launches;
            continue;
        }
        for (int h = 0; h <= A + B + C - 3; ++h) {
            const int a_lo = std::max(0, h - (B - 1) - (C - 1)), a_hi = std::min(A - 1, h);
            const int b_lo = std::max(0, h - (A - 1) - (C - 1)), b_hi = std::min(B - 1, h);
            if (a_hi < a_lo || b_hi < b_lo) continue;
            const int a_cnt = a_hi - a_lo + 1, b_cnt = b_hi - b_lo + 1;
            const int nthr = a_cnt * b_cnt;
            hipLaunchKernelGGL(k_sweep_plane, dim3((nthr + 255) / 256), dim3(256), 0, st, ws->soup, ws->cell, g, di,
                               dj, dk, h, a_lo, b_lo, b_cnt, nthr);
            ++launches;
        }
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev[19], st));
    {
        const uint64_t rows = (uint64_t)nj * nk;
        if (layout == SDFGEN_LAYOUT_KFAST)
            hipLaunchKernelGGL(k_sign_kfast, dim3(grid_for((uint64_t)nj * ((nk + 63) / 64), 1, 65536)), dim3(256), 0, st,
                               ws->cell, ws->cnt, g, d_out, 0, nk);
        else
            hipLaunchKernelGGL(k_sign, dim3(grid_for(rows * 64, 256, 65536)), dim3(256), 0, st, ws->cell, ws->cnt, g,
                               layout, d_out, 0, nk);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev[20], st));
    // every status word of the call gathered on the device and read back in ONE copy (four small
    // copies cost ~70 us at the end of every call: kernel trace)
    unsigned long long stv[STATUS_N] = {};
    hipLaunchKernelGGL(k_status, dim3(1), dim3(256), 0, st, ws->status, ws->err_flag,
                       (impl == 1 && ws->wf.ctrl) ? ws->wf.ctrl + 1 : nullptr, ws->evals,
                       (impl == 1 && ws->wf.count) ? ws->wf.stats : nullptr, sparse_sweeps ? ws->sp.ctl : nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(stv, ws->status, sizeof(stv), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int flag = (int)stv[0], wf_err = (int)stv[1];
    const unsigned long long evals = stv[2], *wf_stats = stv + 3, *sp_ctl = stv + STATUS_SP;
    HIPCHK(hipGetLastError());
    if ((rc = check_oob(err, "make_level_set3"))) return rc;

    sdfgen_hip_profile p;
    memset(&p, 0, sizeof(p));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[20]));
    p.total_ms = ms;
    HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    p.prep_ms = ms;
    HIPCHK(hipEventElapsedTime(&ms, ev[1], ev[2]));
    p.band_ms = ms;
    HIPCHK(hipEventElapsedTime(&ms, ev[3], ev[19]));
    p.sweep_ms = ms;
    for (int s = 0; s < 16; ++s) {
        if (!evrec(s)) {
            p.sweep_launch_ms[s] = 0.f;   // inside sweep 0's launch
            continue;
        }
        int e = s + 1;   // the next recorded event
        while (e < 16 && !evrec(e)) ++e;
        HIPCHK(hipEventElapsedTime(&ms, ev[3 + s], ev[(e >= 16) ? 19 : 3 + e]));
        p.sweep_launch_ms[s] = ms;
    }
    HIPCHK(hipEventElapsedTime(&ms, ev[19], ev[20]));
    p.sign_ms = ms;
    p.sweep_launches = launches;
    p.sweep_impl = impl;
    p.band_evals = evals;
#ifdef ST_STEP_PROF
    if (ws->wf.count) {
        const double steps = (double)(wf_stats[8] + wf_stats[9] + wf_stats[10]);
        fprintf(stderr, "step profile: %.0f wave-steps (single no-eval %.3f, single eval %.3f, multi %.3f, pairs/multi %.1f); "
                        "cycles/step poll %.0f mask %.0f eval %.0f writeback %.0f\n", steps, wf_stats[8] / steps,
                wf_stats[9] / steps, wf_stats[10] / steps, wf_stats[10] ? (double)wf_stats[11] / wf_stats[10] : 0.0,
                wf_stats[4] / steps, wf_stats[5] / steps, wf_stats[6] / steps, wf_stats[7] / steps);
        fprintf(stderr, "step profile: eval cycles per step of the twin path %.0f (%.0f steps), of the compaction path %.0f "
                        "(%.0f steps)\n", wf_stats[12] / std::max(1.0, (double)wf_stats[9]), (double)wf_stats[9],
                wf_stats[13] / std::max(1.0, (double)wf_stats[10]), (double)wf_stats[10]);
        fprintf(stderr, "step profile: failed polls %.0f per wave-step: own data not landed %.3f, wave w-1 behind %.3f, "
                        "wave w+1 ring space %.3f, halo %.3f (a poll can fail on several)\n", wf_stats[1] / steps,
                wf_stats[3] / steps, wf_stats[14] / steps, (wf_stats[15] & 0xffffffffull) / steps, (wf_stats[15] >> 32) / steps);
        fprintf(stderr, "step profile: helper %.0f iterations that landed data, %.0f cycles each, %.2f own steps and %.2f halo "
                        "entries per iteration; %.0f idle polls\n", (double)wf_stats[16],
                wf_stats[17] / std::max(1.0, (double)wf_stats[16]), wf_stats[18] / std::max(1.0, (double)wf_stats[16]),
                wf_stats[19] / std::max(1.0, (double)wf_stats[16]), (double)wf_stats[2]);
    }
#endif
    p.sweep_evals = wf_stats[0];
    p.sweep_stalls = wf_stats[1];
    p.helper_polls = wf_stats[2];
    p.own_waits = wf_stats[3];
    p.sparse_sweeps = sparse_sweeps;
    p.tile_multi = multi_n;
    p.chain_steps = multi_n > 1 ? ws->wf.chain_steps : 0.0;
    p.tile_cfg = multi_n > 1 ? ws->wf.cfg : 0;
    p.slabs = 1;
    p.sparse_first = sparse_sweeps ? sparse_first : 16;
#ifdef SP_JACOBI_COUNT
    fprintf(stderr, "jacobi candidates %llu lane-passes %llu (slot use %.3f)\n", sp_ctl[SP_DIAG], sp_ctl[SP_DIAG + 1],
            sp_ctl[SP_DIAG + 1] ? sp_ctl[SP_DIAG] / (2.0 * sp_ctl[SP_DIAG + 1]) : 0.0);
#endif
#ifdef SP_ITER_PROF
    {
        const double nb = std::max(1.0, (double)sp_ctl[SP_DIAGX + 24]), ni = std::max(1.0, (double)sp_ctl[SP_DIAGX + 25]);
        fprintf(stderr, "repair iterations: busy %.0f idle %.0f; cycles per busy iteration:", nb, ni);
        for (int q = 0; q < 12; ++q) fprintf(stderr, " %.0f", sp_ctl[SP_DIAGX + q] / nb);
        fprintf(stderr, "; per idle iteration:");
        for (int q = 0; q < 12; ++q) fprintf(stderr, " %.0f", sp_ctl[SP_DIAGX + 12 + q] / ni);
        fprintf(stderr, "  (ticket, tail, append wait, poll, evaluate, store, atomics, hand-off rest, append issue, "
                        "hand-off (ballots+writes), copy+exit+sleep, join after the busy block)\n");
    }
#endif
    p.sparse_rechecks = sp_ctl[SP_RUNS];
    p.sparse_claims = sp_ctl[SP_ENQ];
    if (sparse_sweeps) p.sweep_impl = 2;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof = p;
    }
    if (wf_err) {
        st_watchdog_report(ws->wf, "make_level_set3");
        return err.set(SDFGEN_HIP_ERUNTIME, "GPU sweep watchdog fired (lost tile hand-off, code %d)", wf_err);
    }
    if (sp_ctl[SP_ERR] & 4ull) return err.set(SDFGEN_HIP_ERUNTIME, "GPU sparse sweep: Jacobi list overflow");
    if (sp_ctl[SP_ERR]) return err.set(SDFGEN_HIP_ERUNTIME, "GPU sparse sweep watchdog fired (work list stalled)");
    if (flag) return err.set(SDFGEN_HIP_EINDEX, "triangle vertex index out of range (>= %llu vertices)",
                             (unsigned long long)nvert);
    return 0;
}

int device_count_impl()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}


// ---------------------------------------------------------------------------
// Z-slab sessions: one slab of k planes per GPU (one process per GPU, or several
// slabs in one process).  DESIGN.md §7.
//   * band, ray parity, sign: local to the slab (boxes clamped to the whole grid first);
//   * first pass (sweeps 1-8): the tile wavefront over this slab's oriented c range, all eight
//     sweeps in ONE overlapped launch scheduled for the whole grid (tile_sweep_multi); the plane
//     just upstream arrives as tagged granules in a per-sweep inbox written by the upstream GPU
//     (xGMI, IPC- or peer-mapped), and this slab's last plane is written into the downstream
//     GPU's inbox -- the wavefront pipelines straight across GPUs;
//   * second pass (sweeps 9-16): Jacobi + change-driven repair per slab (sweep_sparse.hpp); the
//     neighbour planes are kept in halo planes, changes of a boundary plane are pushed to the
//     neighbour (with a recheck request for the downstream one), and a neighbour handshake
//     (DONE / READY flags) separates the sweeps.
// Everything a neighbour writes lives in ONE uncached block per slab (`comm`), exported once.
// ---------------------------------------------------------------------------
struct CommLayout {
    size_t plane = 0;            // cells per plane (ni * nj)
    size_t ring_cap = 0;         // inbound ring entries per side
    size_t off_halo = 0, off_ring = 0, off_flags = 0, bytes = 0;
    void init(size_t plane_cells)
    {
        plane = plane_cells;
        ring_cap = 4 * plane + 4096;   // boundary relabels per sweep (error bit 8 beyond)
        off_halo = 8 * plane * sizeof(u64);                        // 8 per-sweep tile inboxes
        off_ring = off_halo + 4 * plane * sizeof(uint32_t);        // halo planes [side][parity]
        off_flags = (off_ring + 2 * ring_cap * sizeof(uint32_t) + 127) / 128 * 128;
        const size_t raw = off_flags + SP_FL_WORDS * SP_FL_STRIDE * sizeof(u64);
        bytes = (raw + (2u << 20) - 1) / (2u << 20) * (2u << 20);  // whole 2 MiB: a dedicated allocation
    }
    u64 *inbox(char *base, int sweep) const { return (u64 *)base + plane * (size_t)(sweep % 8); }
    uint32_t *halo(char *base, int side, int par) const { return (uint32_t *)(base + off_halo) + plane * (size_t)(2 * side + par); }
    uint32_t *ring(char *base, int side) const { return (uint32_t *)(base + off_ring) + ring_cap * (size_t)side; }
    u64 *flags(char *base) const { return (u64 *)(base + off_flags); }
};

struct SlabSession {
    int device = -1, nslabs = 1, slab = 0, ni = 0, nj = 0, nk = 0, k_begin = 0, k_end = 0;
    hipStream_t stream = nullptr;
    // Cell state of this slab's planes only (k in [k_begin, k_end)): cell_mem holds them, and
    // cell = cell_mem - k_begin * ni * nj so the kernels index it with global cell numbers
    // (every kernel of a slab touches only its own planes; the neighbour planes arrive through
    // the inboxes and halo planes).  Same for cnt and the sparse pass's second buffer alt.
    u64 *cell = nullptr, *cell_mem = nullptr, *alt = nullptr, *alt_mem = nullptr;
    uint32_t *cnt = nullptr, *cnt_mem = nullptr;
    float4 *soup = nullptr;
    uint32_t *tri = nullptr;
    float *xyz = nullptr, *out = nullptr;
    int *err_flag = nullptr;
    unsigned *arrive = nullptr;
    unsigned long long *evals = nullptr;
    unsigned long long *tm = nullptr;     // phase timers (geom.hpp TM_*), zeroed per call
    size_t cap_soup = 0, cap_tri = 0, cap_xyz = 0, cap_out = 0;
    TileSweepWorkspace wf;
    SparseSweepWorkspace sp;
    BandWork band;
    CommLayout cl;
    char *comm = nullptr;          // uncached, IPC-exported: inboxes, halo planes, inbound rings, flags
    char *peer[2] = {nullptr, nullptr};   // the lower / upper neighbour's comm (mapped, comm_import)
    unsigned long long sync_epoch = 0;    // neighbour handshakes issued (same count on every slab)
    uint64_t prepared_ntri = ~0ull;       // slab_prepare was run for this many triangles
    int sparse_sweeps = 0, tile_multi = 0;
    hipEvent_t ev[24] = {};
    int launches = 0;
    int peer_dev[2] = {-1, -1};           // the neighbours' devices (-1: none, or not known for an IPC mapping)
    std::mutex mu;
};

// "slab s (device d, PCI p; lower slab s-1 on device dl PCI pl; upper ...)": the rank pair a failed
// hand-off involves, named in slab_finish's errors so that a watchdog on a multi-GPU node is diagnosable
void slab_where(const SlabSession *S, char *buf, size_t len)
{
    auto pci = [](int dev, char *b, size_t n) {
        if (dev < 0 || hipDeviceGetPCIBusId(b, (int)n, dev) != hipSuccess) snprintf(b, n, "?");
    };
    char own[32], lo[32], up[32];
    pci(S->device, own, sizeof(own));
    pci(S->peer_dev[0], lo, sizeof(lo));
    pci(S->peer_dev[1], up, sizeof(up));
    int n = snprintf(buf, len, "slab %d of %d (device %d, PCI %s", S->slab, S->nslabs, S->device, own);
    if (S->slab > 0 && n > 0 && (size_t)n < len)
        n += snprintf(buf + n, len - n, "; lower slab %d on device %d, PCI %s", S->slab - 1, S->peer_dev[0], lo);
    if (S->slab < S->nslabs - 1 && n > 0 && (size_t)n < len)
        n += snprintf(buf + n, len - n, "; upper slab %d on device %d, PCI %s", S->slab + 1, S->peer_dev[1], up);
    if (n > 0 && (size_t)n < len) snprintf(buf + n, len - n, ")");
}

// Uncached blocks are never returned to the runtime while the process runs.  After hipFree of
// an uncached (MTYPE UC) block, a later plain hipMalloc that is handed the same virtual range has
// been seen to lose stores and read zeros on the GPU: the first one-GPU call after an in-process
// two-slab call placed its halo buffer exactly on a freed comm block and failed (digest mismatch
// or a tile hand-off never arriving, 3 of 3 runs), and never failed when the block was kept
// ("freed uncached memory").  So freed sessions hand their block back to this
// per-process pool, the next session on the device takes the smallest free block that fits, and
// the pool (a few 2 MiB blocks per grid plane size) lives until the process exits.  The IPC
// handle of a block is exported once; peers map each handle once (comm_import) and keep it, for
// the same reason on the importing side.
struct CommBlock {
    int device;
    char *p;
    size_t bytes;
    bool busy;
    bool exported;
    hipIpcMemHandle_t handle;
};
std::mutex g_comm_mu;
std::vector<CommBlock> g_comm;

int comm_acquire(int device, size_t bytes, char **out, Err &err)
{
    // power-of-two size classes from 2 MiB: the pool never shrinks, so its growth is bounded by the
    // concurrently live sessions per class -- a caller cycling through many plane sizes reuses blocks
    // instead of adding one per size
    size_t cls = (size_t)2 << 20;
    while (cls < bytes) cls <<= 1;
    bytes = cls;
    std::lock_guard<std::mutex> lk(g_comm_mu);
    CommBlock *best = nullptr;
    for (CommBlock &b : g_comm)
        if (!b.busy && b.device == device && b.bytes >= bytes && (!best || b.bytes < best->bytes)) best = &b;
    if (!best) {
        CommBlock b{};
        b.device = device;
        b.bytes = bytes;
        HIPCHK(hipExtMallocWithFlags((void **)&b.p, bytes, hipDeviceMallocUncached));
        g_comm.push_back(b);
        best = &g_comm.back();
    }
    best->busy = true;
    *out = best->p;
    return 0;
}

void comm_return(char *p)
{
    std::lock_guard<std::mutex> lk(g_comm_mu);
    for (CommBlock &b : g_comm)
        if (b.p == p) b.busy = false;
}

int comm_export(char *p, hipIpcMemHandle_t *h, Err &err)
{
    std::lock_guard<std::mutex> lk(g_comm_mu);
    for (CommBlock &b : g_comm)
        if (b.p == p) {
            if (!b.exported) {
                HIPCHK(hipIpcGetMemHandle(&b.handle, p));
                b.exported = true;
            }
            *h = b.handle;
            return 0;
        }
    return err.set(SDFGEN_HIP_ERUNTIME, "slab communication block not found");
}

// Imported neighbour blocks stay mapped for the life of the process, like the pool: closing a mapping
// would hand its virtual range back to this process's allocator, the situation the pool avoids.  Growth
// bound: one mapping per distinct exported block a peer ever showed us (a peer's pool reuses blocks, so
// long-lived peer processes add none after their first sessions).  Keyed by the handle bytes: a handle
// is only ever reused by the exporting process for the same block (hipIpcGetMemHandle of a live
// allocation), and a peer that exited and a new one whose handle bytes collide would map a stale block --
// callers that replace peer processes call sdfgen_hip_slab_close_imports in the survivors between jobs
// (opt-in: with no slab session alive it closes every imported mapping, comm_close_imports).
struct CommImport {
    int device;
    hipIpcMemHandle_t handle;
    void *p;
};
std::vector<CommImport> g_comm_imports;
int g_live_slabs = 0;   // slab sessions alive in this process (under g_comm_mu)
std::vector<int> g_dev_slabs;   // ... per device (under g_comm_mu)

// Slab sessions sharing `device`: this process's live ones, or SDFGEN_SLABS_PER_DEVICE when the caller
// knows of more (ranks of other processes on the same GPU -- a one-GPU rehearsal of a multi-GPU run).
int slab_share(int device)
{
    int n = 1;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        if (device >= 0 && (size_t)device < g_dev_slabs.size()) n = std::max(n, g_dev_slabs[device]);
    }
    if (const char *e = getenv("SDFGEN_SLABS_PER_DEVICE")) n = std::max(n, atoi(e));
    return n;
}

// Hardware queues the HIP runtime gives this process per device (its GPU_MAX_HW_QUEUES, default 4).
// Slab sessions of one device whose streams share a hardware queue run their kernels one after the
// other -- and a slab's kernels wait on its neighbours' -- so more sessions than queues cannot work.
int hw_queues()
{
    const char *e = getenv("GPU_MAX_HW_QUEUES");
    const int q = e ? atoi(e) : 4;
    return q > 0 ? q : 4;
}

// Close every imported neighbour mapping once no slab session of this process is alive.  Returns the
// number closed (0 while a session is alive).
int comm_close_imports()
{
    std::lock_guard<std::mutex> lk(g_comm_mu);
    if (g_live_slabs > 0) return 0;
    int n = 0;
    for (const CommImport &m : g_comm_imports) {
        (void)hipSetDevice(m.device);
        if (hipIpcCloseMemHandle(m.p) == hipSuccess) ++n;
    }
    (void)hipGetLastError();
    g_comm_imports.clear();
    return n;
}

int comm_import(int device, const hipIpcMemHandle_t &h, void **out, Err &err)
{
    std::lock_guard<std::mutex> lk(g_comm_mu);
    for (const CommImport &m : g_comm_imports)
        if (m.device == device && memcmp(&m.handle, &h, sizeof(h)) == 0) {
            *out = m.p;
            return 0;
        }
    void *p = nullptr;
    HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    g_comm_imports.push_back(CommImport{device, h, p});
    *out = p;
    return 0;
}

// Resolve every kernel a slab launches before any of its work is enqueued.  A kernel's first
// launch makes the HIP runtime load it (deferred code-object loading); doing that while this
// process's other slabs already run kernels that wait on work not yet enqueued has been seen to
// block the enqueuing thread -- the in-process multi-slab path deadlocked until a watchdog fired
// (DESIGN.md §7).  hipFuncGetAttributes loads the kernel without launching it.
int slab_preload_kernels(Err &err)
{
    if (getenv("SDFGEN_NO_KERNEL_PRELOAD")) return 0;   // diagnostics
    const void *k[] = {(const void *)k_prep_soup, (const void *)k_init, (const void *)k_band_lds,
                       (const void *)k_band_big_scan, (const void *)k_band_big,
                       (const void *)k_sign, (const void *)k_sign_kfast, (const void *)k_sweep_tile<StCfgLat, true, false, false>,
                       (const void *)k_sweep_tile<StCfgLat, true, false, true>,
                       (const void *)k_sweep_tile<StCfgThr, true, false, false>,
                       (const void *)k_sweep_tile<StCfgThr, true, false, true>,
                       (const void *)k_sweep_tile<StCfgQuad, true, false, false>,
                       (const void *)k_sweep_tile<StCfgQuad, true, false, true>,
                       (const void *)k_sweep_tile<StCfgDuo, true, false, false>,
                       (const void *)k_sweep_tile<StCfgDuo, true, false, true>,
                       (const void *)k_sweep_tile<StCfgOct, true, false, false>,
                       (const void *)k_sweep_tile<StCfgOct, true, false, true>,
                       (const void *)k_sweep_tile<StCfgQfp, true, false, true>, (const void *)k_sp_jacobi<true>,
                       (const void *)k_sp_jlist<true>, (const void *)k_sp_recheck<true>, (const void *)k_sp_slab_wait,
                       (const void *)k_sp_slab_halo, (const void *)k_sp_slab_export};
    for (const void *f : k) {
        hipFuncAttributes a;
        HIPCHK(hipFuncGetAttributes(&a, f));
    }
    return 0;
}

int slab_alloc(SlabSession *S, Err &err)
{
    HIPCHK(hipSetDevice(S->device));
    if (int rc = slab_preload_kernels(err)) return rc;
    HIPCHK(hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking));
    for (auto &e : S->ev) HIPCHK(hipEventCreate(&e));
    const size_t plane = (size_t)S->ni * S->nj;
    const uint64_t n = plane * (uint64_t)(S->k_end - S->k_begin);   // this slab's planes only
    HIPCHK(hipMalloc((void **)&S->cell_mem, n * sizeof(u64)));
    HIPCHK(hipMalloc((void **)&S->cnt_mem, n * sizeof(uint32_t)));
    S->cell = S->cell_mem - plane * (size_t)S->k_begin;
    S->cnt = S->cnt_mem - plane * (size_t)S->k_begin;
    HIPCHK(hipMalloc((void **)&S->err_flag, sizeof(int)));
    HIPCHK(hipMalloc((void **)&S->evals, sizeof(unsigned long long)));
    HIPCHK(hipMalloc((void **)&S->arrive, sizeof(unsigned)));
    HIPCHK(hipMalloc((void **)&S->tm, TM_N * sizeof(unsigned long long)));
    // The communication block is written by the NEIGHBOUR GPUs (system-scope stores over xGMI,
    // through an IPC or peer mapping) while this GPU's kernels poll it.  Plain hipMalloc memory
    // is coarse-grained: HIP makes remote writes to it visible only at kernel boundaries (an L2
    // of this GPU may keep serving a stale line).  Uncached device memory (MTYPE UC) is held in
    // no cache, so every system-scope load of a poll reads what the remote system-scope store
    // wrote, mid-kernel.  Whole 2 MiB: a dedicated allocation that IPC maps as is.
    S->cl.init(plane);
    if (int rc = comm_acquire(S->device, S->cl.bytes, &S->comm, err)) return rc;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        ++g_live_slabs;
        if ((size_t)S->device >= g_dev_slabs.size()) g_dev_slabs.resize(S->device + 1, 0);
        ++g_dev_slabs[S->device];
    }
    HIPCHK(hipMemset(S->comm, 0, S->cl.bytes));   // epoch 0 is never published, flags start at 0
    HIPCHK(hipDeviceSynchronize());
    return 0;
}

void slab_free(SlabSession *S)
{
    if (S->device < 0) return;
    (void)hipSetDevice(S->device);
    if (S->stream) (void)hipStreamSynchronize(S->stream);
    // the neighbours' blocks stay mapped (comm_import) and this slab's block goes back to the pool
    if (S->comm) {
        comm_return(S->comm);
        std::lock_guard<std::mutex> lk(g_comm_mu);
        --g_live_slabs;
        if ((size_t)S->device < g_dev_slabs.size()) --g_dev_slabs[S->device];
    }
    S->comm = nullptr;
    (void)hipFree(S->cell_mem);
    (void)hipFree(S->alt_mem);
    (void)hipFree(S->cnt_mem);
    (void)hipFree(S->soup);
    (void)hipFree(S->tri);
    (void)hipFree(S->xyz);
    (void)hipFree(S->out);
    (void)hipFree(S->err_flag);
    (void)hipFree(S->evals);
    (void)hipFree(S->arrive);
    (void)hipFree(S->tm);
    tile_sweep_release(S->wf);
    sparse_sweep_release(S->sp);
    band_release(S->band);
    for (auto &e : S->ev)
        if (e) (void)hipEventDestroy(e);
    if (S->stream) (void)hipStreamDestroy(S->stream);
}

// Oriented c range of this slab for a sweep with k direction dk (see sweep_tile.hpp).
void slab_c_range(const SlabSession *S, int dk, int *cs, int *ce) { st_slab_c_range(S->k_begin, S->k_end, S->nk, dk, cs, ce); }

// Upstream / downstream neighbour side of a sweep: 0 = lower slab, 1 = upper slab (-1: none).
int slab_up_side(const SlabSession *S, int dk)
{
    const int side = dk > 0 ? 0 : 1;
    return (side == 0 ? S->slab > 0 : S->slab < S->nslabs - 1) ? side : -1;
}
int slab_down_side(const SlabSession *S, int dk)
{
    const int side = dk > 0 ? 1 : 0;
    return (side == 0 ? S->slab > 0 : S->slab < S->nslabs - 1) ? side : -1;
}

// Enqueue the whole pipeline for this slab on S->stream (inputs/outputs on S->device).
// Decisions every slab of the grid takes identically (dims and environment only): the
// neighbours must agree on who writes which inbox / flag in which order.
bool slab_multi_on() { return getenv("SDFGEN_TILE_MULTI") == nullptr || atoi(getenv("SDFGEN_TILE_MULTI")) != 0; }
bool slab_sparse_on(const SlabSession *S)
{
    return sparse_sweep_supported((uint64_t)S->ni * S->nj * S->nk, S->ni, S->nj, S->nk) &&
           (getenv("SDFGEN_SLAB_SPARSE") == nullptr || atoi(getenv("SDFGEN_SLAB_SPARSE")) != 0);
}

// Whole grid's slab boundaries and this slab's per-sweep inboxes for the first-pass launch.
void slab_plan(const SlabSession *S, StSlabPlan &plan, TileSlab io[8])
{
    plan.nslabs = S->nslabs;
    plan.slab = S->slab;
    plan.kb.resize(S->nslabs + 1);
    for (int r = 0; r <= S->nslabs; ++r) plan.kb[r] = (int)((long long)r * S->nk / S->nslabs);
    for (int q = 0; q < 8; ++q) {
        TileSlab &sl = io[q];
        const int dk = SWEEP_DIRS[q][2];
        const int up = slab_up_side(S, dk), down = slab_down_side(S, dk);
        sl.on = true;
        slab_c_range(S, dk, &sl.cs, &sl.ce);
        sl.in = up >= 0 ? S->cl.inbox(S->comm, q) : nullptr;
        sl.out = down >= 0 ? S->cl.inbox(S->peer[down], q) : nullptr;
        plan.in[q] = sl.in;
        plan.out[q] = sl.out;
    }
}

// Every allocation, table upload and stream synchronisation of a call (ntri triangles).  A thread
// that drives several slabs prepares all of them before it enqueues any: a host-side wait after
// one slab's kernels are running (they wait on neighbours) would wait for work this thread has
// not enqueued yet -- measured as a deadlock broken only by the watchdogs.
int slab_prepare(SlabSession *S, uint64_t ntri, Err &err)
{
    const int ni = S->ni, nj = S->nj, nk = S->nk;
    const uint64_t plane_cells = (uint64_t)ni * nj;
    const int kc = S->k_end - S->k_begin;
    hipStream_t st = S->stream;
    HIPCHK(hipSetDevice(S->device));
    if (!S->soup || S->cap_soup < 3 * std::max<uint64_t>(ntri, 1)) {
        if (S->soup) HIPCHK(hipFree(S->soup));
        S->soup = nullptr;
        S->cap_soup = 0;
        HIPCHK(hipMalloc((void **)&S->soup, 3 * std::max<uint64_t>(ntri, 1) * sizeof(float4)));
        S->cap_soup = 3 * std::max<uint64_t>(ntri, 1);
    }
    if (int rc = band_reserve(S->band, ntri, err)) return rc;
    int ti = -1;
    for (int dk = -1; dk <= 1; dk += 2) {
        int cs, ce;
        slab_c_range(S, dk, &cs, &ce);
        if (ni >= 2 && nj >= 2 && ce > cs)
            if (int rc = st_prepare(S->wf, st, ni, nj, cs, ce, &ti))
                return err.set(rc == -5 ? SDFGEN_HIP_ENOMEM : SDFGEN_HIP_ERUNTIME, "GPU slab buffers: %s", sdf_last_hip_name());
    }
    if (ni >= 2 && nj >= 2 && nk >= 2 && slab_multi_on()) {
        StSlabPlan plan;
        TileSlab io[8];
        slab_plan(S, plan, io);
        const float o0[3] = {0.f, 0.f, 0.f};
        if (int rc = tile_sweep_multi(S->wf, st, nullptr, nullptr, o0, 1.f, ni, nj, nk, 0, 8, SWEEP_DIRS, err.buf,
                                      err.len, &plan, true))
            return rc;
    }
    if (slab_sparse_on(S)) {
        if (int rc = sp_reserve(S->sp, plane_cells * kc, st))
            return err.set(rc == -5 ? SDFGEN_HIP_ENOMEM : SDFGEN_HIP_ERUNTIME, "GPU slab sparse buffers: %s", sdf_last_hip_name());
        if (!S->alt_mem) {
            HIPCHK(hipMalloc((void **)&S->alt_mem, plane_cells * kc * sizeof(u64)));
            S->alt = S->alt_mem - plane_cells * (size_t)S->k_begin;
        }
    }
    HIPCHK(hipStreamSynchronize(st));
    S->prepared_ntri = ntri;
    return 0;
}

int slab_enqueue(SlabSession *S, const uint32_t *d_tri, uint64_t ntri, const float *d_xyz, uint64_t nvert,
                 const float origin[3], float dx, int band, int layout, float *d_out, Err &err)
{
    const int ni = S->ni, nj = S->nj, nk = S->nk;
    const uint64_t plane_cells = (uint64_t)ni * nj;
    const int kc = S->k_end - S->k_begin;
    const bool tdbg = getenv("SDFGEN_DEBUG_TIMING") != nullptr;   // diagnostics: host time per phase
    const auto t_start = std::chrono::steady_clock::now();
    auto tmark = [&](const char *what) {
        if (tdbg)
            fprintf(stderr, "slab %d enqueue %-12s %.3f ms\n", S->slab, what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    };
    if (S->prepared_ntri != ntri || !S->soup)
        if (int rc = slab_prepare(S, ntri, err)) return rc;
    tmark("prepare");
    hipStream_t st = S->stream;
    const bool do_sweep = ni >= 2 && nj >= 2 && nk >= 2 && ntri > 0;
    const bool multi = slab_multi_on(), sparse = slab_sparse_on(S);
    StSlabPlan plan;
    TileSlab io[8];
    slab_plan(S, plan, io);
    auto tile_io = [&](int s, TileSlab &sl) { sl = io[s % 8]; };
    Grid g{origin[0], origin[1], origin[2], dx, ni, nj, nk};
    const float init = (float)(ni + nj + nk) * dx;
    const u64 init_key = ((u64)__builtin_bit_cast(uint32_t, init) << 32) | 0xffffffffull;
    hipEvent_t *ev = S->ev;
    HIPCHK(hipEventRecord(ev[0], st));
    HIPCHK(zero_async(S->err_flag, sizeof(int), st));
    HIPCHK(zero_async(S->evals, sizeof(unsigned long long), st));
    HIPCHK(zero_async(S->tm, TM_N * sizeof(unsigned long long), st));
    S->wf.tm = S->tm;
    if (S->wf.ctrl) HIPCHK(zero_async(S->wf.ctrl + 1, 15 * sizeof(int), st));
    if (S->sp.ctl) HIPCHK(zero_async(S->sp.ctl, SP_NCTL * sizeof(u64), st));
    if (ntri) {
        hipLaunchKernelGGL(k_prep_soup, dim3(grid_for(ntri, 256, 8192)), dim3(256), 0, st, d_tri, ntri, d_xyz, nvert,
                           S->soup, S->err_flag);
        HIPCHK(hipGetLastError());
    }
    const uint64_t nslab = plane_cells * kc;
    hipLaunchKernelGGL(k_init, dim3(grid_for(nslab, 256, 8192)), dim3(256), 0, st, S->cell + plane_cells * S->k_begin,
                       S->cnt + plane_cells * S->k_begin, nslab, init_key);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev[1], st));
    if (int rc = band_enqueue(S->band, st, S->soup, ntri, g, band, init, S->cell, S->cnt, S->evals, S->k_begin, S->k_end,
                              err))
        return rc;
    HIPCHK(hipEventRecord(ev[2], st));
    tmark("band");
    S->launches = 0;
    S->sparse_sweeps = 0;
    S->tile_multi = 0;
    {
        // Co-resident slabs on one GPU: each slab's persistent grids are capped by the library (sweep_tile.hpp
        // st_share_grid, sp_share_workers) from the occupancy query and the slab sessions sharing the device,
        // so that every slab keeps workgroups resident while its neighbours wait on it; SDFGEN_TILE_GRID
        // overrides (diagnostics)
        const char *gr = getenv("SDFGEN_TILE_GRID");
        S->wf.grid_override = gr ? atoi(gr) : 0;
        S->wf.share = slab_share(S->device);
    }
    S->wf.clo = plane_cells * (uint64_t)S->k_begin;
    S->wf.chi = plane_cells * (uint64_t)S->k_end;
    S->wf.ntri = ntri;
    S->sp.ntri = ntri;
    u64 *cur = S->cell;   // the state buffer holding the result so far
    for (int s = 0; s < 8 && do_sweep; ++s) {   // first pass
        HIPCHK(hipEventRecord(ev[3 + s], st));
        if (multi) {
            if (s == 0) {
                if (int rc = tile_sweep_multi(S->wf, st, S->soup, cur, origin, dx, ni, nj, nk, 0, 8, SWEEP_DIRS,
                                              err.buf, err.len, &plan))
                    return rc;
                ++S->launches;
                S->tile_multi = 8;
            }
            continue;
        }
        const int di = SWEEP_DIRS[s][0], dj = SWEEP_DIRS[s][1], dk = SWEEP_DIRS[s][2];
        TileSlab sl;
        tile_io(s, sl);
        S->wf.cur_sweep = s;
        if (int rc = tile_sweep(S->wf, st, S->soup, cur, origin, dx, ni, nj, nk, di, dj, dk, err.buf, err.len, sl))
            return rc;
        ++S->launches;
    }
    tmark("first pass");
    const char *nsw_env = getenv("SDFGEN_DEBUG_NSWEEPS");   // diagnostics: stop after the first pass
    if (nsw_env && atoi(nsw_env) <= 8) {
        for (int s = 8; s < 16; ++s) HIPCHK(hipEventRecord(ev[3 + s], st));
    } else if (do_sweep && sparse) {
        // second pass as Jacobi + repair per slab, in place (alt keeps the changed cells' pre-sweep
        // values) unless SDFGEN_SPARSE_INPLACE=0: then the state alternates between cell and alt
        {
            const char *e = getenv("SDFGEN_SPARSE_WORKERS");   // diagnostics
            S->sp.workers = e ? atoi(e) : sp_workers_for((unsigned long long)ni * nj * (S->k_end - S->k_begin));
            // a slab's repair kernel ends only after its upstream neighbour's: with several slabs on one GPU
            // every one of them must stay resident (8 x 256 one-wave workgroups at 171 VGPRs are the chip's
            // 2,048 slots for them -- the repair watchdogs fired without a cap)
            if (!e) S->sp.workers = std::min(S->sp.workers, sp_share_workers(slab_share(S->device)));
            const char *ip = getenv("SDFGEN_SPARSE_INPLACE");
            S->sp.inplace = !(ip && atoi(ip) == 0);
        }
        // our boundary planes into the neighbours' parity-0 halo planes, then DONE
        SpExportParams E;
        memset(&E, 0, sizeof(E));
        E.cell = cur;
        E.plane = plane_cells;
        E.c_first = plane_cells * (u64)S->k_begin;
        E.c_last = plane_cells * (u64)(S->k_end - 1);
        for (int side = 0; side < 2; ++side) {
            const bool has = side == 0 ? S->slab > 0 : S->slab < S->nslabs - 1;
            if (!has) continue;
            E.nb_hS[side] = S->cl.halo(S->peer[side], 1 - side, 0);
            E.nb_flags[side] = S->cl.flags(S->peer[side]);
        }
        E.epoch = ++S->sync_epoch;
        E.arrive = S->arrive;
        HIPCHK(hipMemsetAsync(S->arrive, 0, sizeof(unsigned), st));
        if (!getenv("SDFGEN_DEBUG_NO_EXPORT"))   // diagnostics
            hipLaunchKernelGGL(k_sp_slab_export, dim3(grid_for(plane_cells, 256, 256)), dim3(256), 0, st, E);
        HIPCHK(hipGetLastError());
        u64 *other = S->alt;
        const char *stg_env = getenv("SDFGEN_DEBUG_SPARSE_STAGE");
        int n_sparse = nsw_env ? std::max(0, std::min(8, atoi(nsw_env) - 8)) : 8;   // diagnostics
        if (stg_env && atoi(stg_env) == 0) n_sparse = 0;                             // diagnostics: export only
        for (int m = 0; m < n_sparse; ++m) {
            const int s = 8 + m;
            HIPCHK(hipEventRecord(ev[3 + s], st));
            SpSlabSweep L;
            memset(&L, 0, sizeof(L));
            L.S = cur;
            L.X = S->sp.inplace ? cur : other;   // in place: `other` keeps the changed cells' pre-sweep values
            L.sv = S->sp.inplace ? other : nullptr;
            L.k_lo = S->k_begin;
            L.k_hi = S->k_end;
            for (int side = 0; side < 2; ++side) {
                L.hS[side] = S->cl.halo(S->comm, side, m & 1);
                L.hX[side] = S->cl.halo(S->comm, side, (m + 1) & 1);
                L.in_ring[side] = S->cl.ring(S->comm, side);
                const bool has = side == 0 ? S->slab > 0 : S->slab < S->nslabs - 1;
                if (!has) continue;
                L.nb_hX[side] = S->cl.halo(S->peer[side], 1 - side, (m + 1) & 1);
                L.nb_ring[side] = S->cl.ring(S->peer[side], 1 - side);
                L.nb_flags[side] = S->cl.flags(S->peer[side]);
            }
            L.ring_cap = S->cl.ring_cap;
            L.flags = S->cl.flags(S->comm);
            L.prev_epoch = S->sync_epoch;
            L.epoch = ++S->sync_epoch;
            L.arrive = S->arrive;
            L.tm = S->tm;
            L.tm_m = m;
            if (int rc = sparse_sweep_slab(S->sp, st, S->soup, L, origin, dx, ni, nj, nk, s))
                return err.set(rc == -5 ? SDFGEN_HIP_ENOMEM : SDFGEN_HIP_ERUNTIME, "GPU slab sparse sweep setup failed: %s", sdf_last_hip_name());
            S->launches += 3;
            ++S->sparse_sweeps;
            if (!S->sp.inplace) std::swap(cur, other);
        }
        for (int m = n_sparse; m < 8; ++m) HIPCHK(hipEventRecord(ev[11 + m], st));
    } else {
        for (int s = 8; s < 16 && do_sweep; ++s) {
            HIPCHK(hipEventRecord(ev[3 + s], st));
            const int di = SWEEP_DIRS[s % 8][0], dj = SWEEP_DIRS[s % 8][1], dk = SWEEP_DIRS[s % 8][2];
            TileSlab sl;
            tile_io(s, sl);
            S->wf.cur_sweep = s;
            if (int rc = tile_sweep(S->wf, st, S->soup, cur, origin, dx, ni, nj, nk, di, dj, dk, err.buf, err.len, sl))
                return rc;
            ++S->launches;
        }
    }
    tmark("sweeps");
    for (int s = 0; s < 16; ++s)   // sweeps not run (tiny grids) still need their events recorded
        if (!do_sweep) HIPCHK(hipEventRecord(ev[3 + s], st));
    HIPCHK(hipEventRecord(ev[19], st));
    {
        const uint64_t rows = (uint64_t)nj * kc;
        if (layout == SDFGEN_LAYOUT_KFAST)
            hipLaunchKernelGGL(k_sign_kfast, dim3(grid_for((uint64_t)nj * ((kc + 63) / 64), 1, 65536)), dim3(256), 0, st,
                               cur, S->cnt, g, d_out, S->k_begin, kc);
        else
            hipLaunchKernelGGL(k_sign, dim3(grid_for(rows * 64, 256, 65536)), dim3(256), 0, st, cur, S->cnt, g,
                               layout, d_out, S->k_begin, kc);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev[20], st));
    return 0;
}

int slab_finish(SlabSession *S, uint64_t nvert, sdfgen_hip_profile *prof, Err &err)
{
    hipStream_t st = S->stream;
    int flag = 0, wf_err[2] = {0, 0};
    unsigned long long evals = 0, sp_ctl[4] = {0, 0, 0, 0}, tm[TM_N];
    HIPCHK(hipMemcpyAsync(&flag, S->err_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(tm, S->tm, sizeof(tm), hipMemcpyDeviceToHost, st));
    if (S->wf.ctrl) HIPCHK(hipMemcpyAsync(wf_err, S->wf.ctrl + 1, sizeof(wf_err), hipMemcpyDeviceToHost, st));
    if (S->sparse_sweeps && S->sp.ctl) HIPCHK(hipMemcpyAsync(sp_ctl, S->sp.ctl, sizeof(sp_ctl), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&evals, S->evals, sizeof(evals), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    {
        char where[32];
        snprintf(where, sizeof(where), "GPU slab %d", S->slab);
        if (int rc = check_oob(err, where)) return rc;
    }
    if (prof) {
        sdfgen_hip_profile p;
        memset(&p, 0, sizeof(p));
        float ms = 0;
        hipEvent_t *ev = S->ev;
        HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[20]));
        p.total_ms = ms;
        HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        p.prep_ms = ms;
        HIPCHK(hipEventElapsedTime(&ms, ev[1], ev[2]));
        p.band_ms = ms;
        HIPCHK(hipEventElapsedTime(&ms, ev[3], ev[19]));
        p.sweep_ms = ms;
        for (int s = 0; s < 16; ++s) {
            HIPCHK(hipEventElapsedTime(&ms, ev[3 + s], ev[(s == 15) ? 19 : 4 + s]));
            p.sweep_launch_ms[s] = ms;
        }
        HIPCHK(hipEventElapsedTime(&ms, ev[19], ev[20]));
        p.sign_ms = ms;
        p.sweep_launches = S->launches;
        p.sweep_impl = S->sparse_sweeps ? 2 : 1;   // as on one GPU; `slabs` says it ran split
        p.band_evals = evals;
        p.sparse_sweeps = S->sparse_sweeps;
        p.sparse_first = S->sparse_sweeps ? 8 : 16;
        p.sparse_rechecks = sp_ctl[SP_RUNS];
        p.sparse_claims = sp_ctl[SP_ENQ];
        p.tile_multi = S->tile_multi;
        p.chain_steps = S->tile_multi ? S->wf.chain_steps : 0.0;
        p.tile_cfg = S->tile_multi ? S->wf.cfg : 0;
        p.slabs = S->nslabs;
        int khz = 0;   // device wall clock (wall_clock64) rate
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, S->device) != hipSuccess || khz <= 0)
            khz = 100000;
        const double tick_ms = 1.0 / khz;
        for (int m = 0; m < 8; ++m) {
            p.slab_wait_done_ms[m] = tm[TM_WAIT_DONE + m] * tick_ms;
            p.slab_wait_ready_ms[m] = tm[TM_WAIT_READY + m] * tick_ms;
            p.slab_repair_ms[m] = tm[TM_REPAIR + m] * tick_ms;
            p.slab_inbound_ms[m] = tm[TM_INBOUND + m] * tick_ms;
            p.slab_inbound_entries[m] = tm[TM_INBOUND_N + m];
        }
        p.slab_inbox_idle_ms = tm[TM_INBOX_IDLE] * tick_ms;
        p.slab_other_idle_ms = tm[TM_OTHER_IDLE] * tick_ms;
        p.slab_inbox_tasks = tm[TM_INBOX_TASKS];
        p.slab_other_tasks = tm[TM_OTHER_TASKS];
        *prof = p;
    }
    char who[256];
    slab_where(S, who, sizeof(who));
    if (wf_err[0] & 4) {
        // the first-pass inbox is written by the slab upstream in the failed sweep's k direction
        const int sw = wf_err[1] - 1, up = (sw >= 0 && SWEEP_DIRS[sw % 8][2] < 0) ? S->slab + 1 : S->slab - 1;
        return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: upstream slab %d's plane never arrived (sweep %d)", who, up, sw);
    }
    if (wf_err[0])
        return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: sweep watchdog fired (lost tile hand-off, code %d, sweep %d)", who,
                       wf_err[0], wf_err[1] - 1);
    if (sp_ctl[SP_ERR] & 16ull)
        return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: a neighbour slab's second-pass handshake never came", who);
    if (sp_ctl[SP_ERR] & 8ull) return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: inbound boundary ring overflow", who);
    if (sp_ctl[SP_ERR] & 4ull) return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: Jacobi list overflow", who);
    if (sp_ctl[SP_ERR]) return err.set(SDFGEN_HIP_ERUNTIME, "GPU %s: sparse sweep watchdog fired", who);
    if (flag) return err.set(SDFGEN_HIP_EINDEX, "triangle vertex index out of range (>= %llu vertices)",
                             (unsigned long long)nvert);
    return 0;
}

// ngpu > 1 in sdfgen_hip_make_level_set3: one Z-slab session per device (0..n-1), connected
// in-process, driven from this thread.  Every slab's kernels are enqueued before any result is
// copied back: a slab's sweeps wait on its neighbours' planes, and a D2H copy into pageable
// memory blocks the host until its slab has finished.
// SDFGEN_DEBUG_SLABS_ONE_DEVICE (diagnostics/tests on a one-GPU box): every slab on device 0;
// then SDFGEN_TILE_GRID must cap the persistent grids so all slabs stay co-resident.
}  // namespace

struct sdfgen_hip_slab {
    SlabSession s;
};

namespace {

struct SlabRef {
    sdfgen_hip_slab *h = nullptr;
};
SlabSession *slab_of(sdfgen_hip_slab *h) { return &h->s; }

int run_zslab_local(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert, const float origin[3],
                    float dx, int ni, int nj, int nk, int band, int n, int layout, float *phi_out, Err &err)
{
    const bool one_dev = getenv("SDFGEN_DEBUG_SLABS_ONE_DEVICE") != nullptr;
    std::vector<SlabRef> S(n);
    struct Cleanup {
        std::vector<SlabRef> &s;
        ~Cleanup()
        {
            for (auto &r : s) sdfgen_hip_slab_destroy(r.h);
        }
    } cleanup{S};
    int rc;
    for (int g = 0; g < n; ++g)
        if ((rc = sdfgen_hip_slab_create(one_dev ? 0 : g, n, g, ni, nj, nk, &S[g].h, err.buf, err.len))) return rc;
    for (int g = 0; g < n; ++g)
        if ((rc = sdfgen_hip_slab_connect_local(S[g].h, g > 0 ? S[g - 1].h : nullptr,
                                                g < n - 1 ? S[g + 1].h : nullptr, err.buf, err.len)))
            return rc;
    // all allocations and uploads first, then every slab's kernels: setting a slab up while an
    // earlier slab's kernels already wait on it can block this thread
    for (int g = 0; g < n; ++g) {
        SlabSession *T = slab_of(S[g].h);
        HIPCHK(hipSetDevice(T->device));
        const uint64_t nout = (uint64_t)ni * nj * (T->k_end - T->k_begin);
        HIPCHK(hipMalloc((void **)&T->tri, std::max<size_t>(12 * ntri, 16)));
        T->cap_tri = 12 * ntri;
        HIPCHK(hipMalloc((void **)&T->xyz, std::max<size_t>(12 * nvert, 16)));
        T->cap_xyz = 12 * nvert;
        HIPCHK(hipMalloc((void **)&T->out, std::max<size_t>(4 * nout, 16)));
        T->cap_out = 4 * nout;
        if (ntri) HIPCHK(hipMemcpyAsync(T->tri, tri, 12 * ntri, hipMemcpyHostToDevice, T->stream));
        if (nvert) HIPCHK(hipMemcpyAsync(T->xyz, xyz, 12 * nvert, hipMemcpyHostToDevice, T->stream));
        if ((rc = slab_prepare(T, ntri, err))) return rc;
        HIPCHK(hipStreamSynchronize(T->stream));
    }
    for (int g = 0; g < n; ++g) {
        SlabSession *T = slab_of(S[g].h);
        HIPCHK(hipSetDevice(T->device));
        if ((rc = slab_enqueue(T, T->tri, ntri, T->xyz, nvert, origin, dx, band, layout, T->out, err))) return rc;
    }
    for (int g = 0; g < n; ++g) {   // slab results into the caller's grid
        SlabSession *T = slab_of(S[g].h);
        HIPCHK(hipSetDevice(T->device));
        const size_t nks = (size_t)(T->k_end - T->k_begin);
        if (layout == SDFGEN_LAYOUT_ARRAY3)   // i-fastest: the slab's planes are one contiguous range
            HIPCHK(hipMemcpyAsync(phi_out + (size_t)T->k_begin * ni * nj, T->out, 4 * nks * ni * nj,
                                  hipMemcpyDeviceToHost, T->stream));
        else   // k-fastest: rows of nks values land at stride nk
            HIPCHK(hipMemcpy2DAsync(phi_out + T->k_begin, 4 * (size_t)nk, T->out, 4 * nks, 4 * nks,
                                    (size_t)ni * nj, hipMemcpyDeviceToHost, T->stream));
    }
    int first = 0;
    sdfgen_hip_profile slowest;
    memset(&slowest, 0, sizeof(slowest));
    for (int g = 0; g < n; ++g) {   // collect every slab's status, report the first failure
        Err e2{nullptr, 0};
        SlabSession *T = slab_of(S[g].h);
        HIPCHK(hipSetDevice(T->device));
        sdfgen_hip_profile p;
        memset(&p, 0, sizeof(p));
        rc = slab_finish(T, nvert, &p, first ? e2 : err);
        if (rc && !first) first = rc;
        if (!rc && (g == 0 || p.total_ms > slowest.total_ms)) slowest = p;
    }
    if (!first) {   // sdfgen_hip_last_profile of an ngpu > 1 call: the slowest slab's (its `slabs` = n)
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof = slowest;
    }
    return first;
}

}  // namespace

extern "C" {

int sdfgen_hip_abi_version(void) { return SDFGEN_HIP_ABI_VERSION; }

int sdfgen_hip_device_count(void) { return device_count_impl(); }

int sdfgen_hip_topology(int max_dev, int *ndev, char *pci_bus_ids, int *peer)
{
    DeviceGuard dg_;
    if (!ndev || max_dev < 0) return SDFGEN_HIP_EINVAL;
    const int n = std::max(device_count_impl(), 0);
    *ndev = n;
    const int m = std::min(n, max_dev);
    for (int i = 0; i < m; ++i) {
        if (pci_bus_ids) {
            char *b = pci_bus_ids + (size_t)SDFGEN_HIP_PCI_ID_BYTES * i;
            if (hipDeviceGetPCIBusId(b, SDFGEN_HIP_PCI_ID_BYTES, i) != hipSuccess) b[0] = 0;
        }
        if (peer)
            for (int j = 0; j < m; ++j) {
                int ok = i == j;
                if (i != j && hipDeviceCanAccessPeer(&ok, i, j) != hipSuccess) ok = -1;
                peer[(size_t)i * max_dev + j] = ok;
            }
    }
    (void)hipGetLastError();
    return 0;
}

int sdfgen_hip_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                               const float origin[3], float dx, int ni, int nj, int nk, int exact_band, int ngpu,
                               int out_layout, float *phi_out, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    int rc = validate(ntri, nvert, dx, ni, nj, nk, out_layout, err);
    if (rc) return rc;
    if (!phi_out || !origin || (ntri && (!tri || !xyz)))
        return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    if (ngpu < 0) return err.set(SDFGEN_HIP_EINVAL, "ngpu = %d (0 = all devices, 1 = the current device, n > 1)", ngpu);
    const int ndev = device_count_impl();
    if (ndev <= 0) return err.set(SDFGEN_HIP_ENODEV, "GPU backend requested but no HIP GPU device is available");
    const int want = ngpu == SDFGEN_NGPU_ALL ? ndev : ngpu;
    if (want > ndev && !getenv("SDFGEN_DEBUG_SLABS_ONE_DEVICE"))
        return err.set(SDFGEN_HIP_ENODEV, "ngpu = %d but only %d HIP device(s) visible", ngpu, ndev);
    if (want > 1 && nk >= 4) {
        const int n = std::min(want, nk / 2);
        return run_zslab_local(tri, ntri, xyz, nvert, origin, dx, ni, nj, nk, exact_band, n, out_layout, phi_out,
                               err);
    }
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    Workspace *ws = nullptr;
    if ((rc = get_ws(dev, &ws, err))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    HIPCHK(hipSetDevice(dev));
    const uint64_t n = (uint64_t)ni * nj * nk;
    if ((rc = grow(&ws->tri, &ws->cap_tri, std::max<uint64_t>(3 * ntri, 1), err))) return rc;
    if ((rc = grow(&ws->xyz, &ws->cap_xyz, std::max<uint64_t>(3 * nvert, 1), err))) return rc;
    if ((rc = grow(&ws->out, &ws->cap_out, n, err))) return rc;
    float *d_out = ws->out;
    hipStream_t st = ws->stream;
    if (ntri) {
        HIPCHK(hipMemcpyAsync(ws->tri, tri, 3 * ntri * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ws->xyz, xyz, 3 * nvert * sizeof(float), hipMemcpyHostToDevice, st));
    }
    rc = run_pipeline(ws, st, ws->tri, ntri, ws->xyz, nvert, origin, dx, ni, nj, nk, exact_band, out_layout, d_out,
                      err);
    if (rc == 0) {
        // a pageable copy: its cost here is mostly first-touch page faults of the caller's
        // fresh buffer (a pinned, 8-thread staged copy-out measured no faster)
        hipError_t e = hipMemcpyAsync(phi_out, d_out, n * sizeof(float), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = err.set(SDFGEN_HIP_ERUNTIME, "GPU (HIP) error %s copying phi", hipGetErrorName(e));
    }
    return rc;
}

int sdfgen_hip_make_level_set3_device(int device, const uint32_t *d_tri, uint64_t ntri, const float *d_xyz,
                                      uint64_t nvert, const float origin[3], float dx, int ni, int nj, int nk,
                                      int exact_band, int out_layout, float *d_phi_out, void *hip_stream,
                                      char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    int rc = validate(ntri, nvert, dx, ni, nj, nk, out_layout, err);
    if (rc) return rc;
    if (!d_phi_out || !origin || (ntri && (!d_tri || !d_xyz)))
        return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    const int ndev = device_count_impl();
    if (device < 0 || device >= ndev) return err.set(SDFGEN_HIP_ENODEV, "GPU device %d not available", device);
    HIPCHK(hipSetDevice(device));
    Workspace *ws = nullptr;
    if ((rc = get_ws(device, &ws, err))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    HIPCHK(hipSetDevice(device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ws->stream;
    return run_pipeline(ws, st, d_tri, ntri, d_xyz, nvert, origin, dx, ni, nj, nk, exact_band, out_layout, d_phi_out,
                        err);
}

// Diagnostics: stage 1 only (prep, init, band + ray parity) on the current device, with the
// pre-sweep state copied back: phi and closest_tri per cell (i-fastest) and the intersection
// counts -- what oracle_band computes (cpu_lib/makelevelset3.cpp:196-236).  *big_n = big-triangle
// entries the band phase handed to k_band_big.
int sdfgen_hip_debug_band(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert, const float origin[3],
                          float dx, int ni, int nj, int nk, int exact_band, float *phi, int32_t *ct, uint32_t *cnt,
                          uint64_t *big_n, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    int rc = validate(ntri, nvert, dx, ni, nj, nk, SDFGEN_LAYOUT_ARRAY3, err);
    if (rc) return rc;
    if (!phi || !ct || !cnt || !origin || (ntri && (!tri || !xyz))) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    if (device_count_impl() <= 0) return err.set(SDFGEN_HIP_ENODEV, "no HIP GPU device is available");
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    Workspace *ws = nullptr;
    if ((rc = get_ws(dev, &ws, err))) return rc;
    std::lock_guard<std::mutex> lk(ws->mu);
    HIPCHK(hipSetDevice(dev));
    const uint64_t n = (uint64_t)ni * nj * nk;
    if ((rc = grow(&ws->tri, &ws->cap_tri, std::max<uint64_t>(3 * ntri, 1), err))) return rc;
    if ((rc = grow(&ws->xyz, &ws->cap_xyz, std::max<uint64_t>(3 * nvert, 1), err))) return rc;
    if ((rc = grow(&ws->cell, &ws->cap_cell, sp_pad(n), err))) return rc;   // (k_sp_jscan2 reads past the last cell)
    if ((rc = grow(&ws->cnt, &ws->cap_cnt, n, err))) return rc;
    if ((rc = grow(&ws->soup, &ws->cap_soup, 3 * std::max<uint64_t>(ntri, 1), err))) return rc;
    if (!ws->err_flag) {
        HIPCHK(hipMalloc((void **)&ws->err_flag, sizeof(int)));
        HIPCHK(hipMalloc((void **)&ws->evals, sizeof(unsigned long long)));
        HIPCHK(hipMalloc((void **)&ws->status, STATUS_N * sizeof(unsigned long long)));
    }
    hipStream_t st = ws->stream;
    if (ntri) {
        HIPCHK(hipMemcpyAsync(ws->tri, tri, 3 * ntri * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ws->xyz, xyz, 3 * nvert * sizeof(float), hipMemcpyHostToDevice, st));
    }
    Grid g{origin[0], origin[1], origin[2], dx, ni, nj, nk};
    const float init = (float)(ni + nj + nk) * dx;
    const u64 init_key = ((u64)__builtin_bit_cast(uint32_t, init) << 32) | 0xffffffffull;
    HIPCHK(zero_async(ws->err_flag, sizeof(int), st));
    if (ntri) {
        hipLaunchKernelGGL(k_prep_soup, dim3(grid_for(ntri, 256, 8192)), dim3(256), 0, st, ws->tri, ntri, ws->xyz, nvert,
                           ws->soup, ws->err_flag);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_init, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, ws->cell, ws->cnt, n, init_key);
    HIPCHK(hipGetLastError());
    if ((rc = band_enqueue(ws->band, st, ws->soup, ntri, g, exact_band, init, ws->cell, ws->cnt, nullptr, 0, nk, err)))
        return rc;
    int flag = 0;
    uint32_t nb = 0;
    HIPCHK(hipMemcpyAsync(&flag, ws->err_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    if (ntri) HIPCHK(hipMemcpyAsync(&nb, ws->band.big.n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(cnt, ws->cnt, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    std::vector<u64> cells(n);
    HIPCHK(hipMemcpyAsync(cells.data(), ws->cell, n * sizeof(u64), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if ((rc = check_oob(err, "debug_band"))) return rc;
    if (flag) return err.set(SDFGEN_HIP_EINDEX, "triangle vertex index out of range (>= %llu vertices)",
                             (unsigned long long)nvert);
    for (uint64_t q = 0; q < n; ++q) {
        const uint32_t hi = (uint32_t)(cells[q] >> 32);
        memcpy(phi + q, &hi, 4);
        ct[q] = lbl_of((uint32_t)cells[q]);
    }
    if (big_n) *big_n = nb;
    return 0;
}

int sdfgen_hip_last_profile(sdfgen_hip_profile *out)
{
    if (!out) return SDFGEN_HIP_EINVAL;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    *out = g_prof;
    return 0;
}

int sdfgen_hip_release(void)
{
    DeviceGuard dg_;
    std::lock_guard<std::mutex> lk(g_mu);
    // every workspace is freed; the first failing call (a sticky fault of an earlier kernel surfaces here)
    // is what the return code reports
    hipError_t first = hipSuccess;
    auto chk = [&first](hipError_t e) { if (first == hipSuccess && e != hipSuccess) first = e; };
    for (Workspace *w : g_ws) {
        chk(hipSetDevice(w->device));
        chk(hipFree(w->cell));
        chk(hipFree(w->cnt));
        chk(hipFree(w->soup));
        chk(hipFree(w->tri));
        chk(hipFree(w->xyz));
        chk(hipFree(w->err_flag));
        chk(hipFree(w->evals));
        chk(hipFree(w->status));
        chk(hipFree(w->out));
        tile_sweep_release(w->wf);
        sparse_sweep_release(w->sp);
        band_release(w->band);
        for (auto &e : w->ev) chk(hipEventDestroy(e));
        chk(hipStreamDestroy(w->stream));
        delete w;
    }
    g_ws.clear();
    if (first != hipSuccess) {
        sdf_last_hip = first;
        return SDFGEN_HIP_ERUNTIME;
    }
    // the pool of uncached communication blocks and the imported neighbour blocks (Z-slabs over IPC) are
    // kept: freeing them is what the pool avoids; sdfgen_hip_slab_close_imports is the
    // caller's explicit choice
    return 0;
}

int sdfgen_hip_slab_close_imports(void)
{
    DeviceGuard dg_;
    return comm_close_imports();
}

int sdfgen_hip_debug_sweep_trace(int device, uint64_t *out, uint64_t max_entries, uint64_t *n_out)
{
    DeviceGuard dg_;
    Err err{nullptr, 0};
    *n_out = 0;
    Workspace *ws = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (Workspace *w : g_ws)
            if (w->device == device) ws = w;
    }
    if (!ws || !ws->wf.trace) return SDFGEN_HIP_EINVAL;
    std::lock_guard<std::mutex> lk(ws->mu);
    HIPCHK(hipSetDevice(device));
    const uint64_t n = std::min<uint64_t>(max_entries, ws->wf.cap_trace);
    HIPCHK(hipMemcpy(out, ws->wf.trace, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    *n_out = n;
    return 0;
}

int sdfgen_hip_debug_ptd(int device, int variant, uint64_t n, const float *pts, float *out, char *errbuf,
                         size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (device < 0 || device >= device_count_impl()) return err.set(SDFGEN_HIP_ENODEV, "no GPU device %d", device);
    HIPCHK(hipSetDevice(device));
    float *dp = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc((void **)&dp, std::max<uint64_t>(n, 1) * 12 * sizeof(float)));
    HIPCHK(hipMalloc((void **)&dout, std::max<uint64_t>(n, 1) * sizeof(float)));
    HIPCHK(hipMemcpy(dp, pts, n * 12 * sizeof(float), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_ptd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, dp, dout, variant);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dp));
    HIPCHK(hipFree(dout));
    return 0;
}

int sdfgen_hip_debug_pit2d(int device, uint64_t n, const double *pit, double *out4, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (device < 0 || device >= device_count_impl()) return err.set(SDFGEN_HIP_ENODEV, "no GPU device %d", device);
    HIPCHK(hipSetDevice(device));
    double *dp = nullptr, *dout = nullptr;
    HIPCHK(hipMalloc((void **)&dp, std::max<uint64_t>(n, 1) * 8 * sizeof(double)));
    HIPCHK(hipMalloc((void **)&dout, std::max<uint64_t>(n, 1) * 4 * sizeof(double)));
    HIPCHK(hipMemcpy(dp, pit, n * 8 * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_pit2d, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, dp, dout);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(out4, dout, n * 4 * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dp));
    HIPCHK(hipFree(dout));
    return 0;
}


// ---------------------------------------------------------------- Z-slab sessions

int sdfgen_hip_slab_create(int device, int nslabs, int slab, int ni, int nj, int nk, sdfgen_hip_slab **out,
                           char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    if (!out) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    *out = nullptr;
    int rc = validate(0, 0, 1.0f, ni, nj, nk, SDFGEN_LAYOUT_ARRAY3, err);
    if (rc) return rc;
    if (nslabs < 1 || slab < 0 || slab >= nslabs) return err.set(SDFGEN_HIP_EINVAL, "slab %d of %d", slab, nslabs);
    if (nk < 2 * nslabs) return err.set(SDFGEN_HIP_EINVAL, "nz = %d too small for %d slabs (need >= 2 planes each)", nk, nslabs);
    if (device < 0 || device >= device_count_impl()) return err.set(SDFGEN_HIP_ENODEV, "GPU device %d not available", device);
    {
        int live = 0;
        {
            std::lock_guard<std::mutex> lk(g_comm_mu);
            if ((size_t)device < g_dev_slabs.size()) live = g_dev_slabs[device];
        }
        if (live + 1 > hw_queues())
            return err.set(SDFGEN_HIP_EINVAL,
                           "%d slab sessions on device %d need as many hardware queues; this process has %d "
                           "(GPU_MAX_HW_QUEUES): slabs sharing a queue would run one after the other while each waits "
                           "on its neighbours", live + 1, device, hw_queues());
    }
    sdfgen_hip_slab *h = new sdfgen_hip_slab();
    SlabSession *S = &h->s;
    S->device = device;
    S->nslabs = nslabs;
    S->slab = slab;
    S->ni = ni;
    S->nj = nj;
    S->nk = nk;
    S->k_begin = (int)((long long)slab * nk / nslabs);
    S->k_end = (int)((long long)(slab + 1) * nk / nslabs);
    if ((rc = slab_alloc(S, err))) {
        slab_free(S);
        delete h;
        return rc;
    }
    *out = h;
    return 0;
}

int sdfgen_hip_slab_range(const sdfgen_hip_slab *h, int *k_begin, int *k_end)
{
    if (!h || !k_begin || !k_end) return SDFGEN_HIP_EINVAL;
    *k_begin = h->s.k_begin;
    *k_end = h->s.k_end;
    return 0;
}

int sdfgen_hip_slab_export(sdfgen_hip_slab *h, void *handle, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (!h || !handle) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    static_assert(sizeof(hipIpcMemHandle_t) <= SDFGEN_HIP_IPC_HANDLE_BYTES, "IPC handle size");
    HIPCHK(hipSetDevice(h->s.device));
    hipIpcMemHandle_t m;
    if (int rc = comm_export(h->s.comm, &m, err)) return rc;
    memset(handle, 0, SDFGEN_HIP_IPC_HANDLE_BYTES);
    memcpy(handle, &m, sizeof(m));
    return 0;
}

int sdfgen_hip_slab_connect_ipc(sdfgen_hip_slab *h, const void *lower, const void *upper, char *errbuf,
                                size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    SlabSession *S = &h->s;
    if ((S->slab > 0) != (lower != nullptr) || (S->slab < S->nslabs - 1) != (upper != nullptr))
        return err.set(SDFGEN_HIP_EINVAL, "slab %d of %d needs exactly its existing neighbours", S->slab, S->nslabs);
    HIPCHK(hipSetDevice(S->device));
    const void *hs[2] = {lower, upper};
    for (int side = 0; side < 2; ++side) {
        if (!hs[side]) continue;
        hipIpcMemHandle_t m;
        memcpy(&m, hs[side], sizeof(m));
        void *p = nullptr;
        if (int rc = comm_import(S->device, m, &p, err)) return rc;
        S->peer[side] = (char *)p;
        // Which GPU holds the neighbour's block is not known here: hipPointerGetAttributes on an IPC
        // mapping reports the importing device, not the owner, and the 64-byte handle has no
        // room for the owner's id.  So the neighbour's device stays "unknown" (-1) in slab_where's errors;
        // a failed mapping fails in hipIpcOpenMemHandle above, and bench.py's `topology` record ties each
        // rank to its device and PCI id.  (connect_local knows both devices and checks peer access.)
        S->peer_dev[side] = -1;
        // the mapping must cover the neighbour's whole block (same grid => same layout)
        void *base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, p) == hipSuccess && base &&
            (char *)base + size < (char *)p + S->cl.bytes)
            return err.set(SDFGEN_HIP_ERUNTIME, "IPC mapping of slab %d's neighbour is %zu bytes, expected %zu",
                           S->slab, size, S->cl.bytes);
    }
    return 0;
}

int sdfgen_hip_slab_connect_local(sdfgen_hip_slab *h, sdfgen_hip_slab *lower, sdfgen_hip_slab *upper, char *errbuf,
                                  size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    SlabSession *S = &h->s;
    if ((S->slab > 0) != (lower != nullptr) || (S->slab < S->nslabs - 1) != (upper != nullptr))
        return err.set(SDFGEN_HIP_EINVAL, "slab %d of %d needs exactly its existing neighbours", S->slab, S->nslabs);
    HIPCHK(hipSetDevice(S->device));
    for (sdfgen_hip_slab *o : {lower, upper}) {
        if (!o || o->s.device == S->device) continue;
        int ok = 0;
        HIPCHK(hipDeviceCanAccessPeer(&ok, S->device, o->s.device));
        if (!ok) return err.set(SDFGEN_HIP_ERUNTIME, "GPU %d cannot access GPU %d", S->device, o->s.device);
        hipError_t e = hipDeviceEnablePeerAccess(o->s.device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
        (void)hipGetLastError();
    }
    S->peer[0] = lower ? lower->s.comm : nullptr;
    S->peer[1] = upper ? upper->s.comm : nullptr;
    S->peer_dev[0] = lower ? lower->s.device : -1;
    S->peer_dev[1] = upper ? upper->s.device : -1;
    return 0;
}

int sdfgen_hip_slab_enqueue(sdfgen_hip_slab *h, const uint32_t *d_tri, uint64_t ntri, const float *d_xyz,
                            uint64_t nvert, const float origin[3], float dx, int exact_band, int out_layout,
                            float *d_phi_slab, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    SlabSession *S = &h->s;
    int rc = validate(ntri, nvert, dx, S->ni, S->nj, S->nk, out_layout, err);
    if (rc) return rc;
    if (!d_phi_slab || !origin || (ntri && (!d_tri || !d_xyz)))
        return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    std::lock_guard<std::mutex> lk(S->mu);
    HIPCHK(hipSetDevice(S->device));
    return slab_enqueue(S, d_tri, ntri, d_xyz, nvert, origin, dx, exact_band, out_layout, d_phi_slab, err);
}

int sdfgen_hip_slab_prepare(sdfgen_hip_slab *h, uint64_t ntri, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    std::lock_guard<std::mutex> lk(h->s.mu);
    return slab_prepare(&h->s, ntri, err);
}

int sdfgen_hip_slab_finish(sdfgen_hip_slab *h, uint64_t nvert, sdfgen_hip_profile *prof, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    std::lock_guard<std::mutex> lk(h->s.mu);
    HIPCHK(hipSetDevice(h->s.device));
    return slab_finish(&h->s, nvert, prof, err);
}

int sdfgen_hip_slab_run(sdfgen_hip_slab *h, const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                        const float origin[3], float dx, int exact_band, int out_layout, float *phi_slab,
                        sdfgen_hip_profile *prof, char *errbuf, size_t errlen)
{
    DeviceGuard dg_;
    Err err{errbuf, errlen};
    if (errbuf && errlen) errbuf[0] = 0;
    if (!h) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    SlabSession *S = &h->s;
    int rc = validate(ntri, nvert, dx, S->ni, S->nj, S->nk, out_layout, err);
    if (rc) return rc;
    if (!phi_slab || !origin || (ntri && (!tri || !xyz))) return err.set(SDFGEN_HIP_EINVAL, "null pointer argument");
    std::lock_guard<std::mutex> lk(S->mu);
    HIPCHK(hipSetDevice(S->device));
    const uint64_t nout = (uint64_t)S->ni * S->nj * (S->k_end - S->k_begin);
    auto grow_raw = [&](auto **p, size_t *cap, size_t bytes) -> int {
        if (*p && *cap >= bytes) return 0;
        if (*p) HIPCHK(hipFree(*p));
        *p = nullptr;
        *cap = 0;
        HIPCHK(hipMalloc((void **)p, std::max<size_t>(bytes, 16)));
        *cap = bytes;
        return 0;
    };
    if ((rc = grow_raw(&S->tri, &S->cap_tri, 12 * ntri))) return rc;
    if ((rc = grow_raw(&S->xyz, &S->cap_xyz, 12 * nvert))) return rc;
    if ((rc = grow_raw(&S->out, &S->cap_out, 4 * nout))) return rc;
    if (ntri) HIPCHK(hipMemcpyAsync(S->tri, tri, 12 * ntri, hipMemcpyHostToDevice, S->stream));
    if (nvert) HIPCHK(hipMemcpyAsync(S->xyz, xyz, 12 * nvert, hipMemcpyHostToDevice, S->stream));
    if ((rc = slab_enqueue(S, S->tri, ntri, S->xyz, nvert, origin, dx, exact_band, out_layout, S->out, err)))
        return rc;
    HIPCHK(hipMemcpyAsync(phi_slab, S->out, 4 * nout, hipMemcpyDeviceToHost, S->stream));
    return slab_finish(S, nvert, prof, err);
}

int sdfgen_hip_slab_debug_dump(sdfgen_hip_slab *h, int which, void *out, uint64_t max_bytes, uint64_t *n_bytes)
{
    DeviceGuard dg_;
    if (!h || !out || !n_bytes) return SDFGEN_HIP_EINVAL;
    SlabSession *S = &h->s;
    if (hipSetDevice(S->device) != hipSuccess || hipStreamSynchronize(S->stream) != hipSuccess) return SDFGEN_HIP_ERUNTIME;
    const void *src = nullptr;
    size_t bytes = 0;
    if (which == 0) { src = S->comm; bytes = S->cl.bytes; }
    else if (which == 1 && S->wf.ctrl) { src = S->wf.ctrl; bytes = 16 * sizeof(int); }
    else if (which == 2 && S->wf.mdone) { src = S->wf.mdone; bytes = S->wf.cap_mtasks * sizeof(unsigned); }
    else if (which == 3 && S->wf.mtasks) { src = S->wf.mtasks; bytes = S->wf.cap_mtasks * sizeof(int4); }
    else if (which == 4 && S->wf.mdeps) { src = S->wf.mdeps; bytes = S->wf.cap_mtasks * ST_MAXDEP * sizeof(int); }
    bytes = std::min<size_t>(bytes, max_bytes);
    *n_bytes = bytes;
    if (bytes && hipMemcpy(out, src, bytes, hipMemcpyDeviceToHost) != hipSuccess) return SDFGEN_HIP_ERUNTIME;
    return 0;
}

int sdfgen_hip_slab_destroy(sdfgen_hip_slab *h)
{
    DeviceGuard dg_;
    if (!h) return 0;
    slab_free(&h->s);
    delete h;
    return 0;
}

}  // extern "C"
