// cpu_backend.cpp -- the library's native CPU backend (HardwareBackend::CPU).
//
// Same algorithm and bits as the reference CPU implementation
// (cpu_lib/makelevelset3.cpp:192-304, single-thread semantics) and as the HIP
// path, but multi-threaded WITHOUT the reference's sweep race:
//   band   : triangles in any order, per-cell packed-key atomic min
//            (f32bits(d)<<32 | t) == the CPU's ascending-t strict-< rule;
//            ray-parity counts by atomic add.
//   sweep  : per (pass, direction), the oriented j range is cut into one block
//            per thread; thread t processes k-planes in sweep order and starts
//            plane c only after thread t-1 (its upwind neighbour in j) has
//            finished plane c -- a pipelined wavefront that respects every
//            Gauss-Seidel dependency, so any thread count gives identical bits.
//   sign   : rows in parallel.
// Compiled by hipcc as host code (geometry shared with the kernels via geom.hpp).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <new>
#include <vector>

#include "geom.hpp"
#include "sdfgen_cpu.h"

using namespace sdfhip;

namespace {

typedef unsigned long long u64;

int set_err(char *buf, size_t len, int code, const char *fmt, ...)
{
    if (buf && len) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, len, fmt, ap);
        va_end(ap);
    }
    return code;
}

inline size_t cidx(int i, int j, int k, int ni, int nj)
{
    return (size_t)i + (size_t)ni * ((size_t)j + (size_t)nj * (size_t)k);
}

class Barrier {
   public:
    explicit Barrier(int n) : n_(n) {}
    void wait()
    {
        std::unique_lock<std::mutex> lk(mu_);
        int gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen != gen_; });
        }
    }

   private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0, gen_ = 0;
};

const int SWEEP_DIRS[8][3] = {{+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
                              {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};

struct Job {
    const uint32_t *tri;
    uint64_t ntri;
    const float *xyz;
    float ox, oy, oz, dx;
    int ni, nj, nk, band;
    float init;
    u64 *cell;
    uint32_t *cnt;
    std::atomic<uint64_t> next_tri{0};
    std::atomic<uint64_t> next_row{0};
    std::vector<std::atomic<int>> progress;
    int nthreads;
    Barrier *bar;
    int layout;
    float *out;
    int k_lo = 0, k_hi = 0;   // planes owned (whole grid: 0..nk)
};

inline f3 vtx(const Job &J, uint32_t q) { return mk3(J.xyz[3 * (size_t)q], J.xyz[3 * (size_t)q + 1], J.xyz[3 * (size_t)q + 2]); }

inline void atomic_min_u64(u64 *p, u64 v)
{
    u64 cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
}

// :203-236.  Planes outside [J.k_lo, J.k_hi) are skipped (a Z-slab); boxes are clamped
// to the whole grid first, as the reference does.
void band_triangle(Job &J, uint64_t t)
{
    const f3 xp = vtx(J, J.tri[3 * t]), xq = vtx(J, J.tri[3 * t + 1]), xr = vtx(J, J.tri[3 * t + 2]);
    const double ox = J.ox, oy = J.oy, oz = J.oz, ddx = J.dx;
    double fip = ((double)xp.x - ox) / ddx, fjp = ((double)xp.y - oy) / ddx, fkp = ((double)xp.z - oz) / ddx;
    double fiq = ((double)xq.x - ox) / ddx, fjq = ((double)xq.y - oy) / ddx, fkq = ((double)xq.z - oz) / ddx;
    double fir = ((double)xr.x - ox) / ddx, fjr = ((double)xr.y - oy) / ddx, fkr = ((double)xr.z - oz) / ddx;
    const int b = J.band;
    int i0 = clampi(wrap_add(trunc_to_int(dmin3(fip, fiq, fir)), -b), 0, J.ni - 1);
    int i1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fip, fiq, fir)), b), 1), 0, J.ni - 1);
    int j0 = clampi(wrap_add(trunc_to_int(dmin3(fjp, fjq, fjr)), -b), 0, J.nj - 1);
    int j1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fjp, fjq, fjr)), b), 1), 0, J.nj - 1);
    int k0 = clampi(wrap_add(trunc_to_int(dmin3(fkp, fkq, fkr)), -b), 0, J.nk - 1);
    int k1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fkp, fkq, fkr)), b), 1), 0, J.nk - 1);
    k0 = std::max(k0, J.k_lo);
    k1 = std::min(k1, J.k_hi - 1);
    for (int k = k0; k <= k1; ++k)
        for (int j = j0; j <= j1; ++j)
            for (int i = i0; i <= i1; ++i) {
                f3 gx = mk3((float)i * J.dx + J.ox, (float)j * J.dx + J.oy, (float)k * J.dx + J.oz);
                float d = ptd(gx, xp, xq, xr);
                if (d < J.init) atomic_min_u64(J.cell + cidx(i, j, k, J.ni, J.nj), ((u64)f2u(d) << 32) | (u64)(uint32_t)t);
            }
    j0 = clampi(trunc_to_int(std::ceil(dmin3(fjp, fjq, fjr))), 0, J.nj - 1);
    j1 = clampi(trunc_to_int(std::floor(dmax3(fjp, fjq, fjr))), 0, J.nj - 1);
    k0 = clampi(trunc_to_int(std::ceil(dmin3(fkp, fkq, fkr))), 0, J.nk - 1);
    k1 = clampi(trunc_to_int(std::floor(dmax3(fkp, fkq, fkr))), 0, J.nk - 1);
    k0 = std::max(k0, J.k_lo);
    k1 = std::min(k1, J.k_hi - 1);
    for (int k = k0; k <= k1; ++k)
        for (int j = j0; j <= j1; ++j) {
            double a, bb, c;
            if (pit2d((double)j, (double)k, fjp, fkp, fjq, fkq, fjr, fkr, a, bb, c)) {
                double fi = (a * fip + bb * fiq) + c * fir;
                int ii = trunc_to_int(std::ceil(fi));
                if (ii < 0) __atomic_fetch_add(J.cnt + cidx(0, j, k, J.ni, J.nj), 1u, __ATOMIC_RELAXED);
                else if (ii < J.ni) __atomic_fetch_add(J.cnt + cidx(ii, j, k, J.ni, J.nj), 1u, __ATOMIC_RELAXED);
            }
        }
}

// check_neighbour chain :90-102, :143-149 (skips are exact: see sdfgen_hip.hip sweep_cell)
inline void sweep_cell(Job &J, int i, int j, int k, int di, int dj, int dk)
{
    const size_t c0 = cidx(i, j, k, J.ni, J.nj);
    const u64 own = J.cell[c0];
    float phi = u2f((uint32_t)(own >> 32));
    int32_t ct = (int32_t)(uint32_t)own;
    const int32_t ct_orig = ct;
    const size_t nbi[7] = {cidx(i - di, j, k, J.ni, J.nj),      cidx(i, j - dj, k, J.ni, J.nj),
                           cidx(i - di, j - dj, k, J.ni, J.nj), cidx(i, j, k - dk, J.ni, J.nj),
                           cidx(i - di, j, k - dk, J.ni, J.nj), cidx(i, j - dj, k - dk, J.ni, J.nj),
                           cidx(i - di, j - dj, k - dk, J.ni, J.nj)};
    int32_t nb[7];
    for (int q = 0; q < 7; ++q) nb[q] = (int32_t)(uint32_t)J.cell[nbi[q]];
    const f3 gx = mk3((float)i * J.dx + J.ox, (float)j * J.dx + J.oy, (float)k * J.dx + J.oz);
    bool changed = false;
    for (int q = 0; q < 7; ++q) {
        const int32_t t = nb[q];
        bool skip = (t < 0) || (t == ct_orig);
        for (int r = 0; r < q && !skip; ++r) skip = (nb[r] == t);
        if (skip) continue;
        const uint32_t *tv = J.tri + 3 * (size_t)t;
        float d = ptd(gx, vtx(J, tv[0]), vtx(J, tv[1]), vtx(J, tv[2]));
        if (d < phi) {
            phi = d;
            ct = t;
            changed = true;
        }
    }
    if (changed) J.cell[c0] = ((u64)f2u(phi) << 32) | (u64)(uint32_t)ct;
}

void worker(Job &J, int tid)
{
    const int T = J.nthreads;
    // ---- band ----
    for (;;) {
        uint64_t t0 = J.next_tri.fetch_add(64);
        if (t0 >= J.ntri) break;
        uint64_t t1 = std::min<uint64_t>(J.ntri, t0 + 64);
        for (uint64_t t = t0; t < t1; ++t) band_triangle(J, t);
    }
    J.bar->wait();
    // ---- sweeps ----
    const int A = J.ni - 1, B = J.nj - 1, C = J.nk - 1;
    if (A > 0 && B > 0 && C > 0 && J.ntri > 0) {
        const int nb = std::min(T, B);
        const int b_lo = (int)((int64_t)tid * B / nb), b_hi = (int)((int64_t)(tid + 1) * B / nb);
        for (int s = 0; s < 16; ++s) {
            const int di = SWEEP_DIRS[s % 8][0], dj = SWEEP_DIRS[s % 8][1], dk = SWEEP_DIRS[s % 8][2];
            if (tid < nb) {
                for (int c = 0; c < C; ++c) {
                    if (tid > 0)
                        while (J.progress[tid - 1].load(std::memory_order_acquire) <= c) std::this_thread::yield();
                    const int k = dk > 0 ? c + 1 : J.nk - 2 - c;
                    for (int b = b_lo; b < b_hi; ++b) {
                        const int j = dj > 0 ? b + 1 : J.nj - 2 - b;
                        for (int a = 0; a < A; ++a) sweep_cell(J, di > 0 ? a + 1 : J.ni - 2 - a, j, k, di, dj, dk);
                    }
                    J.progress[tid].store(c + 1, std::memory_order_release);
                }
            }
            J.bar->wait();
            if (tid < nb) J.progress[tid].store(0, std::memory_order_relaxed);
            J.bar->wait();
        }
    }
    // ---- sign (:294-303) + output layout ----
    const uint64_t rows = (uint64_t)J.nj * J.nk;
    for (;;) {
        uint64_t r0 = J.next_row.fetch_add(16);
        if (r0 >= rows) break;
        for (uint64_t r = r0; r < std::min<uint64_t>(rows, r0 + 16); ++r) {
            const int j = (int)(r % J.nj), k = (int)(r / J.nj);
            int total = 0;
            for (int i = 0; i < J.ni; ++i) {
                const size_t q = cidx(i, j, k, J.ni, J.nj);
                total += (int)J.cnt[q];
                uint32_t bits = (uint32_t)(J.cell[q] >> 32);
                if (total % 2 == 1) bits ^= 0x80000000u;
                const float v = u2f(bits);
                if (J.layout == 0) J.out[q] = v;
                else J.out[((size_t)i * J.nj + j) * J.nk + k] = v;
            }
        }
    }
}

}  // namespace

extern "C" int sdfgen_cpu_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                                          const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                                          int num_threads, int out_layout, float *phi_out, char *errbuf,
                                          size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (ni <= 0 || nj <= 0 || nk <= 0)
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "Grid dimensions must be positive (nx, ny, nz > 0)");
    if (!(dx > 0.0f) || !std::isfinite(dx))
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "Cell spacing dx must be positive");
    if (out_layout != 0 && out_layout != 1)
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "out_layout must be 0 or 1");
    if (!phi_out || !origin || (ntri && (!tri || !xyz)))
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "null pointer argument");
    if (ntri > 0x7fffffffull) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "too many triangles");
    for (uint64_t q = 0; q < 3 * ntri; ++q)
        if ((uint64_t)tri[q] >= nvert)
            return set_err(errbuf, errlen, SDFGEN_CPU_EINDEX, "triangle %llu references vertex %u >= %llu vertices",
                           (unsigned long long)(q / 3), tri[q], (unsigned long long)nvert);
    const size_t n = (size_t)ni * nj * nk;
    std::vector<u64> cell;
    std::vector<uint32_t> cnt;
    try {
        cell.resize(n);
        cnt.assign(n, 0u);
    } catch (...) {
        return set_err(errbuf, errlen, SDFGEN_CPU_ENOMEM, "out of host memory for %zu cells", n);
    }
    int T = num_threads > 0 ? num_threads : (int)std::thread::hardware_concurrency();
    if (T <= 0) T = 4;
    T = std::min(T, 512);
    Job J;
    J.tri = tri;
    J.ntri = ntri;
    J.xyz = xyz;
    J.ox = origin[0];
    J.oy = origin[1];
    J.oz = origin[2];
    J.dx = dx;
    J.ni = ni;
    J.nj = nj;
    J.nk = nk;
    J.band = exact_band;
    J.k_lo = 0;
    J.k_hi = nk;
    J.init = (float)(ni + nj + nk) * dx;  // :197
    const u64 init_key = ((u64)f2u(J.init) << 32) | 0xffffffffull;
    std::fill(cell.begin(), cell.end(), init_key);
    J.cell = cell.data();
    J.cnt = cnt.data();
    J.progress = std::vector<std::atomic<int>>(T);
    for (auto &p : J.progress) p.store(0);
    J.nthreads = T;
    Barrier bar(T);
    J.bar = &bar;
    J.layout = out_layout;
    J.out = phi_out;
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    for (int t = 1; t < T; ++t) pool.emplace_back(worker, std::ref(J), t);
    worker(J, 0);
    for (auto &th : pool) th.join();
    return SDFGEN_CPU_OK;
}

// ---------------------------------------------------------------------------
// CPU Z-slab sessions (include/sdfgen_cpu.h): the host-side counterpart of
// sdfgen_hip_slab_*, for multi-process runs without GPUs (and the gloo tests).
// One sweep at a time: the caller passes the upstream slab's final boundary plane in
// and ships this slab's boundary plane on, so slabs run one after another within a
// sweep (the GPU sessions pipeline them).  Single-threaded per slab; bit-identical.
// ---------------------------------------------------------------------------
struct sdfgen_cpu_slab {
    int nslabs, slab, ni, nj, nk, k_begin, k_end;
    std::vector<u64> cell;
    std::vector<uint32_t> cnt;
    const uint32_t *tri = nullptr;
    const float *xyz = nullptr;
    uint64_t ntri = 0;
    float ox = 0, oy = 0, oz = 0, dx = 0;
};

extern "C" int sdfgen_cpu_slab_create(int nslabs, int slab, int ni, int nj, int nk, sdfgen_cpu_slab **out,
                                      char *errbuf, size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (!out) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "null pointer argument");
    *out = nullptr;
    if (ni <= 0 || nj <= 0 || nk <= 0)
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "Grid dimensions must be positive (nx, ny, nz > 0)");
    if (nslabs < 1 || slab < 0 || slab >= nslabs) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "slab %d of %d", slab, nslabs);
    if (nk < 2 * nslabs)
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "nz = %d too small for %d slabs (need >= 2 planes each)", nk, nslabs);
    sdfgen_cpu_slab *S = new (std::nothrow) sdfgen_cpu_slab();
    if (!S) return set_err(errbuf, errlen, SDFGEN_CPU_ENOMEM, "out of host memory");
    S->nslabs = nslabs;
    S->slab = slab;
    S->ni = ni;
    S->nj = nj;
    S->nk = nk;
    S->k_begin = (int)((long long)slab * nk / nslabs);
    S->k_end = (int)((long long)(slab + 1) * nk / nslabs);
    try {
        S->cell.resize((size_t)ni * nj * nk);
        S->cnt.assign((size_t)ni * nj * nk, 0u);
    } catch (...) {
        delete S;
        return set_err(errbuf, errlen, SDFGEN_CPU_ENOMEM, "out of host memory");
    }
    *out = S;
    return SDFGEN_CPU_OK;
}

extern "C" int sdfgen_cpu_slab_range(const sdfgen_cpu_slab *S, int *k_begin, int *k_end)
{
    if (!S || !k_begin || !k_end) return SDFGEN_CPU_EINVAL;
    *k_begin = S->k_begin;
    *k_end = S->k_end;
    return SDFGEN_CPU_OK;
}

extern "C" int sdfgen_cpu_slab_band(sdfgen_cpu_slab *S, const uint32_t *tri, uint64_t ntri, const float *xyz,
                                    uint64_t nvert, const float origin[3], float dx, int exact_band, char *errbuf,
                                    size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (!S || !origin || (ntri && (!tri || !xyz))) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "null pointer argument");
    if (!(dx > 0.0f) || !std::isfinite(dx)) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "Cell spacing dx must be positive");
    for (uint64_t q = 0; q < 3 * ntri; ++q)
        if ((uint64_t)tri[q] >= nvert)
            return set_err(errbuf, errlen, SDFGEN_CPU_EINDEX, "triangle %llu references vertex %u >= %llu vertices",
                           (unsigned long long)(q / 3), tri[q], (unsigned long long)nvert);
    S->tri = tri;
    S->xyz = xyz;
    S->ntri = ntri;
    S->ox = origin[0];
    S->oy = origin[1];
    S->oz = origin[2];
    S->dx = dx;
    Job J;
    J.tri = tri;
    J.ntri = ntri;
    J.xyz = xyz;
    J.ox = origin[0];
    J.oy = origin[1];
    J.oz = origin[2];
    J.dx = dx;
    J.ni = S->ni;
    J.nj = S->nj;
    J.nk = S->nk;
    J.band = exact_band;
    J.k_lo = S->k_begin;
    J.k_hi = S->k_end;
    J.init = (float)(S->ni + S->nj + S->nk) * dx;
    const u64 init_key = ((u64)f2u(J.init) << 32) | 0xffffffffull;
    std::fill(S->cell.begin(), S->cell.end(), init_key);
    std::fill(S->cnt.begin(), S->cnt.end(), 0u);
    J.cell = S->cell.data();
    J.cnt = S->cnt.data();
    for (uint64_t t = 0; t < ntri; ++t) band_triangle(J, t);
    return SDFGEN_CPU_OK;
}

// Sweep `sweep` (0..15) over this slab.  plane_in: the upstream slab's boundary plane
// (ni*nj cells, k = k_begin-1 for k-up sweeps / k_end for k-down), NULL for the first
// slab; plane_out (NULL for the last): this slab's last plane after the sweep.
extern "C" int sdfgen_cpu_slab_sweep(sdfgen_cpu_slab *S, int sweep, const uint64_t *plane_in, uint64_t *plane_out,
                                     char *errbuf, size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (!S || sweep < 0 || sweep > 15) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "bad sweep");
    const int di = SWEEP_DIRS[sweep % 8][0], dj = SWEEP_DIRS[sweep % 8][1], dk = SWEEP_DIRS[sweep % 8][2];
    const size_t pc = (size_t)S->ni * S->nj;
    const int k_up = dk > 0 ? S->k_begin - 1 : S->k_end;    // upstream plane
    const int k_last = dk > 0 ? S->k_end - 1 : S->k_begin;  // this slab's last plane
    const bool first = dk > 0 ? S->slab == 0 : S->slab == S->nslabs - 1;
    const bool last = dk > 0 ? S->slab == S->nslabs - 1 : S->slab == 0;
    if (!first != (plane_in != nullptr) || !last != (plane_out != nullptr))
        return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "slab %d sweep %d: plane_in/plane_out must match the neighbours",
                       S->slab, sweep);
    if (plane_in) std::copy(plane_in, plane_in + pc, S->cell.begin() + pc * (size_t)k_up);
    if (S->ni >= 2 && S->nj >= 2 && S->nk >= 2 && S->ntri > 0) {
        Job J;
        J.tri = S->tri;
        J.ntri = S->ntri;
        J.xyz = S->xyz;
        J.ox = S->ox;
        J.oy = S->oy;
        J.oz = S->oz;
        J.dx = S->dx;
        J.ni = S->ni;
        J.nj = S->nj;
        J.nk = S->nk;
        J.cell = S->cell.data();
        // reference loop order (:130-151) restricted to this slab's k planes
        const int k0 = dk > 0 ? std::max(S->k_begin, 1) : std::min(S->k_end, S->nk - 1) - 1;
        const int k1 = dk > 0 ? S->k_end : S->k_begin - 1;
        for (int k = k0; k != k1; k += dk)
            for (int j = dj > 0 ? 1 : S->nj - 2; j != (dj > 0 ? S->nj : -1); j += dj)
                for (int i = di > 0 ? 1 : S->ni - 2; i != (di > 0 ? S->ni : -1); i += di) sweep_cell(J, i, j, k, di, dj, dk);
    }
    if (plane_out) std::copy(S->cell.begin() + pc * (size_t)k_last, S->cell.begin() + pc * (size_t)(k_last + 1), plane_out);
    return SDFGEN_CPU_OK;
}

extern "C" int sdfgen_cpu_slab_sign(sdfgen_cpu_slab *S, int out_layout, float *phi_slab, char *errbuf, size_t errlen)
{
    if (errbuf && errlen) errbuf[0] = 0;
    if (!S || !phi_slab) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "null pointer argument");
    if (out_layout != 0 && out_layout != 1) return set_err(errbuf, errlen, SDFGEN_CPU_EINVAL, "out_layout must be 0 or 1");
    const int kc = S->k_end - S->k_begin;
    for (int k = S->k_begin; k < S->k_end; ++k)
        for (int j = 0; j < S->nj; ++j) {
            int total = 0;
            for (int i = 0; i < S->ni; ++i) {
                const size_t q = cidx(i, j, k, S->ni, S->nj);
                total += (int)S->cnt[q];
                uint32_t bits = (uint32_t)(S->cell[q] >> 32);
                if (total % 2 == 1) bits ^= 0x80000000u;
                const float v = u2f(bits);
                if (out_layout == 0) phi_slab[cidx(i, j, k - S->k_begin, S->ni, S->nj)] = v;
                else phi_slab[((size_t)i * S->nj + j) * kc + (k - S->k_begin)] = v;
            }
        }
    return SDFGEN_CPU_OK;
}

extern "C" int sdfgen_cpu_slab_destroy(sdfgen_cpu_slab *S)
{
    delete S;
    return SDFGEN_CPU_OK;
}
