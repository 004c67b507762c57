/*
 * oracle/sdf_oracle.c -- CPU restatement of the reference make_level_set3 hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (via oracle/oracle.py).  The product library
 * (sdfgenfast_amd/csrc) never links, loads or calls anything in oracle/.
 *
 * It restates, in plain C99, the single-threaded semantics of
 *   /root/reference/cpu_lib/makelevelset3.cpp:192-304  (sdfgen::cpu::make_level_set3,
 *   num_threads=1 -- the multi-threaded sweep races)
 * with the exact floating-point evaluation order of the reference's value
 * types (common/vec.h:216-255, 331-337, 377-383; common/util.h:22-23, 59-61,
 * 113-115, 341-347).  It must be compiled with contraction off
 * (-ffp-contract=off) and without -ffast-math; on x86-64 without -march it
 * uses SSE2 scalar arithmetic, exactly like the reference's Release build.
 *
 * Parity pinning: tests/test_oracle_golden.py checks this restatement
 * bit-for-bit against fixtures produced by the reference's own
 * cpu_lib/makelevelset3.cpp compiled from /root/reference by
 * oracle/Makefile (target _ref) -- see tests/golden/make_golden.py.
 */
#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* std::min / std::max as used by the reference (common/util.h:22-23). */
static inline float fmin_std(float a, float b) { return (b < a) ? b : a; }
static inline float fmax_std(float a, float b) { return (a < b) ? b : a; }
static inline double dmin_std(double a, double b) { return (b < a) ? b : a; }
static inline double dmax_std(double a, double b) { return (a < b) ? b : a; }
/* min(a1,a2,a3) = min(a1, min(a2,a3))   common/util.h:59-61, 113-115 */
static inline double dmin3(double a, double b, double c) { return dmin_std(a, dmin_std(b, c)); }
static inline double dmax3(double a, double b, double c) { return dmax_std(a, dmax_std(b, c)); }
/* clamp   common/util.h:341-347 */
static inline int clampi(int a, int lo, int hi) { return (a < lo) ? lo : ((a > hi) ? hi : a); }

/* C++ int(double) on x86-64 (cvttsd2si): truncation, INT_MIN when out of range/NaN. */
static inline int trunc_to_int(double v)
{
    if (v > -2147483649.0 && v < 2147483648.0) return (int)v;
    return INT32_MIN;
}
/* int + int with two's-complement wrap (what the reference's x86 build does). */
static inline int wrap_add(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }

/* mag2: ((a0*a0)+a1*a1)+a2*a2   common/vec.h:216-222 */
static inline float mag2f(const float a[3]) { return (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]; }
/* dot: ((a0*b0)+a1*b1)+a2*b2    common/vec.h:377-383 */
static inline float dotf(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
/* dist: sqrt(dist2)              common/vec.h:239-255 */
static inline float distf(const float a[3], const float b[3])
{
    float d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    return sqrtf((d0 * d0 + d1 * d1) + d2 * d2);
}

/* point_segment_distance   cpu_lib/makelevelset3.cpp:21-34 */
static float psd(const float x0[3], const float x1[3], const float x2[3])
{
    float e[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
    double m2 = (double)mag2f(e);
    float t[3] = {x2[0] - x0[0], x2[1] - x0[1], x2[2] - x0[2]};
    float s12 = (float)((double)dotf(t, e) / m2);
    if (s12 < 0) s12 = 0;
    else if (s12 > 1) s12 = 1;
    float w = 1.0f - s12;
    /* s12*x1 + (1-s12)*x2  (vec.h:331-337 then vec.h:92-103) */
    float p[3] = {x1[0] * s12 + x2[0] * w, x1[1] * s12 + x2[1] * w, x1[2] * s12 + x2[2] * w};
    return distf(x0, p);
}

/* point_triangle_distance   cpu_lib/makelevelset3.cpp:49-70 */
float oracle_ptd(const float x0[3], const float x1[3], const float x2[3], const float x3[3])
{
    float x13[3] = {x1[0] - x3[0], x1[1] - x3[1], x1[2] - x3[2]};
    float x23[3] = {x2[0] - x3[0], x2[1] - x3[1], x2[2] - x3[2]};
    float x03[3] = {x0[0] - x3[0], x0[1] - x3[1], x0[2] - x3[2]};
    float m13 = mag2f(x13), m23 = mag2f(x23), d = dotf(x13, x23);
    float invdet = 1.f / fmax_std(m13 * m23 - d * d, 1e-30f);
    float a = dotf(x13, x03), b = dotf(x23, x03);
    float w23 = invdet * (m23 * a - d * b);
    float w31 = invdet * (m13 * b - d * a);
    float w12 = (1.0f - w23) - w31;
    if (w23 >= 0 && w31 >= 0 && w12 >= 0) {
        float p[3];
        for (int c = 0; c < 3; ++c) p[c] = (x1[c] * w23 + x2[c] * w31) + x3[c] * w12;
        return distf(x0, p);
    } else {
        if (w23 > 0) return fmin_std(psd(x0, x1, x2), psd(x0, x1, x3));
        else if (w31 > 0) return fmin_std(psd(x0, x1, x2), psd(x0, x2, x3));
        else return fmin_std(psd(x0, x1, x3), psd(x0, x2, x3));
    }
}

/* orientation   cpu_lib/makelevelset3.cpp:155-165 */
static int orientation(double x1, double y1, double x2, double y2, double *twice_signed_area)
{
    *twice_signed_area = y1 * x2 - x1 * y2;
    if (*twice_signed_area > 0) return 1;
    else if (*twice_signed_area < 0) return -1;
    else if (y2 > y1) return 1;
    else if (y2 < y1) return -1;
    else if (x1 > x2) return 1;
    else if (x1 < x2) return -1;
    else return 0;
}

/* point_in_triangle_2d   cpu_lib/makelevelset3.cpp:169-187 (assert compiled out) */
int oracle_pit2d(double x0, double y0, double x1, double y1, double x2, double y2,
                 double x3, double y3, double *a, double *b, double *c)
{
    x1 -= x0; x2 -= x0; x3 -= x0;
    y1 -= y0; y2 -= y0; y3 -= y0;
    int signa = orientation(x2, y2, x3, y3, a);
    if (signa == 0) return 0;
    int signb = orientation(x3, y3, x1, y1, b);
    if (signb != signa) return 0;
    int signc = orientation(x1, y1, x2, y2, c);
    if (signc != signa) return 0;
    double sum = (*a + *b) + *c;
    *a /= sum;
    *b /= sum;
    *c /= sum;
    return 1;
}

static inline size_t cidx(int i, int j, int k, int ni, int nj)
{
    return (size_t)i + (size_t)ni * ((size_t)j + (size_t)nj * (size_t)k);
}

static int check_args(const uint32_t *tri, uint64_t ntri, uint64_t nvert, int ni, int nj, int nk)
{
    if (ni <= 0 || nj <= 0 || nk <= 0) return -1;
    for (uint64_t t = 0; t < ntri; ++t)
        for (int c = 0; c < 3; ++c)
            if ((uint64_t)tri[3 * t + c] >= nvert) return -2;
    return 0;
}

/*
 * Stage 1: init + narrow band + ray-parity counts.
 *   cpu_lib/makelevelset3.cpp:196-236
 * phi, ct, cnt: ni*nj*nk entries, i-fastest (common/array3.h:114).
 */
int oracle_band(const uint32_t *tri, uint64_t ntri, const float *x, uint64_t nvert,
                const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                float *phi, int32_t *ct, int32_t *cnt)
{
    int rc = check_args(tri, ntri, nvert, ni, nj, nk);
    if (rc) return rc;
    size_t n = (size_t)ni * nj * nk;
    float init = (float)(ni + nj + nk) * dx; /* (ni+nj+nk)*dx, int*float :197 */
    for (size_t q = 0; q < n; ++q) { phi[q] = init; ct[q] = -1; cnt[q] = 0; }

    for (uint64_t t = 0; t < ntri; ++t) {
        const float *xp = x + 3 * (size_t)tri[3 * t + 0];
        const float *xq = x + 3 * (size_t)tri[3 * t + 1];
        const float *xr = x + 3 * (size_t)tri[3 * t + 2];
        /* :206-208 */
        double fip = ((double)xp[0] - origin[0]) / dx, fjp = ((double)xp[1] - origin[1]) / dx, fkp = ((double)xp[2] - origin[2]) / dx;
        double fiq = ((double)xq[0] - origin[0]) / dx, fjq = ((double)xq[1] - origin[1]) / dx, fkq = ((double)xq[2] - origin[2]) / dx;
        double fir = ((double)xr[0] - origin[0]) / dx, fjr = ((double)xr[1] - origin[1]) / dx, fkr = ((double)xr[2] - origin[2]) / dx;
        /* :210-212 */
        int i0 = clampi(wrap_add(trunc_to_int(dmin3(fip, fiq, fir)), -exact_band), 0, ni - 1);
        int i1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fip, fiq, fir)), exact_band), 1), 0, ni - 1);
        int j0 = clampi(wrap_add(trunc_to_int(dmin3(fjp, fjq, fjr)), -exact_band), 0, nj - 1);
        int j1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fjp, fjq, fjr)), exact_band), 1), 0, nj - 1);
        int k0 = clampi(wrap_add(trunc_to_int(dmin3(fkp, fkq, fkr)), -exact_band), 0, nk - 1);
        int k1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fkp, fkq, fkr)), exact_band), 1), 0, nk - 1);
        /* :213-220 */
        for (int k = k0; k <= k1; ++k)
            for (int j = j0; j <= j1; ++j)
                for (int i = i0; i <= i1; ++i) {
                    float gx[3] = {(float)i * dx + origin[0], (float)j * dx + origin[1], (float)k * dx + origin[2]};
                    float d = oracle_ptd(gx, xp, xq, xr);
                    size_t q = cidx(i, j, k, ni, nj);
                    if (d < phi[q]) { phi[q] = d; ct[q] = (int32_t)t; }
                }
        /* :222-235 */
        j0 = clampi(trunc_to_int(ceil(dmin3(fjp, fjq, fjr))), 0, nj - 1);
        j1 = clampi(trunc_to_int(floor(dmax3(fjp, fjq, fjr))), 0, nj - 1);
        k0 = clampi(trunc_to_int(ceil(dmin3(fkp, fkq, fkr))), 0, nk - 1);
        k1 = clampi(trunc_to_int(floor(dmax3(fkp, fkq, fkr))), 0, nk - 1);
        for (int k = k0; k <= k1; ++k)
            for (int j = j0; j <= j1; ++j) {
                double a, b, c;
                if (oracle_pit2d((double)j, (double)k, fjp, fkp, fjq, fkq, fjr, fkr, &a, &b, &c)) {
                    double fi = (a * fip + b * fiq) + c * fir;
                    int ii = trunc_to_int(ceil(fi));
                    if (ii < 0) ++cnt[cidx(0, j, k, ni, nj)];
                    else if (ii < ni) ++cnt[cidx(ii, j, k, ni, nj)];
                }
            }
    }
    return 0;
}

/*
 * Stage 1 again, split over host threads by planes: thread r fills k in [k_lo, k_hi) and runs
 * EVERY triangle in ascending t over those planes only.  A cell sees the same triangles in the
 * same order as in oracle_band (the band boxes and ray lattices are the reference's whole-grid
 * boxes, cut to the planes afterwards), so phi / ct / cnt are bit-identical -- pinned against
 * oracle_band by tests/test_oracle_golden.py.  For big parity cases (> 2^32 band evaluations).
 * phi, ct and cnt must be initialised by the caller (oracle_band_mt does it).
 */
typedef struct {
    const uint32_t *tri; uint64_t ntri; const float *x; const float *origin; float dx;
    int ni, nj, nk, exact_band, k_lo, k_hi; float *phi; int32_t *ct; int32_t *cnt;
} band_job;

static void band_planes(const band_job *J)
{
    const float *origin = J->origin;
    const float dx = J->dx;
    const int ni = J->ni, nj = J->nj, nk = J->nk, exact_band = J->exact_band;
    for (uint64_t t = 0; t < J->ntri; ++t) {
        const float *xp = J->x + 3 * (size_t)J->tri[3 * t + 0];
        const float *xq = J->x + 3 * (size_t)J->tri[3 * t + 1];
        const float *xr = J->x + 3 * (size_t)J->tri[3 * t + 2];
        double fip = ((double)xp[0] - origin[0]) / dx, fjp = ((double)xp[1] - origin[1]) / dx, fkp = ((double)xp[2] - origin[2]) / dx;
        double fiq = ((double)xq[0] - origin[0]) / dx, fjq = ((double)xq[1] - origin[1]) / dx, fkq = ((double)xq[2] - origin[2]) / dx;
        double fir = ((double)xr[0] - origin[0]) / dx, fjr = ((double)xr[1] - origin[1]) / dx, fkr = ((double)xr[2] - origin[2]) / dx;
        int i0 = clampi(wrap_add(trunc_to_int(dmin3(fip, fiq, fir)), -exact_band), 0, ni - 1);
        int i1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fip, fiq, fir)), exact_band), 1), 0, ni - 1);
        int j0 = clampi(wrap_add(trunc_to_int(dmin3(fjp, fjq, fjr)), -exact_band), 0, nj - 1);
        int j1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fjp, fjq, fjr)), exact_band), 1), 0, nj - 1);
        int k0 = clampi(wrap_add(trunc_to_int(dmin3(fkp, fkq, fkr)), -exact_band), 0, nk - 1);
        int k1 = clampi(wrap_add(wrap_add(trunc_to_int(dmax3(fkp, fkq, fkr)), exact_band), 1), 0, nk - 1);
        if (k0 < J->k_lo) k0 = J->k_lo;
        if (k1 > J->k_hi - 1) k1 = J->k_hi - 1;
        for (int k = k0; k <= k1; ++k)
            for (int j = j0; j <= j1; ++j)
                for (int i = i0; i <= i1; ++i) {
                    float gx[3] = {(float)i * dx + origin[0], (float)j * dx + origin[1], (float)k * dx + origin[2]};
                    float d = oracle_ptd(gx, xp, xq, xr);
                    size_t q = cidx(i, j, k, ni, nj);
                    if (d < J->phi[q]) { J->phi[q] = d; J->ct[q] = (int32_t)t; }
                }
        j0 = clampi(trunc_to_int(ceil(dmin3(fjp, fjq, fjr))), 0, nj - 1);
        j1 = clampi(trunc_to_int(floor(dmax3(fjp, fjq, fjr))), 0, nj - 1);
        k0 = clampi(trunc_to_int(ceil(dmin3(fkp, fkq, fkr))), 0, nk - 1);
        k1 = clampi(trunc_to_int(floor(dmax3(fkp, fkq, fkr))), 0, nk - 1);
        if (k0 < J->k_lo) k0 = J->k_lo;
        if (k1 > J->k_hi - 1) k1 = J->k_hi - 1;
        for (int k = k0; k <= k1; ++k)
            for (int j = j0; j <= j1; ++j) {
                double a, b, c;
                if (oracle_pit2d((double)j, (double)k, fjp, fkp, fjq, fkq, fjr, fkr, &a, &b, &c)) {
                    double fi = (a * fip + b * fiq) + c * fir;
                    int ii = trunc_to_int(ceil(fi));
                    if (ii < 0) ++J->cnt[cidx(0, j, k, ni, nj)];
                    else if (ii < ni) ++J->cnt[cidx(ii, j, k, ni, nj)];
                }
            }
    }
}

static void *band_thread(void *arg)
{
    band_planes((const band_job *)arg);
    return NULL;
}

int oracle_band_mt(const uint32_t *tri, uint64_t ntri, const float *x, uint64_t nvert,
                   const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                   float *phi, int32_t *ct, int32_t *cnt, int nthreads)
{
    int rc = check_args(tri, ntri, nvert, ni, nj, nk);
    if (rc) return rc;
    size_t n = (size_t)ni * nj * nk;
    float init = (float)(ni + nj + nk) * dx;
    for (size_t q = 0; q < n; ++q) { phi[q] = init; ct[q] = -1; cnt[q] = 0; }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nk) nthreads = nk;
    if (nthreads > 256) nthreads = 256;
    band_job jobs[256];
    pthread_t th[256];
    for (int r = 0; r < nthreads; ++r) {
        band_job J = {tri, ntri, x, origin, dx, ni, nj, nk, exact_band,
                      (int)((int64_t)nk * r / nthreads), (int)((int64_t)nk * (r + 1) / nthreads), phi, ct, cnt};
        jobs[r] = J;
    }
    int started = 0;
    for (int r = 1; r < nthreads; ++r) {
        if (pthread_create(&th[r], NULL, band_thread, &jobs[r]) != 0) break;
        started = r;
    }
    band_planes(&jobs[0]);
    for (int r = started + 1; r < nthreads; ++r) band_planes(&jobs[r]);   /* threads that failed to start */
    for (int r = 1; r <= started; ++r) pthread_join(th[r], NULL);
    return 0;
}

/*
 * Stage 2: 2 passes x 8 directions of Gauss-Seidel sweeps, single thread.
 *   cpu_lib/makelevelset3.cpp:90-102 (check_neighbour), :130-151 (sweep_range),
 *   :243-291 (pass/direction driver).
 */
static const int SWEEP_DIRS[8][3] = {
    {+1, +1, +1}, {-1, -1, -1}, {+1, +1, -1}, {-1, -1, +1},
    {+1, -1, +1}, {-1, +1, -1}, {+1, -1, -1}, {-1, +1, +1}};

static void check_neighbour(const uint32_t *tri, const float *x, float *phi, int32_t *ct,
                            const float gx[3], size_t c0, size_t c1)
{
    int32_t t = ct[c1];
    if (t >= 0) {
        const float *xp = x + 3 * (size_t)tri[3 * (size_t)t + 0];
        const float *xq = x + 3 * (size_t)tri[3 * (size_t)t + 1];
        const float *xr = x + 3 * (size_t)tri[3 * (size_t)t + 2];
        float d = oracle_ptd(gx, xp, xq, xr);
        if (d < phi[c0]) { phi[c0] = d; ct[c0] = t; }
    }
}

void oracle_sweep_one(const uint32_t *tri, const float *x, const float origin[3], float dx,
                      int ni, int nj, int nk, float *phi, int32_t *ct, int di, int dj, int dk)
{
    int i0 = di > 0 ? 1 : ni - 2, i1 = di > 0 ? ni : -1;
    int j0 = dj > 0 ? 1 : nj - 2, j1 = dj > 0 ? nj : -1;
    int k0 = dk > 0 ? 1 : nk - 2, k1 = dk > 0 ? nk : -1;
    if (ni < 2 || nj < 2 || nk < 2) return; /* empty ranges (loops below would not run either) */
    for (int k = k0; k != k1; k += dk)
        for (int j = j0; j != j1; j += dj)
            for (int i = i0; i != i1; i += di) {
                float gx[3] = {(float)i * dx + origin[0], (float)j * dx + origin[1], (float)k * dx + origin[2]};
                size_t c = cidx(i, j, k, ni, nj);
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i - di, j, k, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i, j - dj, k, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i - di, j - dj, k, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i, j, k - dk, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i - di, j, k - dk, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i, j - dj, k - dk, ni, nj));
                check_neighbour(tri, x, phi, ct, gx, c, cidx(i - di, j - dj, k - dk, ni, nj));
            }
}

/* nsweeps: how many of the 16 (pass, direction) sweeps to run, in order (16 = full). */
void oracle_sweep(const uint32_t *tri, const float *x, const float origin[3], float dx,
                  int ni, int nj, int nk, float *phi, int32_t *ct, int nsweeps)
{
    for (int s = 0; s < nsweeps && s < 16; ++s)
        oracle_sweep_one(tri, x, origin, dx, ni, nj, nk, phi, ct,
                         SWEEP_DIRS[s % 8][0], SWEEP_DIRS[s % 8][1], SWEEP_DIRS[s % 8][2]);
}

/* Stage 3: sign from the prefix parity of intersection counts.  :295-303 */
void oracle_sign(int ni, int nj, int nk, const int32_t *cnt, float *phi)
{
    for (int k = 0; k < nk; ++k)
        for (int j = 0; j < nj; ++j) {
            int total = 0;
            for (int i = 0; i < ni; ++i) {
                size_t q = cidx(i, j, k, ni, nj);
                total += cnt[q];
                if (total % 2 == 1) phi[q] = -phi[q];
            }
        }
}

/* Whole pipeline; phi_out is i-fastest (Array3f layout).  Returns 0, -1 bad dims, -2 bad index, -3 OOM. */
int oracle_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *x, uint64_t nvert,
                           const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                           float *phi_out)
{
    size_t n = (size_t)ni * nj * nk;
    if (ni <= 0 || nj <= 0 || nk <= 0) return -1;
    int32_t *ct = (int32_t *)malloc(n * sizeof(int32_t));
    int32_t *cnt = (int32_t *)malloc(n * sizeof(int32_t));
    if (!ct || !cnt) { free(ct); free(cnt); return -3; }
    int rc = oracle_band(tri, ntri, x, nvert, origin, dx, ni, nj, nk, exact_band, phi_out, ct, cnt);
    if (rc == 0) {
        oracle_sweep(tri, x, origin, dx, ni, nj, nk, phi_out, ct, 16);
        oracle_sign(ni, nj, nk, cnt, phi_out);
    }
    free(ct);
    free(cnt);
    return rc;
}

/* Batched point-triangle distance: pts = n x 12 floats (x0,x1,x2,x3). */
void oracle_ptd_batch(uint64_t n, const float *pts, float *out)
{
    for (uint64_t q = 0; q < n; ++q) {
        const float *p = pts + 12 * q;
        out[q] = oracle_ptd(p, p + 3, p + 6, p + 9);
    }
}

/* Batched point_in_triangle_2d: in = n x 8 doubles, out = n x (flag, a, b, c). */
void oracle_pit2d_batch(uint64_t n, const double *in, double *out)
{
    for (uint64_t q = 0; q < n; ++q) {
        const double *p = in + 8 * q;
        double a = 0, b = 0, c = 0;
        int r = oracle_pit2d(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], &a, &b, &c);
        out[4 * q] = r ? 1.0 : 0.0;
        out[4 * q + 1] = a;
        out[4 * q + 2] = b;
        out[4 * q + 3] = c;
    }
}
