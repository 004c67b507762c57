// geom.hpp -- geometry for the gfx950 SDF kernels (and the native CPU backend).
//
// Bit-exact restatement of the reference's CPU arithmetic:
//   point_segment_distance  cpu_lib/makelevelset3.cpp:21-34
//   point_triangle_distance cpu_lib/makelevelset3.cpp:49-70
//   orientation             cpu_lib/makelevelset3.cpp:155-165
//   point_in_triangle_2d    cpu_lib/makelevelset3.cpp:169-187
// with the evaluation order of common/vec.h (mag2 :216-222, dist :239-255,
// dot :377-383, scalar*Vec :331-337) and std::min/max of common/util.h:22-23.
// Every translation unit including this file is compiled -ffp-contract=off
// (the CPU oracle has no FMA), float '/' and sqrt are the IEEE
// correctly-rounded forms, and min/max are written as the std:: selects
// ((b<a)?b:a), never v_min_f32, whose NaN rule differs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

// The same functions serve the device kernels and the library's native CPU backend
// (cpu_backend.cpp, host code of the same hipcc build): SDF_HD marks them for both.
#define SDF_HD __host__ __device__ __forceinline__

namespace sdfhip {

#if defined(__HIPCC__)
// Zeroing of small per-call control words as a compute kernel: hipMemsetAsync runs as a runtime
// blit whose hand-over to the next compute kernel left a ~6 us gap in the stream (kernel trace:
// one before every second-pass sweep).  A template, so each translation unit may instantiate it.
template <int = 0>
__global__ void k_zero32(uint32_t *__restrict__ p, size_t n)
{
    for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < n; x += (size_t)gridDim.x * blockDim.x) p[x] = 0u;
}
// bytes: a multiple of 4
inline hipError_t zero_async(void *p, size_t bytes, hipStream_t st)
{
    const size_t n = bytes / 4;
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_zero32<>, dim3(blocks), dim3(256), 0, st, (uint32_t *)p, n);
    return hipGetLastError();
}
// The HIP status behind the last failed runtime call of this thread's sweep set-up helpers
// (st_grow, sp_grow, the stream syncs before a buffer grows): their error messages name it, so a
// sticky fault of an earlier kernel surfaces as that fault, not as "allocation failed".
inline thread_local hipError_t sdf_last_hip = hipSuccess;
// Record e and map it to the library's status: -5 (out of memory) or -4 (runtime / kernel error).
inline int sdf_hip_rc(hipError_t e)
{
    sdf_last_hip = e;
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? -5 : -4;
}
inline const char *sdf_last_hip_name() { return sdf_last_hip == hipSuccess ? "no HIP error recorded" : hipGetErrorName(sdf_last_hip); }
#endif

// IEEE correctly-rounded float sqrt and division on both sides.  NOTE: on ROCm 7.2
// __fsqrt_rn() lowers to a bare v_sqrt_f32 (1 ulp, NOT correctly rounded); the
// plain builtin gets the v_sqrt + two-FMA-residual fix-up that is.  Plain '/' gets
// the v_div_scale/v_div_fmas/v_div_fixup IEEE sequence.
SDF_HD float sqrt_rn(float x) { return __builtin_sqrtf(x); }
SDF_HD float div_rn(float a, float b) { return a / b; }

struct f3 {
    float x, y, z;
};

SDF_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }

// Low word of a device cell / granule: the closest triangle in 27 bits (all ones = none)
// and, in the top 5 bits, the sweep (+1) in which the cell took that label (0 = band).
// The sweeps' "already examined" skip reads the latter (sweep_sparse.hpp); the band's
// atomicMin keys (phi << 32 | t) are unchanged by it.  Limits meshes to 2^27-1 triangles.
constexpr uint32_t LBL_BITS = 27u, LBL_MASK = (1u << LBL_BITS) - 1u;
SDF_HD int lbl_of(uint32_t w) { const uint32_t l = w & LBL_MASK; return l == LBL_MASK ? -1 : (int)l; }
SDF_HD int lc_of(uint32_t w) { return (int)(w >> LBL_BITS); }
// Debug builds (make BOUNDS=1 -> -DSDFGEN_BOUNDS): every global index the sweep kernels form
// is checked against the buffer it addresses; the first violation is recorded as
// (site << 48 | index) in sdf_oob and the access is redirected to `lo`, so a bad index is
// reported by the host (sdfgen_hip.hip: check_oob) instead of faulting the GPU.
#ifdef SDFGEN_BOUNDS
static __device__ unsigned long long sdf_oob;
__device__ __forceinline__ unsigned long long sdf_chk(unsigned site, unsigned long long x, unsigned long long lo,
                                                      unsigned long long hi)
{
    if (x >= lo && x < hi) return x;
    atomicCAS(&sdf_oob, 0ull, ((unsigned long long)site << 48) | (x & 0xffffffffffffull));
    return lo;
}
#define SDF_CHK(site, x, lo, hi) sdf_chk((site), (unsigned long long)(x), (unsigned long long)(lo), (unsigned long long)(hi))
#else
#define SDF_CHK(site, x, lo, hi) (x)
#endif

// Z-slab phase timers (SlabSession::tm, zeroed per call; wall_clock64 ticks unless a count): where
// a slab's time goes around its neighbours, reported per rank by the N > 1 bench line.
enum : int {
    TM_WAIT_DONE = 0,      // [8] k_sp_slab_wait(DONE) spin per second-pass sweep (the longer side)
    TM_WAIT_READY = 8,     // [8] k_sp_slab_wait(READY) spin
    TM_REPAIR = 16,        // [8] k_sp_recheck: workgroup 0's start .. the last wave's exit
    TM_INBOUND = 24,       // [8] inbound lanes: start .. the upstream slab's DONE seen and its COUNT drained
    TM_INBOUND_N = 32,     // [8] inbound-ring entries taken (count)
    TM_REPAIR_T0 = 40,     // [8] scratch: workgroup 0's start stamp
    TM_INBOX_IDLE = 48,    // first pass: helper-wave idle ticks of the tasks reading the upstream inbox
    TM_INBOX_TASKS = 49,   //   ... their number
    TM_OTHER_IDLE = 50,    // first pass: helper-wave idle ticks of the other tasks
    TM_OTHER_TASKS = 51,   //   ... their number
    TM_N = 64
};

SDF_HD uint32_t lo_word(int label, int lc) { return ((uint32_t)lc << LBL_BITS) | ((uint32_t)label & LBL_MASK); }
SDF_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

SDF_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
SDF_HD f3 sub3(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
SDF_HD float mag2(f3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
SDF_HD float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
SDF_HD float fmin_std(float a, float b) { return (b < a) ? b : a; }
SDF_HD float fmax_std(float a, float b) { return (a < b) ? b : a; }
SDF_HD double dmin_std(double a, double b) { return (b < a) ? b : a; }
SDF_HD double dmax_std(double a, double b) { return (a < b) ? b : a; }
SDF_HD double dmin3(double a, double b, double c) { return dmin_std(a, dmin_std(b, c)); }
SDF_HD double dmax3(double a, double b, double c) { return dmax_std(a, dmax_std(b, c)); }
SDF_HD int clampi(int a, int lo, int hi) { return (a < lo) ? lo : ((a > hi) ? hi : a); }

// C++ int(double) as compiled for x86-64 (cvttsd2si): truncation toward zero,
// INT_MIN when out of range or NaN.  (v_cvt_i32_f64 would saturate instead.)
SDF_HD int trunc_to_int(double v)
{
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : (int)0x80000000;
}
SDF_HD int wrap_add(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }

SDF_HD float dist3(f3 a, f3 b)
{
    f3 d = sub3(a, b);
    return sqrt_rn((d.x * d.x + d.y * d.y) + d.z * d.z);
}

// point_segment_distance.  The reference divides in FP64: (float)((double)dot / (double)m2).
SDF_HD float psd(f3 x0, f3 x1, f3 x2)
{
    f3 e = sub3(x2, x1);
    double m2 = (double)mag2(e);
    f3 t = sub3(x2, x0);
    float s12 = (float)((double)dot3(t, e) / m2);
    if (s12 < 0.0f) s12 = 0.0f;
    else if (s12 > 1.0f) s12 = 1.0f;
    float w = 1.0f - s12;
    f3 p = mk3(x1.x * s12 + x2.x * w, x1.y * s12 + x2.y * w, x1.z * s12 + x2.z * w);
    return dist3(x0, p);
}

// psd before its final sqrt: the squared distance (the device kernels take ONE correctly
// rounded sqrt of the smallest candidate, see ptd_wave)
SDF_HD float psd_sq(f3 x0, f3 x1, f3 x2)
{
    f3 e = sub3(x2, x1);
    double m2 = (double)mag2(e);
    f3 t = sub3(x2, x0);
    float s12 = (float)((double)dot3(t, e) / m2);
    if (s12 < 0.0f) s12 = 0.0f;
    else if (s12 > 1.0f) s12 = 1.0f;
    float w = 1.0f - s12;
    f3 d = sub3(x0, mk3(x1.x * s12 + x2.x * w, x1.y * s12 + x2.y * w, x1.z * s12 + x2.z * w));
    return (d.x * d.x + d.y * d.y) + d.z * d.z;
}

// point_triangle_distance.
SDF_HD float ptd(f3 x0, f3 x1, f3 x2, f3 x3)
{
    f3 x13 = sub3(x1, x3), x23 = sub3(x2, x3), x03 = sub3(x0, x3);
    float m13 = mag2(x13), m23 = mag2(x23), d = dot3(x13, x23);
    float invdet = div_rn(1.0f, fmax_std(m13 * m23 - d * d, 1e-30f));
    float a = dot3(x13, x03), b = dot3(x23, x03);
    float w23 = invdet * (m23 * a - d * b);
    float w31 = invdet * (m13 * b - d * a);
    float w12 = (1.0f - w23) - w31;
    if (w23 >= 0.0f && w31 >= 0.0f && w12 >= 0.0f) {
        f3 p = mk3((x1.x * w23 + x2.x * w31) + x3.x * w12,
                   (x1.y * w23 + x2.y * w31) + x3.y * w12,
                   (x1.z * w23 + x2.z * w31) + x3.z * w12);
        return dist3(x0, p);
    }
    if (w23 > 0.0f) return fmin_std(psd(x0, x1, x2), psd(x0, x1, x3));
    if (w31 > 0.0f) return fmin_std(psd(x0, x1, x2), psd(x0, x2, x3));
    return fmin_std(psd(x0, x1, x3), psd(x0, x2, x3));
}

// point_triangle_distance with no divergent branches (for wave-wide evaluation on
// the GPU).  Bit-identical to ptd(): every case performs the same operations on the
// same operands, and min(first, second) keeps the reference's argument order
// (cpu_lib/makelevelset3.cpp:63-68), which matters for NaN:
//   w23 > 0 : min(psd(x1,x2), psd(x1,x3))
//   w31 > 0 : min(psd(x1,x2), psd(x2,x3))
//   else    : min(psd(x1,x3), psd(x2,x3))
SDF_HD float ptd_nb(f3 x0, f3 x1, f3 x2, f3 x3)
{
    f3 x13 = sub3(x1, x3), x23 = sub3(x2, x3), x03 = sub3(x0, x3);
    float m13 = mag2(x13), m23 = mag2(x23), d = dot3(x13, x23);
    float invdet = div_rn(1.0f, fmax_std(m13 * m23 - d * d, 1e-30f));
    float a = dot3(x13, x03), b = dot3(x23, x03);
    float w23 = invdet * (m23 * a - d * b);
    float w31 = invdet * (m13 * b - d * a);
    float w12 = (1.0f - w23) - w31;
    const bool inside = (w23 >= 0.0f && w31 >= 0.0f && w12 >= 0.0f);
    f3 p = mk3((x1.x * w23 + x2.x * w31) + x3.x * w12,
               (x1.y * w23 + x2.y * w31) + x3.y * w12,
               (x1.z * w23 + x2.z * w31) + x3.z * w12);
    const float d_in = dist3(x0, p);
    const bool c23 = w23 > 0.0f, c31 = !c23 && (w31 > 0.0f);
    const f3 fa = x1;                         // first segment (fa, fb)
    const f3 fb = (c23 || c31) ? x2 : x3;
    const f3 sa = (c23) ? x1 : x2;            // second segment (sa, x3)
    const float first = psd(x0, fa, fb);
    const float second = psd(x0, sa, x3);
    const float d_edge = fmin_std(first, second);
    return inside ? d_in : d_edge;
}

// The triangle-only reciprocal of ptd's barycentric solve, exactly as ptd computes it.  The
// device kernels take it precomputed (k_prep_soup stores it in the third vertex's w), which
// takes a division off every distance's dependency chain.
SDF_HD float tri_invdet(f3 x1, f3 x2, f3 x3)
{
    const f3 x13 = sub3(x1, x3), x23 = sub3(x2, x3);
    const float m13 = mag2(x13), m23 = mag2(x23), d = dot3(x13, x23);
    return div_rn(1.0f, fmax_std(m13 * m23 - d * d, 1e-30f));
}

// Two point-triangle distances per lane in packed FP32 (v_pk_mul_f32 / v_pk_add_f32: each
// half is an IEEE single operation with round-to-nearest, exactly the scalar op), so a lane
// that owns two (cell, candidate) pairs evaluates both in one pass.  Division, sqrt, compares
// and selects stay scalar per half.  Bit-identical to ptd_nb for each pair.
typedef float f2v __attribute__((ext_vector_type(2)));
struct f3x2 {
    f2v x, y, z;
};
__device__ __forceinline__ f3x2 mk3x2(f3 a, f3 b) { return f3x2{f2v{a.x, b.x}, f2v{a.y, b.y}, f2v{a.z, b.z}}; }
__device__ __forceinline__ f3x2 sub3x2(f3x2 a, f3x2 b) { return f3x2{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f2v mag2x2(f3x2 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
__device__ __forceinline__ f2v dot3x2(f3x2 a, f3x2 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f2v sel2(bool c0, bool c1, f2v a, f2v b) { return f2v{c0 ? a.x : b.x, c1 ? a.y : b.y}; }
__device__ __forceinline__ f3x2 sel3x2(bool c0, bool c1, f3x2 a, f3x2 b)
{
    return f3x2{sel2(c0, c1, a.x, b.x), sel2(c0, c1, a.y, b.y), sel2(c0, c1, a.z, b.z)};
}
__device__ __forceinline__ f2v sqrt2(f2v v) { return f2v{sqrt_rn(v.x), sqrt_rn(v.y)}; }
__device__ __forceinline__ f2v dist3x2(f3x2 a, f3x2 b)
{
    const f3x2 d = sub3x2(a, b);
    return sqrt2((d.x * d.x + d.y * d.y) + d.z * d.z);
}
__device__ __forceinline__ f2v psd2(f3x2 x0, f3x2 x1, f3x2 x2)
{
    const f3x2 e = sub3x2(x2, x1);
    const f2v m2 = mag2x2(e);
    const f3x2 t = sub3x2(x2, x0);
    const f2v dt = dot3x2(t, e);
    // (float)((double)dt / (double)m2) == the IEEE float division dt / m2
    f2v s12 = f2v{(float)((double)dt.x / (double)m2.x), (float)((double)dt.y / (double)m2.y)};
    s12.x = (s12.x < 0.0f) ? 0.0f : ((s12.x > 1.0f) ? 1.0f : s12.x);
    s12.y = (s12.y < 0.0f) ? 0.0f : ((s12.y > 1.0f) ? 1.0f : s12.y);
    const f2v w = 1.0f - s12;
    const f3x2 p = f3x2{x1.x * s12 + x2.x * w, x1.y * s12 + x2.y * w, x1.z * s12 + x2.z * w};
    const f3x2 d = sub3x2(x0, p);
    return (d.x * d.x + d.y * d.y) + d.z * d.z;   // squared (see ptd_wave: one sqrt at the end)
}

// ptd_nb for a wave evaluating many (point, triangle) pairs at once: the inside-projection
// block and the two-segment block each run only if some active lane needs it (wave-uniform
// branches).  Every lane still performs exactly ptd_nb's operations for the case it takes,
// so the result is bit-identical; away from the surface (points project outside the tiny
// triangles) whole waves skip the inside block.
// ONE point-triangle distance per lane, with the independent halves of its arithmetic paired in
// packed FP32: (x13 | x23), (m13 | m23), (a | b), (w23 | w31), the inside point's (x | y), and the
// two edge distances (first | second segment) as one psd2.  Every half performs exactly ptd_nb's
// operation on the same operands, so the bits are ptd_nb's; the step's chain of one evaluation is
// 168 instead of 211 VALU (gfx950 ISA).
__device__ __forceinline__ float ptd_wave(f3 x0, f3 x1, f3 x2, f3 x3, float invdet)
{
    const f3x2 X = sub3x2(mk3x2(x1, x2), mk3x2(x3, x3));      // {x13, x23}
    const f3x2 X03 = sub3x2(mk3x2(x0, x0), mk3x2(x3, x3));    // {x03, x03}
    const f2v M = mag2x2(X);                                  // {m13, m23}
    const float d = dot3(f3{X.x.x, X.y.x, X.z.x}, f3{X.x.y, X.y.y, X.z.y});   // dot(x13, x23)
    const f2v AB = dot3x2(X, X03);                            // {a, b}
    const f2v T = f2v{M.y, M.x} * AB - f2v{d, d} * f2v{AB.y, AB.x};   // {m23 a - d b, m13 b - d a}
    const f2v W = f2v{invdet, invdet} * T;                    // {w23, w31}
    const float w23 = W.x, w31 = W.y;
    const float w12 = (1.0f - w23) - w31;
    const bool inside = (w23 >= 0.0f) & (w31 >= 0.0f) & (w12 >= 0.0f);
    // One sqrt for all branches: the reference returns sqrt(inside) or min(sqrt(e1), sqrt(e2));
    // a correctly rounded sqrt is monotone, so min(sqrt(e1), sqrt(e2)) == sqrt(min(e1, e2)) bit
    // for bit (with std::min's argument order, NaN included; squared sums are never -0).
    float r2 = 0.0f;
    if (__any(inside)) {
        const f2v pxy = (f2v{x1.x, x1.y} * w23 + f2v{x2.x, x2.y} * w31) + f2v{x3.x, x3.y} * w12;
        const float pz = (x1.z * w23 + x2.z * w31) + x3.z * w12;
        const f2v dxy = f2v{x0.x, x0.y} - pxy;
        const float dz = x0.z - pz;
        const f2v sq = dxy * dxy;
        r2 = (sq.x + sq.y) + dz * dz;
    }
    if (__any(!inside)) {
        const bool c23 = w23 > 0.0f, c31 = !c23 & (w31 > 0.0f);
        const f3 fb = (c23 | c31) ? x2 : x3;
        const f3 sa = c23 ? x1 : x2;
        const f2v e = psd2(mk3x2(x0, x0), mk3x2(x1, sa), mk3x2(fb, x3));   // {psd(x1, fb), psd(sa, x3)}
        r2 = inside ? r2 : fmin_std(e.x, e.y);
    }
    return sqrt_rn(r2);
}
__device__ __forceinline__ void ptd_wave2(f3 x0a, f3 x1a, f3 x2a, f3 x3a, float inva, f3 x0b, f3 x1b, f3 x2b, f3 x3b,
                                          float invb, float &da, float &db)
{
    const f3x2 x0 = mk3x2(x0a, x0b), x1 = mk3x2(x1a, x1b), x2 = mk3x2(x2a, x2b), x3 = mk3x2(x3a, x3b);
    const f3x2 x13 = sub3x2(x1, x3), x23 = sub3x2(x2, x3), x03 = sub3x2(x0, x3);
    const f2v m13 = mag2x2(x13), m23 = mag2x2(x23), d = dot3x2(x13, x23);
    const f2v invdet = f2v{inva, invb};   // tri_invdet of each triangle
    const f2v a = dot3x2(x13, x03), b = dot3x2(x23, x03);
    const f2v w23 = invdet * (m23 * a - d * b);
    const f2v w31 = invdet * (m13 * b - d * a);
    const f2v w12 = (1.0f - w23) - w31;
    const bool ia = (w23.x >= 0.0f) & (w31.x >= 0.0f) & (w12.x >= 0.0f);
    const bool ib = (w23.y >= 0.0f) & (w31.y >= 0.0f) & (w12.y >= 0.0f);
    f2v r = f2v{0.0f, 0.0f};   // squared distances until the end (see ptd_wave)
    if (__any(ia | ib)) {
        const f3x2 p = f3x2{(x1.x * w23 + x2.x * w31) + x3.x * w12, (x1.y * w23 + x2.y * w31) + x3.y * w12,
                            (x1.z * w23 + x2.z * w31) + x3.z * w12};
        const f3x2 dd = sub3x2(x0, p);
        r = (dd.x * dd.x + dd.y * dd.y) + dd.z * dd.z;
    }
    if (__any(!ia | !ib)) {
        const bool c23a = w23.x > 0.0f, c31a = !c23a & (w31.x > 0.0f);
        const bool c23b = w23.y > 0.0f, c31b = !c23b & (w31.y > 0.0f);
        const f3x2 fb = sel3x2(c23a | c31a, c23b | c31b, x2, x3);
        const f3x2 sa = sel3x2(c23a, c23b, x1, x2);
        const f2v first = psd2(x0, x1, fb), second = psd2(x0, sa, x3);
        const f2v de = f2v{fmin_std(first.x, second.x), fmin_std(first.y, second.y)};
        r = sel2(ia, ib, r, de);
    }
    da = sqrt_rn(r.x);
    db = sqrt_rn(r.y);
}

// orientation (SOS-robust 2D), FP64.
SDF_HD int orientation(double x1, double y1, double x2, double y2, double &area)
{
    area = y1 * x2 - x1 * y2;
    if (area > 0) return 1;
    if (area < 0) return -1;
    if (y2 > y1) return 1;
    if (y2 < y1) return -1;
    if (x1 > x2) return 1;
    if (x1 < x2) return -1;
    return 0;
}

SDF_HD bool pit2d(double x0, double y0, double x1, double y1, double x2, double y2,
                                      double x3, double y3, double &a, double &b, double &c)
{
    x1 -= x0; x2 -= x0; x3 -= x0;
    y1 -= y0; y2 -= y0; y3 -= y0;
    int sa = orientation(x2, y2, x3, y3, a);
    if (sa == 0) return false;
    int sb = orientation(x3, y3, x1, y1, b);
    if (sb != sa) return false;
    int sc = orientation(x1, y1, x2, y2, c);
    if (sc != sa) return false;
    double sum = (a + b) + c;
    a /= sum;
    b /= sum;
    c /= sum;
    return true;
}

}  // namespace sdfhip
