// oracle/ref_shim.cpp -- extern "C" wrapper around the REFERENCE CPU implementation.
//
// TEST INFRASTRUCTURE ONLY, built only in the development container (the GPU box
// has no /root/reference; the built .so travels with the tree and bench.py's
// cpu_baseline leg times it there -- the reference's multi-threaded CPU path, a
// timing baseline, never a checker of GPU results on the box): oracle/Makefile compiles
// the reference's own cpu_lib/makelevelset3.cpp where it lies under
// /root/reference (it is #included below so that its file-static helpers
// point_triangle_distance / point_in_triangle_2d are reachable) with the
// reference's Release flags (-O3 -DNDEBUG -std=c++11 -fPIC), and writes only
// to oracle/_ref/.  It exists to pin oracle/sdf_oracle.c and to generate the
// golden fixtures in tests/golden/ (tests/golden/make_golden.py).
#include "makelevelset3.cpp"   // resolved with -I$(REF)/cpu_lib
#include <cstdint>

extern "C" {

// sdfgen::cpu::make_level_set3 (cpu_lib/makelevelset3.cpp:192) -> phi in Array3f (i-fastest) order.
int ref_make_level_set3(const uint32_t* tri, uint64_t ntri, const float* x, uint64_t nvert,
                        const float origin[3], float dx, int ni, int nj, int nk,
                        int exact_band, int num_threads, float* phi_out)
{
    std::vector<Vec3ui> t(ntri);
    std::vector<Vec3f> v(nvert);
    for (uint64_t q = 0; q < ntri; ++q) t[q] = Vec3ui(tri[3*q], tri[3*q+1], tri[3*q+2]);
    for (uint64_t q = 0; q < nvert; ++q) v[q] = Vec3f(x[3*q], x[3*q+1], x[3*q+2]);
    Array3f phi;
    sdfgen::cpu::make_level_set3(t, v, Vec3f(origin[0], origin[1], origin[2]), dx, ni, nj, nk,
                                 phi, exact_band, num_threads);
    std::copy(phi.a.begin(), phi.a.end(), phi_out);
    return 0;
}

// point_triangle_distance (cpu_lib/makelevelset3.cpp:49): pts = n x (x0,x1,x2,x3).
void ref_ptd_batch(uint64_t n, const float* pts, float* out)
{
    for (uint64_t q = 0; q < n; ++q) {
        const float* p = pts + 12*q;
        out[q] = point_triangle_distance(Vec3f(p), Vec3f(p+3), Vec3f(p+6), Vec3f(p+9));
    }
}

// point_in_triangle_2d (cpu_lib/makelevelset3.cpp:169): in = n x 8 doubles, out = n x (flag,a,b,c).
void ref_pit2d_batch(uint64_t n, const double* in, double* out)
{
    for (uint64_t q = 0; q < n; ++q) {
        const double* p = in + 8*q;
        double a = 0, b = 0, c = 0;
        bool r = point_in_triangle_2d(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], a, b, c);
        out[4*q] = r ? 1.0 : 0.0; out[4*q+1] = a; out[4*q+2] = b; out[4*q+3] = c;
    }
}

} // extern "C"
