// sdfgen/makelevelset3.h -- the CPU backend entry point, same declaration as the
// reference's /root/reference/cpu_lib/makelevelset3.h:39-41 (sdfgen::cpu::make_level_set3).
// Exported by libsdfgen_hip.so and served by the library's native deterministic CPU backend
// (include/sdfgen_cpu.h): bit-identical to the reference's single-threaded run for any
// num_threads (the reference's k-split sweep races).
#pragma once
#include <vector>

#include "array3.h"
#include "vec.h"

#pragma GCC visibility push(default)
namespace sdfgen {
namespace cpu {
void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, const int exact_band = 1, int num_threads = 0);
}  // namespace cpu
}  // namespace sdfgen
#pragma GCC visibility pop
