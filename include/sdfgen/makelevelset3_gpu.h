// sdfgen/makelevelset3_gpu.h -- the GPU backend entry point, same declaration as the
// reference's /root/reference/gpu_lib/makelevelset3_gpu.h:40-42 (sdfgen::gpu::make_level_set3).
// Exported by libsdfgen_hip.so and served by the hand-written gfx950 kernels through
// sdfgen_hip_make_level_set3 (include/sdfgen_hip.h) on the current device.  Unlike the
// reference (gpu_lib/makelevelset3_gpu.cu:14-20, exit() on a CUDA error) it throws:
// std::invalid_argument / std::out_of_range for bad arguments, std::runtime_error naming
// the GPU otherwise.  Results are the reference CPU path's bits, not the reference CUDA's.
#pragma once
#include <vector>

#include "array3.h"
#include "vec.h"

#pragma GCC visibility push(default)
namespace sdfgen {
namespace gpu {
void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, const int exact_band = 1);
}  // namespace gpu
}  // namespace sdfgen
#pragma GCC visibility pop
