// sdfgen/sdfgen_unified.h -- C++ drop-in for the reference's unified API.
//
// Same declarations as /root/reference/common/sdfgen_unified.h:16-20, 47-57, 68, over
// types with the reference's names, template parameters and data layout (vec.h, array1.h,
// array3.h here): a reference caller (python/sdfgen_py.cpp:206-214, app/main.cpp:273,
// tests/test_utils.cpp:27) compiled against EITHER this header or the reference's own
// common/sdfgen_unified.h links to libsdfgen_hip.so unchanged -- the exported symbol is
// the reference's mangled name (tests/test_cxx_dropin.py builds such callers).
//   Auto -> GPU when a HIP device is visible, else CPU (common/sdfgen_unified.cpp:42-48)
//   GPU  -> hand-written gfx950 kernels via include/sdfgen_hip.h; throws
//           std::runtime_error mentioning "GPU" when no device is usable
//   CPU  -> the native deterministic multi-threaded backend (include/sdfgen_cpu.h)
// Errors throw (std::invalid_argument for bad arguments, std::out_of_range for a
// bad triangle index, std::runtime_error otherwise); nothing calls exit().
#pragma once
#include <vector>

#include "array3.h"
#include "vec.h"

#pragma GCC visibility push(default)  // exported from libsdfgen_hip.so (built -fvisibility=hidden)
namespace sdfgen {

enum class HardwareBackend { Auto, CPU, GPU };

void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, int exact_band = 1,
                     HardwareBackend backend = HardwareBackend::Auto, int num_threads = 0);

bool is_gpu_available();

}  // namespace sdfgen
#pragma GCC visibility pop
