// integration/makelevelset3_gpu_shim.cpp -- drop-in replacement for the reference's
// gpu_lib/makelevelset3_gpu.cu that calls ONLY the C-ABI (include/sdfgen_hip.h).
//
// For a maintainer who keeps the reference's own headers and dispatcher
// (common/sdfgen_unified.cpp:30-71) and swaps the CUDA translation unit for this file:
// compile it with -I gpu_lib -I common -I <this repo>/include, define HAVE_CUDA (the
// dispatcher's "GPU backend compiled in" switch, config.h.in:9) and link
// libsdfgen_hip.so.  (libsdfgen_hip.so also exports sdfgen::gpu::make_level_set3 itself, so
// linking the library in place of gpu_lib works without this file)
// tests/test_cxx_dropin.py compiles this file against /root/reference's headers.
#include <cstdint>
#include <stdexcept>
#include <string>

#include "makelevelset3_gpu.h"  // reference gpu_lib/makelevelset3_gpu.h:40-42
#include "sdfgen_hip.h"

namespace sdfgen {
namespace gpu {

void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, const int exact_band)
{
    if (nx <= 0 || ny <= 0 || nz <= 0) throw std::invalid_argument("Grid dimensions must be positive");
    phi.resize(nx, ny, nz);  // Array3f = Array3<float, Array1<float>>, i fastest; storage phi.a.data
    const float o[3] = {origin[0], origin[1], origin[2]};
    char err[512] = {0};
    const int rc = sdfgen_hip_make_level_set3(
        tri.empty() ? nullptr : reinterpret_cast<const uint32_t *>(tri.data()), tri.size(),  // Vec3ui: packed 12 B
        x.empty() ? nullptr : reinterpret_cast<const float *>(x.data()), x.size(),           // Vec3f: packed 12 B
        o, dx, nx, ny, nz, exact_band, SDFGEN_NGPU_CURRENT, SDFGEN_LAYOUT_ARRAY3, phi.a.data, err, sizeof err);
    if (rc == SDFGEN_HIP_EINVAL) throw std::invalid_argument(err);
    if (rc == SDFGEN_HIP_EINDEX) throw std::out_of_range(err);
    if (rc != SDFGEN_HIP_OK) throw std::runtime_error(std::string("GPU: ") + err);
}

}  // namespace gpu
}  // namespace sdfgen
