// sdfgen_unified.cpp -- sdfgen::make_level_set3 / is_gpu_available on top of the C-ABIs.
// Mirrors /root/reference/common/sdfgen_unified.cpp:19-71 (dispatch), with the
// GPU case served by sdfgen_hip_make_level_set3 and errors thrown instead of exit().
#include "sdfgen/sdfgen_unified.h"

#include <stdexcept>
#include <string>

#include "sdfgen_cpu.h"
#include "sdfgen_hip.h"

namespace sdfgen {

bool is_gpu_available() { return sdfgen_hip_device_count() > 0; }

static void throw_for(int rc, const char *msg)
{
    std::string m(msg && *msg ? msg : "SDF generation failed");
    if (rc == SDFGEN_HIP_EINVAL) throw std::invalid_argument(m);
    if (rc == SDFGEN_HIP_EINDEX) throw std::out_of_range(m);
    throw std::runtime_error(m);
}

void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, int exact_band, HardwareBackend backend, int num_threads)
{
    if (backend == HardwareBackend::Auto) backend = is_gpu_available() ? HardwareBackend::GPU : HardwareBackend::CPU;
    if (nx <= 0 || ny <= 0 || nz <= 0) throw std::invalid_argument("Grid dimensions must be positive");
    phi.resize(nx, ny, nz);
    char err[512] = {0};
    const float o[3] = {origin[0], origin[1], origin[2]};
    const uint32_t *t = tri.empty() ? nullptr : reinterpret_cast<const uint32_t *>(tri.data());
    const float *v = x.empty() ? nullptr : reinterpret_cast<const float *>(x.data());
    int rc;
    if (backend == HardwareBackend::GPU) {
        if (!is_gpu_available())
            throw std::runtime_error("GPU backend requested but no HIP GPU is available. Use HardwareBackend::CPU.");
        rc = sdfgen_hip_make_level_set3(t, tri.size(), v, x.size(), o, dx, nx, ny, nz, exact_band, 0,
                                        SDFGEN_LAYOUT_ARRAY3, phi.data(), err, sizeof(err));
    } else {
        rc = sdfgen_cpu_make_level_set3(t, tri.size(), v, x.size(), o, dx, nx, ny, nz, exact_band, num_threads, 0,
                                        phi.data(), err, sizeof(err));
    }
    if (rc != 0) throw_for(rc, err);
}

}  // namespace sdfgen
