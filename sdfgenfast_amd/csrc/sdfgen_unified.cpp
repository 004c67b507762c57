// sdfgen_unified.cpp -- the reference's C++ entry points on top of the C-ABIs:
//   sdfgen::make_level_set3 / is_gpu_available   common/sdfgen_unified.h:47-57, 68 (dispatch
//                                                 as common/sdfgen_unified.cpp:19-71)
//   sdfgen::gpu::make_level_set3                  gpu_lib/makelevelset3_gpu.h:40-42
//   sdfgen::cpu::make_level_set3                  cpu_lib/makelevelset3.h:39-41
// The GPU case is served by sdfgen_hip_make_level_set3 (hand-written gfx950 kernels), the
// CPU case by sdfgen_cpu_make_level_set3; errors are thrown, never exit().  The types are the
// reference's (include/sdfgen/{vec,array1,array3}.h), so these four symbols are the ones a
// reference caller's object files import.
#include "sdfgen/sdfgen_unified.h"

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "sdfgen/makelevelset3.h"
#include "sdfgen/makelevelset3_gpu.h"
#include "sdfgen_cpu.h"
#include "sdfgen_hip.h"

namespace sdfgen {

bool is_gpu_available() { return sdfgen_hip_device_count() > 0; }

namespace {

void throw_for(int rc, const char *msg)
{
    std::string m(msg && *msg ? msg : "SDF generation failed");
    if (rc == SDFGEN_HIP_EINVAL) throw std::invalid_argument(m);
    if (rc == SDFGEN_HIP_EINDEX) throw std::out_of_range(m);
    throw std::runtime_error(m);
}

// Validate dims and size the caller's Array3f (the callee resizes it, cpu_lib/makelevelset3.cpp:196).
void prepare(int nx, int ny, int nz, Array3f &phi)
{
    if (nx <= 0 || ny <= 0 || nz <= 0) throw std::invalid_argument("Grid dimensions must be positive");
    phi.resize(nx, ny, nz);
}

// The GPU-count knob of the drop-in (Config row): the reference's signatures have no
// device argument (common/sdfgen_unified.h:47-57), so SDFGEN_NGPU picks the devices -- unset or "1": the
// current device (the reference's behaviour, gpu_lib/makelevelset3_gpu.cu:600-603); "all" or "0": every
// visible device; n > 1: devices 0..n-1, the grid split into Z-slabs.  Anything else
// is a std::invalid_argument.
int ngpu_from_env()
{
    const char *e = std::getenv("SDFGEN_NGPU");
    if (!e || !*e) return SDFGEN_NGPU_CURRENT;
    if (std::strcmp(e, "all") == 0) return SDFGEN_NGPU_ALL;
    char *end = nullptr;
    const long n = std::strtol(e, &end, 10);
    if (end == e || *end != 0 || n < 0 || n > 4096)
        throw std::invalid_argument(std::string("SDFGEN_NGPU = '") + e + "' (expected 'all', 0, 1 or a device count)");
    return (int)n;
}

const uint32_t *tri_ptr(const std::vector<Vec3ui> &tri)
{
    return tri.empty() ? nullptr : reinterpret_cast<const uint32_t *>(tri.data());  // packed uint32[n][3]
}
const float *xyz_ptr(const std::vector<Vec3f> &x)
{
    return x.empty() ? nullptr : reinterpret_cast<const float *>(x.data());  // packed float[n][3]
}

}  // namespace

namespace gpu {
void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, const int exact_band)
{
    if (!is_gpu_available())
        throw std::runtime_error("GPU backend requested but no HIP GPU is available. Use HardwareBackend::CPU.");
    prepare(nx, ny, nz, phi);
    char err[512] = {0};
    const float o[3] = {origin[0], origin[1], origin[2]};
    const int rc = sdfgen_hip_make_level_set3(tri_ptr(tri), tri.size(), xyz_ptr(x), x.size(), o, dx, nx, ny, nz,
                                              exact_band, ngpu_from_env(), SDFGEN_LAYOUT_ARRAY3, phi.a.data, err,
                                              sizeof(err));
    if (rc != 0) throw_for(rc, err);
}
}  // namespace gpu

namespace cpu {
void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, const int exact_band, int num_threads)
{
    prepare(nx, ny, nz, phi);
    char err[512] = {0};
    const float o[3] = {origin[0], origin[1], origin[2]};
    const int rc = sdfgen_cpu_make_level_set3(tri_ptr(tri), tri.size(), xyz_ptr(x), x.size(), o, dx, nx, ny, nz,
                                              exact_band, num_threads, SDFGEN_LAYOUT_ARRAY3, phi.a.data, err,
                                              sizeof(err));
    if (rc != 0) throw_for(rc, err);
}
}  // namespace cpu

void make_level_set3(const std::vector<Vec3ui> &tri, const std::vector<Vec3f> &x, const Vec3f &origin, float dx,
                     int nx, int ny, int nz, Array3f &phi, int exact_band, HardwareBackend backend, int num_threads)
{
    if (backend == HardwareBackend::Auto) backend = is_gpu_available() ? HardwareBackend::GPU : HardwareBackend::CPU;
    if (backend == HardwareBackend::GPU) gpu::make_level_set3(tri, x, origin, dx, nx, ny, nz, phi, exact_band);
    else cpu::make_level_set3(tri, x, origin, dx, nx, ny, nz, phi, exact_band, num_threads);
}

}  // namespace sdfgen
