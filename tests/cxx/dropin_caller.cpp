// tests/cxx/dropin_caller.cpp -- a C++ caller of the drop-in boundary, written the way the
// reference's own callers are (tests/test_utils.cpp:16-30 generate_sdf_with_timing,
// app/main.cpp:260-273): std::vector<Vec3ui>/std::vector<Vec3f> mesh, an Array3f the
// caller owns, sdfgen::make_level_set3(..., phi, 1, backend).
//
// It is compiled by tests/test_cxx_dropin.py against EITHER header set, unchanged:
//   -I /root/reference/common   (the reference's sdfgen_unified.h / array3.h / vec.h;
//                                build container only -- proves the exported symbol and
//                                the Array3f layout are the reference's)
//   -I include/sdfgen           (this repository's restatement; built by
//                                __graft_entry__.build(), travels to the GPU box)
// and linked against libsdfgen_hip.so only (no reference library).
//
// usage: dropin_caller <mesh.bin> <cpu|gpu|auto|cpu-direct|gpu-direct> <out.bin>
//   cpu/gpu/auto: sdfgen::make_level_set3 with that HardwareBackend;
//   cpu-direct / gpu-direct: sdfgen::cpu:: / sdfgen::gpu::make_level_set3 (the per-backend
//   entry points the reference's dispatcher calls, common/sdfgen_unified.cpp:57-63)
//   mesh.bin: int32 ntri, int32 nvert, int32 ni, nj, nk, int32 exact_band, float origin[3],
//             float dx, uint32 tri[ntri][3], float xyz[nvert][3]
//   out.bin : float phi[ni*nj*nk], i fastest (Array3f's own storage order)
// usage: dropin_caller --errors     (error contract checks, no compute on a GPU)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "makelevelset3.h"      // sdfgen::cpu (cpu_lib/makelevelset3.h:39-41)
#include "makelevelset3_gpu.h"  // sdfgen::gpu (gpu_lib/makelevelset3_gpu.h:40-42)
#include "sdfgen_unified.h"

static int fail(const char *what)
{
    std::fprintf(stderr, "dropin_caller: %s\n", what);
    return 2;
}

static int error_contract()
{
    std::vector<Vec3f> x;
    x.push_back(Vec3f(0.f, 0.f, 0.f));
    x.push_back(Vec3f(1.f, 0.f, 0.f));
    x.push_back(Vec3f(0.f, 1.f, 0.f));
    std::vector<Vec3ui> tri;
    tri.push_back(Vec3ui(0, 1, 2));
    Array3f phi;
    const Vec3f origin(-0.5f, -0.5f, -0.5f);
    // Non-positive dims -> std::invalid_argument (python/sdfgen_py.cpp:171-182 semantics).
    try {
        sdfgen::make_level_set3(tri, x, origin, 0.25f, 0, 4, 4, phi, 1, sdfgen::HardwareBackend::CPU);
        return fail("dims <= 0 did not throw");
    } catch (const std::invalid_argument &) {
    }
    // A triangle index past the vertex list -> an exception (the reference reads out of bounds).
    tri.push_back(Vec3ui(0, 1, 7));
    try {
        sdfgen::make_level_set3(tri, x, origin, 0.25f, 4, 4, 4, phi, 1, sdfgen::HardwareBackend::CPU);
        return fail("bad triangle index did not throw");
    } catch (const std::exception &) {
    }
    tri.pop_back();
    // GPU requested without a device -> std::runtime_error naming the GPU.
    if (!sdfgen::is_gpu_available()) {
        try {
            sdfgen::make_level_set3(tri, x, origin, 0.25f, 4, 4, 4, phi, 1, sdfgen::HardwareBackend::GPU);
            return fail("GPU without a device did not throw");
        } catch (const std::runtime_error &e) {
            if (std::string(e.what()).find("GPU") == std::string::npos) return fail("GPU error lacks 'GPU'");
        }
    }
    // The library resizes a caller-allocated, differently sized Array3f (shrink and grow).
    Array3f big(9, 9, 9, 7.f);
    sdfgen::make_level_set3(tri, x, origin, 0.25f, 4, 4, 4, big, 1, sdfgen::HardwareBackend::CPU);
    if (big.ni != 4 || big.nj != 4 || big.nk != 4 || big.a.size() != 64) return fail("resize (shrink) wrong");
    Array3f small(1, 1, 1, 7.f);
    sdfgen::make_level_set3(tri, x, origin, 0.25f, 5, 6, 7, small, 1, sdfgen::HardwareBackend::CPU);
    if (small.ni != 5 || small.nj != 6 || small.nk != 7 || small.a.size() != 210) return fail("resize (grow) wrong");
    if (!(small(4, 5, 6) > 0.f)) return fail("far corner not outside");
    std::printf("errors: ok (gpu_available=%d)\n", (int)sdfgen::is_gpu_available());
    return 0;
}

int main(int argc, char **argv)
{
    if (argc == 2 && std::strcmp(argv[1], "--errors") == 0) return error_contract();
    if (argc != 4) return fail("usage: dropin_caller <mesh.bin> <cpu|gpu|auto|cpu-direct|gpu-direct> <out.bin>");
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return fail("cannot open mesh");
    int32_t hdr[6];
    float of[4];
    if (std::fread(hdr, 4, 6, f) != 6 || std::fread(of, 4, 4, f) != 4) return fail("short header");
    const int ntri = hdr[0], nvert = hdr[1], ni = hdr[2], nj = hdr[3], nk = hdr[4], band = hdr[5];
    std::vector<Vec3ui> tri(ntri);
    std::vector<Vec3f> x(nvert);
    if (std::fread(tri.data(), 12, ntri, f) != (size_t)ntri || std::fread(x.data(), 12, nvert, f) != (size_t)nvert)
        return fail("short mesh");
    std::fclose(f);

    sdfgen::HardwareBackend backend = sdfgen::HardwareBackend::Auto;
    if (std::strcmp(argv[2], "cpu") == 0) backend = sdfgen::HardwareBackend::CPU;
    else if (std::strcmp(argv[2], "gpu") == 0) backend = sdfgen::HardwareBackend::GPU;

    Array3f phi;  // caller-owned; the callee resizes it (cpu_lib/makelevelset3.cpp:196)
    try {
        const Vec3f origin(of[0], of[1], of[2]);
        if (std::strcmp(argv[2], "cpu-direct") == 0)
            sdfgen::cpu::make_level_set3(tri, x, origin, of[3], ni, nj, nk, phi, band, 3);
        else if (std::strcmp(argv[2], "gpu-direct") == 0)
            sdfgen::gpu::make_level_set3(tri, x, origin, of[3], ni, nj, nk, phi, band);
        else
            sdfgen::make_level_set3(tri, x, origin, of[3], ni, nj, nk, phi, band, backend);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "dropin_caller: make_level_set3 threw: %s\n", e.what());
        return 3;
    }
    if (phi.ni != ni || phi.nj != nj || phi.nk != nk) return fail("phi has the wrong dims");
    FILE *o = std::fopen(argv[3], "wb");
    if (!o) return fail("cannot open output");
    const size_t n = (size_t)ni * nj * nk;
    if (std::fwrite(&phi.a[0], 4, n, o) != n) return fail("short write");
    std::fclose(o);
    std::printf("ok %dx%dx%d backend=%s gpu_available=%d\n", ni, nj, nk, argv[2], (int)sdfgen::is_gpu_available());
    return 0;
}
