// oracle/mesh_ref_shim.cpp -- extern "C" wrapper around the REFERENCE mesh loaders.
//
// TEST INFRASTRUCTURE ONLY, built only in the development container: oracle/Makefile target
// `ref` compiles the reference's own common/mesh_io.cpp, mesh_io_obj.cpp and mesh_io_stl.cpp
// where they lie under /root/reference (with the reference's headers, Release flags) into
// oracle/_ref/libmeshref.so.  It pins the library's native loaders (sdfgenfast_amd/csrc/
// meshio.cpp) to the reference: tests/test_meshio_ref.py compares them bit for bit and
// tests/golden/make_meshio_golden.py commits the reference's digests as fixtures.
#include "mesh_io.h"   // resolved with -I$(REF)/common

#include <cstdint>
#include <cstring>
#include <iostream>
#include <sstream>
#include <vector>

struct ref_mesh {
    std::vector<Vec3f> v;
    std::vector<Vec3ui> t;
    Vec3f lo, hi;
    std::string log;   // what the loader printed (cout + cerr), for diagnostics
};

extern "C" {

// meshio::load_mesh (common/mesh_io.cpp:29-48). Returns 1 when the reference returns true, 0 when
// it returns false, 2 when it throws (std::stoi on a bad OBJ face token, mesh_io_obj.cpp:104, is
// not caught by the reference; its Python binding turns that into an exception).
// *out is always set (free with ref_mesh_free).
int ref_mesh_load(const char* path, ref_mesh** out)
{
    ref_mesh* m = new ref_mesh();
    std::ostringstream sink;
    std::streambuf* so = std::cout.rdbuf(sink.rdbuf());
    std::streambuf* se = std::cerr.rdbuf(sink.rdbuf());
    int rc;
    try {
        rc = meshio::load_mesh(path, m->v, m->t, m->lo, m->hi) ? 1 : 0;
    } catch (const std::exception& e) {
        sink << "EXCEPTION: " << e.what() << "\n";
        rc = 2;
    }
    std::cout.rdbuf(so);
    std::cerr.rdbuf(se);
    m->log = sink.str();
    *out = m;
    return rc;
}

void ref_mesh_info(const ref_mesh* m, uint64_t* nvert, uint64_t* ntri, float bounds[6])
{
    *nvert = m->v.size();
    *ntri = m->t.size();
    for (int c = 0; c < 3; ++c) {
        bounds[c] = m->lo[c];
        bounds[3 + c] = m->hi[c];
    }
}

void ref_mesh_copy(const ref_mesh* m, float* xyz, uint32_t* tri)
{
    for (size_t q = 0; q < m->v.size(); ++q)
        for (int c = 0; c < 3; ++c) xyz[3 * q + c] = m->v[q][c];
    for (size_t q = 0; q < m->t.size(); ++q)
        for (int c = 0; c < 3; ++c) tri[3 * q + c] = m->t[q][c];
}

const char* ref_mesh_log(const ref_mesh* m) { return m->log.c_str(); }

void ref_mesh_free(ref_mesh* m) { delete m; }

}  // extern "C"
