/*
 * sdfgen_meshio.h -- C-ABI of the library's native mesh loaders (OBJ, binary / ASCII STL).
 *
 * Replaces meshio::load_mesh / load_obj / load_stl (/root/reference/common/mesh_io.h:29-80,
 * common/mesh_io.cpp:29-48, common/mesh_io_obj.cpp:21-157, common/mesh_io_stl.cpp:42-303) --
 * the input side of make_level_set3.  Same line grammar, same vertex
 * and face lists, same float bits (correctly rounded decimal conversion) and the same bounds
 * (update_minmax in file order) as the reference; the file is read at once and OBJ is parsed
 * in parallel chunks.  Binary STL keeps the reference's 3 vertices per facet (no merging).
 * Errors are return codes with a message, never exceptions or exit().
 */
#ifndef SDFGEN_MESHIO_H
#define SDFGEN_MESHIO_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

enum { SDFGEN_MESH_OK = 0, SDFGEN_MESH_EINVAL = -1, SDFGEN_MESH_EIO = -6, SDFGEN_MESH_EFORMAT = -7 };
/* format: AUTO = by extension (.obj / .stl, case-insensitive), STL = binary or ASCII detected as
 * mesh_io_stl.cpp:42-92 does; the reported format is OBJ, STL_BINARY or STL_ASCII. */
enum { SDFGEN_MESH_AUTO = 0, SDFGEN_MESH_OBJ = 1, SDFGEN_MESH_STL = 2, SDFGEN_MESH_STL_BINARY = 3,
       SDFGEN_MESH_STL_ASCII = 4 };

typedef struct sdfgen_mesh sdfgen_mesh;
int sdfgen_mesh_load(const char *path, int format, sdfgen_mesh **out, char *errbuf, size_t errlen);
/* bounds: min x, y, z then max x, y, z (FLT_MAX / -FLT_MAX when never updated) */
int sdfgen_mesh_info(const sdfgen_mesh *m, uint64_t *nvert, uint64_t *ntri, float bounds[6], int *format);
/* xyz: nvert x 3 floats, tri: ntri x 3 uint32 (either may be NULL) */
int sdfgen_mesh_copy(const sdfgen_mesh *m, float *xyz, uint32_t *tri);
int sdfgen_mesh_free(sdfgen_mesh *m);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
