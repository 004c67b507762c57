/*
 * sdfgen_cpu.h -- C-ABI of the library's native CPU backend (HardwareBackend::CPU).
 *
 * Replaces sdfgen::cpu::make_level_set3 (/root/reference/cpu_lib/makelevelset3.h:39-41,
 * cpu_lib/makelevelset3.cpp:192-304).  Same results as the reference's
 * single-threaded run for ANY num_threads (the reference's k-split sweep races
 * and its output depends on the thread count; this one pipelines the
 * Gauss-Seidel wavefront over j-blocks instead).  Same argument meaning and
 * error contract as sdfgen_hip_make_level_set3 (include/sdfgen_hip.h).
 */
#ifndef SDFGEN_CPU_H
#define SDFGEN_CPU_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* The library is built with -fvisibility=hidden: exactly what this header declares is exported. */
#pragma GCC visibility push(default)

enum { SDFGEN_CPU_OK = 0, SDFGEN_CPU_EINVAL = -1, SDFGEN_CPU_EINDEX = -2, SDFGEN_CPU_ENOMEM = -5 };

/* num_threads: 0 = std::thread::hardware_concurrency() (fallback 4), as the reference
 * (cpu_lib/makelevelset3.cpp:240-241).  out_layout: 0 = i-fastest (Array3f), 1 = k-fastest. */
int sdfgen_cpu_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                               const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                               int num_threads, int out_layout, float *phi_out, char *errbuf, size_t errlen);

/* Z-slab sessions on the CPU (multi-process runs without GPUs): the same slab split as
 * sdfgen_hip_slab_* (slab s of n owns k in [s*nk/n, (s+1)*nk/n)).  Per sweep the caller
 * hands in the upstream slab's final boundary plane and forwards this slab's last plane
 * (ni*nj packed cells each: phi bits << 32 | closest triangle).  Upstream = the slab
 * below for k-up sweeps, above for k-down sweeps.  Bit-identical to the whole-grid run. */
typedef struct sdfgen_cpu_slab sdfgen_cpu_slab;
int sdfgen_cpu_slab_create(int nslabs, int slab, int ni, int nj, int nk, sdfgen_cpu_slab **out, char *errbuf,
                           size_t errlen);
int sdfgen_cpu_slab_range(const sdfgen_cpu_slab *s, int *k_begin, int *k_end);
/* tri/xyz must stay alive until the last sweep */
int sdfgen_cpu_slab_band(sdfgen_cpu_slab *s, const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                         const float origin[3], float dx, int exact_band, char *errbuf, size_t errlen);
int sdfgen_cpu_slab_sweep(sdfgen_cpu_slab *s, int sweep, const uint64_t *plane_in, uint64_t *plane_out,
                          char *errbuf, size_t errlen);
int sdfgen_cpu_slab_sign(sdfgen_cpu_slab *s, int out_layout, float *phi_slab, char *errbuf, size_t errlen);
int sdfgen_cpu_slab_destroy(sdfgen_cpu_slab *s);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
