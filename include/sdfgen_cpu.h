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

enum { SDFGEN_CPU_OK = 0, SDFGEN_CPU_EINVAL = -1, SDFGEN_CPU_EINDEX = -2, SDFGEN_CPU_ENOMEM = -5 };

/* num_threads: 0 = std::thread::hardware_concurrency() (fallback 4), as the reference
 * (cpu_lib/makelevelset3.cpp:240-241).  out_layout: 0 = i-fastest (Array3f), 1 = k-fastest. */
int sdfgen_cpu_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                               const float origin[3], float dx, int ni, int nj, int nk, int exact_band,
                               int num_threads, int out_layout, float *phi_out, char *errbuf, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif
