/*
 * sdfgen_hip.h -- C-ABI of the MI355X (gfx950) signed-distance-field backend.
 *
 * This is the drop-in boundary for the reference's hot path
 *   sdfgen::make_level_set3(tri, x, origin, dx, nx, ny, nz, phi, exact_band,
 *                           HardwareBackend, num_threads)
 *     declared   /root/reference/common/sdfgen_unified.h:47-57
 *     dispatched /root/reference/common/sdfgen_unified.cpp:30-71
 *     GPU case   /root/reference/gpu_lib/makelevelset3_gpu.h:40-42 (gpu::make_level_set3)
 *   sdfgen::is_gpu_available()   common/sdfgen_unified.h:68, .cpp:19-28
 * Plain pointers and sizes only; no C++ or torch types cross it.  A reference
 * maintainer binds it from gpu_lib (C++), python/sdfgen_py.cpp (nanobind) or
 * ctypes -- see INTEGRATION.md.
 *
 * Semantics: results are bit-identical to the reference's single-threaded CPU
 * implementation cpu_lib/makelevelset3.cpp:192-304 (distances, closest-triangle
 * tie-breaks and the -0.0 produced by the sign flip), NOT to the reference CUDA
 * backend, whose far field is a different (Eikonal) algorithm.
 *
 * Contract for every entry point:
 *   - returns SDFGEN_HIP_OK (0) on success, a negative SDFGEN_HIP_E* code
 *     otherwise, with a NUL-terminated message in errbuf (if errbuf != NULL);
 *   - never calls exit()/abort(), never retains caller pointers after return;
 *   - synchronous on return (host entry points), reentrant (serialised per
 *     device internally).
 */
#ifndef SDFGEN_HIP_H
#define SDFGEN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* The library is built with -fvisibility=hidden: exactly what this header declares is exported. */
#pragma GCC visibility push(default)

#define SDFGEN_HIP_ABI_VERSION 5   /* 2: sdfgen_hip_profile.slabs / chain_steps, slab_prepare; 3: slab_* phase timers, tile_cfg; 4: sdfgen_hip_topology;
                                      5: sdfgen_hip_slab_close_imports (release keeps IPC mappings) */

enum {
    SDFGEN_HIP_OK = 0,
    SDFGEN_HIP_EINVAL = -1,      /* bad argument (dims <= 0, dx <= 0 / non-finite, layout, ...) */
    SDFGEN_HIP_EINDEX = -2,      /* a triangle references a vertex index >= nvert */
    SDFGEN_HIP_ENODEV = -3,      /* no usable HIP device */
    SDFGEN_HIP_ERUNTIME = -4,    /* HIP runtime / kernel error */
    SDFGEN_HIP_ENOMEM = -5       /* device allocation failed */
};

/* ngpu values of sdfgen_hip_make_level_set3 (any n > 1 is also accepted). */
#define SDFGEN_NGPU_ALL 0
#define SDFGEN_NGPU_CURRENT 1

/* Output layouts for phi_out. */
enum {
    SDFGEN_LAYOUT_ARRAY3 = 0,    /* i-fastest: phi[i + ni*(j + nj*k)] (Array3f, common/array3.h:114) */
    SDFGEN_LAYOUT_KFAST = 1      /* k-fastest: phi[(i*nj + j)*nk + k] (numpy (ni,nj,nk) C-order and
                                    the .sdf body, python/sdfgen_py.cpp:80-86, common/sdf_io.cpp:49-57) */
};

int sdfgen_hip_abi_version(void);

/* Build identity: the first 16 hex digits of the SHA-256 of the sources and build files this
 * library was compiled from (sdfgenfast_amd/Makefile).  No reference counterpart; bench.py uses it
 * to match PMC counter summaries to the library that produced the timed numbers. */
const char *sdfgen_hip_build_id(void);

/* Number of visible HIP devices (0 when none; never an error).
 * Replaces sdfgen::is_gpu_available() (common/sdfgen_unified.cpp:19-28). */
int sdfgen_hip_device_count(void);

/* Node topology for the multi-GPU diagnostics (no reference counterpart: the reference has no
 * multi-GPU layer, README.md:220).  *ndev = visible devices; for the first min(ndev, max_dev):
 * pci_bus_ids (may be NULL) gets SDFGEN_HIP_PCI_ID_BYTES bytes per device ("0000:05:00.0", NUL
 * terminated; empty if unknown), peer (may be NULL) a max_dev x max_dev row-major matrix with
 * peer[i * max_dev + j] = hipDeviceCanAccessPeer(i, j) (1 on the diagonal, -1 if the query failed).
 * bench.py --gpus N records it with each rank's device. */
#define SDFGEN_HIP_PCI_ID_BYTES 32
int sdfgen_hip_topology(int max_dev, int *ndev, char *pci_bus_ids, int *peer);

/*
 * Host-memory entry point; replaces gpu::make_level_set3 (gpu_lib/makelevelset3_gpu.cu:595-777).
 *   tri      : ntri x 3 uint32 vertex indices (std::vector<Vec3ui>::data(), common/vec.h:28)
 *   xyz      : nvert x 3 float32 positions   (std::vector<Vec3f>::data())
 *   origin   : grid origin (3 floats); dx: cell size; ni,nj,nk: grid dims (> 0)
 *   exact_band: band half-width in cells (cpu_lib/makelevelset3.cpp:210-212)
 *   ngpu     : devices to use.  SDFGEN_NGPU_ALL (0) = every visible device;
 *              SDFGEN_NGPU_CURRENT (1) = the current device only (what the reference's GPU
 *              backend does, gpu_lib/makelevelset3_gpu.cu:600-603, and what the C++ and Python
 *              drop-ins pass); n > 1 = devices 0..n-1.  With more than one device the grid is
 *              split into Z-slabs driven from this thread (sdfgen_hip_slab_* sessions connected
 *              in-process over peer memory), at most nk/2 of them; ENODEV if
 *              fewer than n devices are visible, EINVAL for n < 0.
 *   out_layout: SDFGEN_LAYOUT_*
 *   phi_out  : caller-allocated ni*nj*nk floats
 */
int sdfgen_hip_make_level_set3(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                               const float origin[3], float dx, int ni, int nj, int nk,
                               int exact_band, int ngpu, int out_layout, float *phi_out,
                               char *errbuf, size_t errlen);

/*
 * Device-resident entry point (inputs already in HBM of `device`): the same
 * computation on caller-owned device buffers, enqueued on `hip_stream`
 * (a hipStream_t; NULL = the library's own stream) and synchronised before
 * return.  d_phi_out: ni*nj*nk floats on `device`.
 */
int sdfgen_hip_make_level_set3_device(int device, const uint32_t *d_tri, uint64_t ntri,
                                      const float *d_xyz, uint64_t nvert, const float origin[3],
                                      float dx, int ni, int nj, int nk, int exact_band,
                                      int out_layout, float *d_phi_out, void *hip_stream,
                                      char *errbuf, size_t errlen);

/* Per-phase device timings of the last call on the calling process (HIP events
 * recorded on the launch stream around each phase / sweep launch). */
typedef struct sdfgen_hip_profile {
    double total_ms;          /* first kernel start .. last kernel end */
    double prep_ms;           /* triangle gather + workspace init */
    double band_ms;           /* narrow band + ray-parity counts */
    double sweep_ms;          /* all 16 sweeps */
    double sign_ms;           /* sign pass + output layout */
    double sweep_launch_ms[16];  /* per (pass, direction) sweep */
    int sweep_launches;       /* kernel launches issued for the sweeps */
    int sweep_impl;           /* 0 = hyperplane launches, 1 = pipelined 8x8-tile column wavefront,
                                 2 = tile wavefront for the first pass + Jacobi/repair for sparse sweeps
                                 (on one device or, `slabs` > 1, per Z-slab) */
    uint64_t band_evals;      /* point-triangle evaluations in the band phase */
    uint64_t sweep_evals;     /* evaluations in the sweeps (0 unless SDFGEN_COUNT_EVALS is set) */
    uint64_t sweep_stalls;    /* compute-wave polls that found a hand-off not yet landed (same) */
    uint64_t helper_polls;    /* helper-wave polls that found nothing to fetch (same) */
    uint64_t own_waits;       /* compute-wave polls waiting on the column prefetch (same) */
    int sparse_sweeps;        /* sweeps run as Jacobi + change-driven repair */
    int sparse_first;         /* index of the first such sweep (16 = none) */
    uint64_t sparse_rechecks; /* cell re-evaluations in the repair kernels (all sparse sweeps) */
    uint64_t sparse_claims;   /* rechecks run depth-first by the lane that requested them */
    int tile_multi;           /* first-pass sweeps run as ONE overlapped launch (0: one launch per
                                 sweep); its time is then sweep_launch_ms[0] */
    int slabs;                /* Z-slabs the grid was split into (0 or 1: one device) */
    double chain_steps;       /* modelled critical path of the first-pass launch, in tile steps (the
                                 latency roofline's chain length; 0 without the overlapped launch) */
    /* Z-slab phase timers of the last call on this slab (device wall clock; all 0 on one device).
     * Second-pass sweep 9 + m, m = 0..7: */
    double slab_wait_done_ms[8];     /* waiting for the neighbours' DONE of the previous sweep (longer side) */
    double slab_wait_ready_ms[8];    /* waiting for their READY (live halos initialised) */
    double slab_repair_ms[8];        /* the repair kernel: first workgroup's start .. last wave's exit */
    double slab_inbound_ms[8];       /* its inbound lanes: until the upstream slab's repair ended, entries taken */
    uint64_t slab_inbound_entries[8];   /* inbound-ring entries taken (upstream boundary cells that relabelled) */
    /* First pass: */
    double slab_inbox_idle_ms;       /* helper-wave idle time of the tasks reading the upstream GPU's inbox, summed */
    double slab_other_idle_ms;       /* the same for the other tasks */
    uint64_t slab_inbox_tasks, slab_other_tasks;
    int tile_cfg;                    /* first-pass tile kernel: 0 = 2 compute waves x 32 cells (latency-bound
                                        grids), 1 = 1 compute wave x 64 cells (throughput-bound grids),
                                        2 = 4 compute waves x 16 cells, four lanes per cell */
} sdfgen_hip_profile;

int sdfgen_hip_last_profile(sdfgen_hip_profile *out);

/* Free cached device workspaces (they are grow-only between calls).  The process's own pool of
 * uncached communication blocks (power-of-two size classes from 2 MiB, reused by later sessions) and
 * the HIP IPC mappings of neighbour slabs' blocks are kept: a freed uncached range handed to a later
 * hipMalloc has been seen to lose stores, and an imported mapping is uncached too. */
int sdfgen_hip_release(void);

/* ---------------------------------------------------------------------------
 * Z-slab decomposition over several GPUs (north_star: "the voxel grid shards along Z
 * into per-GPU slabs").  No reference counterpart -- the reference is single-device
 * (README.md:220 lists multi-GPU as future work); SURVEY.md §8.e.
 *
 * A session owns planes k in [k_begin, k_end) of an ni x nj x nk grid (slab s of n:
 * k_begin = s*nk/n) and allocates only those planes.  Band, ray parity and sign are local.
 * Sweeps 1-8 run as one overlapped tile-wavefront launch per slab in a schedule computed
 * for all slabs; the boundary plane travels between neighbouring slabs as tagged granules
 * written straight into the neighbour's inbox, so the wavefront pipelines across GPUs
 * inside every sweep.  Sweeps 9-16 run as Jacobi + repair per slab; boundary-plane label
 * changes are pushed into the neighbour's halo plane and inbound ring.  Everything a
 * neighbour writes is one uncached allocation per slab (xGMI; mapped across processes
 * with HIP IPC).  Result bits equal the single-GPU / reference bits.
 *
 * One process per GPU:   create -> export (IPC handle) -> exchange handles (e.g.
 * torch.distributed all_gather) -> connect_ipc(lower, upper) -> barrier -> run.
 * Several slabs in one process (any devices): create each -> connect_local.
 * enqueue/finish split lets one thread drive several sessions concurrently. */
typedef struct sdfgen_hip_slab sdfgen_hip_slab;
#define SDFGEN_HIP_IPC_HANDLE_BYTES 64

int sdfgen_hip_slab_create(int device, int nslabs, int slab, int ni, int nj, int nk, sdfgen_hip_slab **out,
                           char *errbuf, size_t errlen);
int sdfgen_hip_slab_range(const sdfgen_hip_slab *s, int *k_begin, int *k_end);
/* handle: SDFGEN_HIP_IPC_HANDLE_BYTES bytes describing this slab's inboxes */
int sdfgen_hip_slab_export(sdfgen_hip_slab *s, void *handle, char *errbuf, size_t errlen);
/* lower/upper: the neighbours' exported handles (NULL for slab 0 / the last slab) */
int sdfgen_hip_slab_connect_ipc(sdfgen_hip_slab *s, const void *lower, const void *upper, char *errbuf,
                                size_t errlen);
int sdfgen_hip_slab_connect_local(sdfgen_hip_slab *s, sdfgen_hip_slab *lower, sdfgen_hip_slab *upper,
                                  char *errbuf, size_t errlen);
/* Allocate everything a call with ntri triangles needs (enqueue does it too when needed).  A
 * thread that drives SEVERAL slabs must prepare all of them before it enqueues any of them: setting
 * a slab up while another slab's kernels already wait on it can block the thread. */
int sdfgen_hip_slab_prepare(sdfgen_hip_slab *s, uint64_t ntri, char *errbuf, size_t errlen);
/* Opt-in (ABI 5): close this process's IPC mappings of neighbour slabs' communication blocks.  Only
 * when no slab session is alive (returns the number closed, 0 while one is).  For a long-lived process
 * whose peer processes are replaced between jobs (a new peer's handle bytes could equal an exited
 * one's).  The closed virtual ranges return to this process's allocator -- the situation the block
 * pool avoids -- so the library never does this on its own. */
int sdfgen_hip_slab_close_imports(void);
/* Device buffers on the session's GPU; d_phi_slab receives ni*nj*(k_end-k_begin) floats in
 * the chosen layout (ARRAY3: i fastest, the slab's planes only; KFAST: k fastest). */
int sdfgen_hip_slab_enqueue(sdfgen_hip_slab *s, const uint32_t *d_tri, uint64_t ntri, const float *d_xyz,
                            uint64_t nvert, const float origin[3], float dx, int exact_band, int out_layout,
                            float *d_phi_slab, char *errbuf, size_t errlen);
int sdfgen_hip_slab_finish(sdfgen_hip_slab *s, uint64_t nvert, sdfgen_hip_profile *prof, char *errbuf,
                           size_t errlen);
/* Host buffers: upload, enqueue, download into phi_slab, finish. */
int sdfgen_hip_slab_run(sdfgen_hip_slab *s, const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert,
                        const float origin[3], float dx, int exact_band, int out_layout, float *phi_slab,
                        sdfgen_hip_profile *prof, char *errbuf, size_t errlen);
int sdfgen_hip_slab_destroy(sdfgen_hip_slab *s);
/* Diagnostics: copy a slab's device state to host (after its stream drained).  which: 0 = the
 * communication block, 1 = tile-sweep control words, 2 = first-pass completion flags, 3 = its
 * task table, 4 = its dependency table.  *n_bytes = bytes copied (at most max_bytes). */
int sdfgen_hip_slab_debug_dump(sdfgen_hip_slab *s, int which, void *out, uint64_t max_bytes, uint64_t *n_bytes);

/* Diagnostics (used by the parity tests): evaluate the device geometry kernels
 * on host arrays.  pts: n x 12 floats (x0,x1,x2,x3) -> out: n floats;
 * variant 0 = point_triangle_distance as used by the band kernel, 1 = the
 * branch-free form, 2 = the wave-uniform form used by the tile sweep, 3/4 = the
 * packed two-pair form (the first / second half of a pair of adjacent inputs);
 * all must give identical bits.
 * pit: n x 8 doubles (x0,y0,x1,y1,x2,y2,x3,y3) -> out4: n x (flag,a,b,c). */
int sdfgen_hip_debug_ptd(int device, int variant, uint64_t n, const float *pts, float *out,
                         char *errbuf, size_t errlen);
int sdfgen_hip_debug_pit2d(int device, uint64_t n, const double *pit, double *out4,
                           char *errbuf, size_t errlen);

/* Diagnostics (used by the parity tests): stage 1 only -- init, narrow band and ray-parity counts
 * (cpu_lib/makelevelset3.cpp:196-236) -- on the current device, host buffers in and the pre-sweep
 * state out: phi and closest_tri (-1 = none) per cell and the intersection counts, i-fastest, each
 * ni*nj*nk entries.  *big_n (if not NULL) = triangles the band phase spread over the chip as big
 * ones (band box > 4096 cells or ray lattice > 1024 points). */
int sdfgen_hip_debug_band(const uint32_t *tri, uint64_t ntri, const float *xyz, uint64_t nvert, const float origin[3],
                          float dx, int ni, int nj, int nk, int exact_band, float *phi, int32_t *ct, uint32_t *cnt,
                          uint64_t *big_n, char *errbuf, size_t errlen);

/* Diagnostics: per-task [start, first step, middle step, end] wall-clock stamps (100 MHz) of the sweep named by
 * the SDFGEN_TRACE_SWEEP environment variable in the last call (tasks in dequeue order). */
int sdfgen_hip_debug_sweep_trace(int device, uint64_t *out, uint64_t max_entries, uint64_t *n_out);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* SDFGEN_HIP_H */
