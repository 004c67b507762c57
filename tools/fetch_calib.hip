// tools/fetch_calib.hip -- calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// the tile sweep uses (MI355X_MICROARCH.md "HBM": only 16-B coalesced reads and stores are calibrated).
// Every kernel touches a known number of bytes / 128-B lines of a 1 GiB buffer (4x the Infinity
// Cache, so nothing is served on-die across launches); tools/fetch_calib.py runs it under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` and divides.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned long long u64;
#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorName(e_));                                \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

// 16 B per lane, coalesced (the guide's calibrated case)
__global__ void k_read16(const float4 *__restrict__ p, size_t n, float *sink)
{
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1.2345f) sink[0] = acc;
}
// 8 B per lane, coalesced, plain loads (the cell / granule width)
__global__ void k_read8(const u64 *__restrict__ p, size_t n, u64 *sink)
{
    u64 acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
    if (acc == 12345) sink[0] = acc;
}
// 8 B per lane, coalesced, agent-scope atomic loads (the granule polls: global_load_dwordx2 ... sc1)
__global__ void k_read8_agent(const u64 *p, size_t n, u64 *sink)
{
    u64 acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (acc == 12345) sink[0] = acc;
}
// one 8-B agent-scope load per 128-B line (a column's granule stream read one entry at a time)
__global__ void k_read8_agent_line(const u64 *p, size_t nlines, u64 *sink)
{
    u64 acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x)
        acc += __hip_atomic_load(p + 16 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (acc == 12345) sink[0] = acc;
}
// one 16-B plain load per 128-B line, lines in a scattered order (the helper's vertex gathers)
__global__ void k_gather16_line(const float4 *p, size_t nlines, float *sink)
{
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x) {
        const size_t l = (i * 2654435761ull) & (nlines - 1);   // a permutation of the lines (nlines: a power of two)
        const float4 v = p[8 * l];
        acc += v.x;
    }
    if (acc == 1.2345f) sink[0] = acc;
}
// 8 B per lane, coalesced stores: plain and agent-scope atomic (the granule publish)
__global__ void k_write8(u64 *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = i;
}
__global__ void k_write8_agent(u64 *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, (u64)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one 8-B agent-scope store per 128-B line
__global__ void k_write8_agent_line(u64 *p, size_t nlines)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + 16 * i, (u64)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16 passes over a 1 MiB buffer (L2-resident after the first): do agent-scope loads (sc1) refetch
// every line from the memory side, like the first pass, or hit L2 like plain loads?
__global__ void k_reread8_agent(const u64 *p, size_t n, int passes, u64 *sink)
{
    u64 acc = 0;
    for (int r = 0; r < passes; ++r)
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
            acc += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + r;
    if (acc == 12345) sink[0] = acc;
}
__global__ void k_reread8(const u64 *p, size_t n, int passes, u64 *sink)
{
    u64 acc = 0;
    for (int r = 0; r < passes; ++r) {
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
            acc += p[i] + r;
        asm volatile("" ::: "memory");   // every pass loads again
    }
    if (acc == 12345) sink[0] = acc;
}

int main()
{
    const size_t bytes = 1ull << 30, lines = bytes / 128;
    char *buf = nullptr;
    void *sink = nullptr;
    CHK(hipMalloc((void **)&buf, bytes));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(buf, 1, bytes));
    CHK(hipDeviceSynchronize());
    const dim3 g(4096), b(256);
    // each kernel twice: the second launch of a pair is the one tools/fetch_calib.py reads (the first
    // warms nothing that fits on-die: 1 GiB > 256 MiB Infinity Cache)
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read16, g, b, 0, 0, (const float4 *)buf, bytes / 16, (float *)sink);
        hipLaunchKernelGGL(k_read8, g, b, 0, 0, (const u64 *)buf, bytes / 8, (u64 *)sink);
        hipLaunchKernelGGL(k_read8_agent, g, b, 0, 0, (const u64 *)buf, bytes / 8, (u64 *)sink);
        hipLaunchKernelGGL(k_read8_agent_line, g, b, 0, 0, (const u64 *)buf, lines, (u64 *)sink);
        hipLaunchKernelGGL(k_gather16_line, g, b, 0, 0, (const float4 *)buf, lines, (float *)sink);
        hipLaunchKernelGGL(k_write8, g, b, 0, 0, (u64 *)buf, bytes / 8);
        hipLaunchKernelGGL(k_write8_agent, g, b, 0, 0, (u64 *)buf, bytes / 8);
        hipLaunchKernelGGL(k_write8_agent_line, g, b, 0, 0, (u64 *)buf, lines);
        // 16 workgroups over one 1 MiB buffer: are the re-reads served by L2?
        hipLaunchKernelGGL(k_reread8_agent, dim3(16), b, 0, 0, (const u64 *)buf, (size_t)(1u << 17), 16, (u64 *)sink);
        hipLaunchKernelGGL(k_reread8, dim3(16), b, 0, 0, (const u64 *)buf, (size_t)(1u << 17), 16, (u64 *)sink);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
    }
    printf("{\"bytes\": %zu, \"lines\": %zu}\n", bytes, lines);
    CHK(hipFree(buf));
    CHK(hipFree(sink));
    return 0;
}
