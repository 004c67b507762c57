// Staging-buffer probe (diagnostics): kernel stores of 16 MB chunks into pinned host memory of several
// kinds, and the host's memcpy out of it into a pageable array (resident pages), alone and pipelined.
// hipcc --offload-arch=gfx950 -O3 -o tools/stage_probe tools/stage_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorName(e_)); exit(1); } } while (0)
__global__ void k_fill(const float *__restrict__ s, float *__restrict__ d, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main()
{
    const size_t total = 64ull << 20, chunk = 16ull << 20, nch = total / chunk;
    float *d;
    CK(hipMalloc(&d, total));
    CK(hipMemset(d, 0x3f, total));
    float *user = (float *)malloc(total);
    memset(user, 0, total);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t ev[2];
    for (auto &e : ev) CK(hipEventCreate(&e));
    const char *names[] = {"hipHostMalloc Mapped|Coherent", "hipHostMalloc default", "hipHostMalloc NonCoherent",
                           "malloc + hipHostRegister(Mapped)", "hipHostMalloc Mapped|Coherent, ev BlockingSync"};
    for (int kind = 0; kind < 5; ++kind) {
        float *h = nullptr;
        if (kind == 0 || kind == 4) CK(hipHostMalloc((void **)&h, 2 * chunk, hipHostMallocMapped | hipHostMallocCoherent));
        if (kind == 1) CK(hipHostMalloc((void **)&h, 2 * chunk, 0));
        if (kind == 2) CK(hipHostMalloc((void **)&h, 2 * chunk, hipHostMallocNonCoherent));
        if (kind == 3) { h = (float *)malloc(2 * chunk); memset(h, 0, 2 * chunk); CK(hipHostRegister(h, 2 * chunk, hipHostRegisterMapped)); }
        hipEvent_t e2[2];
        for (auto &e : e2) CK(hipEventCreateWithFlags(&e, kind == 4 ? hipEventBlockingSync : hipEventDefault));
        float *hd;
        CK(hipHostGetDevicePointer((void **)&hd, h, 0));
        for (int rep = 0; rep < 3; ++rep) {
            // kernel store alone
            double t0 = now();
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, d, hd, chunk / 4);
            CK(hipStreamSynchronize(st));
            double t1 = now();
            memcpy(user, h, chunk);
            double t2 = now();
            // pipelined: 4 chunks, two slots
            double t3 = now();
            for (size_t c = 0; c < 2; ++c) {
                hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, d + c * chunk / 4, hd + (c & 1) * chunk / 4, chunk / 4);
                CK(hipEventRecord(e2[c & 1], st));
            }
            for (size_t c = 0; c < nch; ++c) {
                CK(hipEventSynchronize(e2[c & 1]));
                memcpy((char *)user + c * chunk, (char *)h + (c & 1) * chunk, chunk);
                if (c + 2 < nch) {
                    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, d + (c + 2) * chunk / 4, hd + (c & 1) * chunk / 4, chunk / 4);
                    CK(hipEventRecord(e2[c & 1], st));
                }
            }
            double t4 = now();
            printf("%-46s store 16 MB %.3f ms (%.1f GB/s), host memcpy 16 MB out %.3f ms (%.1f GB/s), pipelined 64 MB %.3f ms, ok %d\n",
                   names[kind], (t1 - t0) * 1e3, chunk / (t1 - t0) / 1e9, (t2 - t1) * 1e3, chunk / (t2 - t1) / 1e9,
                   (t4 - t3) * 1e3, ((unsigned *)user)[12345] == 0x3f3f3f3fu);
        }
        for (auto &e : e2) CK(hipEventDestroy(e));
        if (kind == 3) { CK(hipHostUnregister(h)); free(h); } else CK(hipHostFree(h));
    }
    double t0 = now();
    CK(hipMemcpy(user, d, total, hipMemcpyDeviceToHost));
    double t1 = now();
    printf("hipMemcpy D2H 64 MB pageable: %.3f ms\n", (t1 - t0) * 1e3);
    return 0;
}
