// PCIe write probe (diagnostics): a kernel storing 67 MB straight into a hipHostRegister'ed
// (mapped) pageable host buffer, against hipMemcpy D2H of the same bytes.
// hipcc --offload-arch=gfx950 -O3 -o tools/pcie_write tools/pcie_write.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorName(e_)); return 1; } } while (0)
__global__ void k_copy4(const float4 *__restrict__ s, float4 *__restrict__ d, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}
__global__ void k_copy1(const float *__restrict__ s, float *__restrict__ d, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char **argv)
{
    const size_t bytes = (size_t)(argc > 1 ? atof(argv[1]) : 67.108864) * 1000000 / 16 * 16;
    const int off = argc > 2 ? atoi(argv[2]) : 0;   // misalign the host buffer by this many bytes
    float *d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 0x3f, bytes));
    char *raw = (char *)malloc(bytes + 4096);
    float *h = (float *)(raw + off);
    memset(h, 0, bytes);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (int rep = 0; rep < 4; ++rep) {
        double t0 = now();
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        double t1 = now();
        printf("hipMemcpy D2H pageable %.3f ms (%.1f GB/s)\n", (t1 - t0) * 1e3, bytes / (t1 - t0) / 1e9);
    }
    for (int g = 0; g < 3; ++g) {
        const unsigned grid = g == 0 ? 1024 : (g == 1 ? 4096 : 16384);
        for (int rep = 0; rep < 3; ++rep) {
            memset(h, 0, 4096);
            double t0 = now();
            CK(hipHostRegister(h, bytes, hipHostRegisterMapped));
            void *hd;
            CK(hipHostGetDevicePointer(&hd, h, 0));
            double t1 = now();
            if (off % 16 == 0) hipLaunchKernelGGL(k_copy4, dim3(grid), dim3(256), 0, st, (const float4 *)d, (float4 *)hd, bytes / 16);
            else hipLaunchKernelGGL(k_copy1, dim3(grid), dim3(256), 0, st, d, (float *)hd, bytes / 4);
            CK(hipStreamSynchronize(st));
            double t2 = now();
            CK(hipHostUnregister(h));
            double t3 = now();
            int bad = 0;
            for (size_t i = 0; i < bytes / 4; i += 4099) bad += ((unsigned *)h)[i] != 0x3f3f3f3fu;
            printf("grid %5u: register %.3f ms, kernel store %.3f ms (%.1f GB/s), unregister %.3f ms, total %.3f ms, bad %d\n",
                   grid, (t1 - t0) * 1e3, (t2 - t1) * 1e3, bytes / (t2 - t1) / 1e9, (t3 - t2) * 1e3, (t3 - t0) * 1e3, bad);
        }
    }
    return 0;
}
