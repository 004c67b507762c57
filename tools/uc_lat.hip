// tools/uc_lat.hip -- diagnostics only: round trip of one 8-byte granule hand-off between two
// workgroups of ONE GPU, in the memory kinds the Z-slab protocol and the single-GPU tiles use
// (the per-phase model's t_hop input):
//   0  hipMalloc (coarse-grained), agent-scope atomic store + agent-scope atomic load poll
//      (the single-GPU tile hand-off granules, sweep_tile.hpp)
//   1  hipMalloc, system-scope store + system-scope load poll
//   2  hipExtMallocWithFlags(hipDeviceMallocUncached), system-scope store + load (the slab comm
//      block: inboxes, halo planes, inbound rings, flags -- what a neighbour GPU writes)
// Block 0 stores round r to word A and waits for r on word B; block 1 (placed on another CU,
// and, by dispatch order, usually on another XCD) echoes.  Every spin is bounded.  The cross-GPU
// (xGMI) round trip cannot be measured on a one-GPU box; this is the on-chip floor of it.
// build: hipcc --offload-arch=gfx950 -O2 tools/uc_lat.hip -o tools/uc_lat
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

enum { ROUNDS = 4000, SPIN = 1 << 22 };

template <int SCOPE>
__global__ void k_pingpong(unsigned long long *w, unsigned long long *out)
{
    if (threadIdx.x != 0 || blockIdx.x > 1) return;
    unsigned long long *mine = w + (blockIdx.x ? 16 : 0), *theirs = w + (blockIdx.x ? 0 : 16);
    const unsigned long long t0 = wall_clock64();
    for (unsigned long long r = 1; r <= ROUNDS; ++r) {
        if (blockIdx.x == 0) __hip_atomic_store(mine, r, __ATOMIC_RELAXED, SCOPE);
        unsigned n = 0;
        while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, SCOPE) != r)
            if (++n > SPIN) { out[2 + blockIdx.x] = r; return; }
        if (blockIdx.x == 1) __hip_atomic_store(mine, r, __ATOMIC_RELAXED, SCOPE);
    }
    if (blockIdx.x == 0) out[0] = wall_clock64() - t0;
}

int main()
{
    int khz = 0;
    CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    unsigned long long *out = nullptr, *plain = nullptr, *uc = nullptr;
    CHK(hipMalloc((void **)&out, 8 * sizeof(unsigned long long)));
    CHK(hipMalloc((void **)&plain, 64 * sizeof(unsigned long long)));
    CHK(hipExtMallocWithFlags((void **)&uc, 1 << 21, hipDeviceMallocUncached));
    const char *names[3] = {"hipMalloc, agent scope (single-GPU tile granules)", "hipMalloc, system scope",
                            "uncached, system scope (Z-slab comm block)"};
    for (int v = 0; v < 3; ++v) {
        for (int rep = 0; rep < 3; ++rep) {
            unsigned long long *w = v == 2 ? uc : plain;
            CHK(hipMemset(w, 0, 64 * sizeof(unsigned long long)));
            CHK(hipMemset(out, 0, 8 * sizeof(unsigned long long)));
            // two blocks: consecutive workgroups are dispatched to different XCDs (round robin)
            if (v == 0) hipLaunchKernelGGL(k_pingpong<__HIP_MEMORY_SCOPE_AGENT>, dim3(2), dim3(64), 0, 0, w, out);
            else hipLaunchKernelGGL(k_pingpong<__HIP_MEMORY_SCOPE_SYSTEM>, dim3(2), dim3(64), 0, 0, w, out);
            CHK(hipDeviceSynchronize());
            unsigned long long h[8];
            CHK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
            if (h[2] || h[3]) printf("%-52s stale (round %llu / %llu)\n", names[v], h[2], h[3]);
            else printf("%-52s round trip %.3f us\n", names[v], h[0] / (khz * 1e-3) / ROUNDS);
        }
    }
    return 0;
}
