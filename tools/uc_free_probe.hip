// tools/uc_free_probe.hip -- is "hipFree of an uncached block, then hipMalloc of the same virtual range"
// unsafe on its own (DESIGN.md §6 "freed uncached memory")?
//
// The round-4 failure: after in-process two-slab calls (whose communication block is one 2 MiB
// hipExtMallocWithFlags(..., hipDeviceMallocUncached) allocation, polled from many CUs at system scope),
// hipFree of that block, and a one-GPU call whose tile halo buffer hipMalloc placed on exactly that range,
// the tile hand-off lost granules (consumers read zeros).  This probe replays only the memory sequence:
//   A  prime:   a block (uncached, or a plain hipMalloc block as the control) carries a producer/consumer
//               hand-off of tagged 8-byte granules between workgroup pairs on every CU, system scope
//   F  free:    hipFree(block)
//   B  reuse:   hipMalloc blocks of 2 .. 128 MiB until one covers the freed range (at most 64 tries; a
//               first version asking for 2 MiB blocks only never got the range back), zero the block
//               with hipMemsetAsync as st_grow does, then the tile sweep's hand-off form (agent scope) on
//               exactly the freed range, twice, and a plain fill read back by hipMemcpy
// and counts granules a consumer never saw (bounded spins: a lost store ends as a count, not a hang) and
// words that read back wrong.  Every kernel's spin has an exit every wave reaches.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/uc_free_probe tools/uc_free_probe.hip
//   run:   tools/uc_free_probe [rounds]     (prints one line per variant and round)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef unsigned long long u64;
#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_));      \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

constexpr size_t BYTES = 2u << 20;           // the slab communication block's size
constexpr size_t NG = BYTES / sizeof(u64);   // granules
constexpr int GRID = 256;                    // one workgroup per CU: pairs (b, b ^ 1) are co-resident
constexpr int THREADS = 256;
constexpr unsigned SPIN_MAX = 1u << 20;      // polls per granule before it counts as lost

// Workgroup b publishes granules {epoch, index} of its chunk, then polls its partner's chunk until every
// granule carries this epoch (or the spin budget runs out: counted in fail[0]); wrong payloads: fail[1].
template <int SCOPE>
__global__ void __launch_bounds__(THREADS) k_handoff(u64 *g, unsigned epoch, unsigned *fail)
{
    constexpr size_t CH = NG / GRID;
    const size_t mine = (size_t)blockIdx.x * CH, theirs = (size_t)(blockIdx.x ^ 1) * CH;
    for (size_t i = threadIdx.x; i < CH; i += THREADS)
        __hip_atomic_store(g + mine + i, ((u64)epoch << 32) | (uint32_t)(mine + i), __ATOMIC_RELAXED, SCOPE);
    unsigned lost = 0, bad = 0;
    for (size_t i = threadIdx.x; i < CH; i += THREADS) {
        u64 v = 0;
        unsigned s = 0;
        for (; s < SPIN_MAX; ++s) {
            v = __hip_atomic_load(g + theirs + i, __ATOMIC_RELAXED, SCOPE);
            if ((unsigned)(v >> 32) == epoch) break;
            if (s > 64) __builtin_amdgcn_s_sleep(2);
        }
        if (s == SPIN_MAX) ++lost;
        else if ((uint32_t)v != (uint32_t)(theirs + i)) ++bad;
    }
    if (lost) atomicAdd(fail, lost);
    if (bad) atomicAdd(fail + 1, bad);
}

__global__ void k_fill(u64 *g, u64 salt)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < NG; i += (size_t)gridDim.x * blockDim.x)
        g[i] = (salt << 32) ^ i;
}

struct Res {
    unsigned lostA, badA, lostB, badB, lostB2, badB2;
    size_t fill_bad, off, blk;
    int tries;
    bool reused;
};

static void handoff(u64 *g, unsigned epoch, bool system, unsigned *d_fail, unsigned *lost, unsigned *bad)
{
    CHK(hipMemset(d_fail, 0, 2 * sizeof(unsigned)));
    if (system) hipLaunchKernelGGL(k_handoff<__HIP_MEMORY_SCOPE_SYSTEM>, dim3(GRID), dim3(THREADS), 0, 0, g, epoch, d_fail);
    else hipLaunchKernelGGL(k_handoff<__HIP_MEMORY_SCOPE_AGENT>, dim3(GRID), dim3(THREADS), 0, 0, g, epoch, d_fail);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    unsigned h[2];
    CHK(hipMemcpy(h, d_fail, sizeof(h), hipMemcpyDeviceToHost));
    *lost = h[0];
    *bad = h[1];
}

static Res run(bool uncached, bool adjacent, unsigned *d_fail, unsigned ep)
{
    Res r{};
    u64 *a = nullptr;
    if (uncached) CHK(hipExtMallocWithFlags((void **)&a, BYTES, hipDeviceMallocUncached));
    else CHK(hipMalloc((void **)&a, BYTES));
    CHK(hipMemset(a, 0, BYTES));
    handoff(a, ep, true, d_fail, &r.lostA, &r.badA);
    // the round-4 failure freed the comm block together with the session's other buffers, and the next
    // call's 4.4 MB halo buffer started exactly at the block's address: free a neighbour block as well
    u64 *nb = nullptr;
    if (adjacent) CHK(hipMalloc((void **)&nb, 8 * BYTES));
    CHK(hipFree(a));
    if (nb) CHK(hipFree(nb));
    // hipMalloc blocks of growing sizes (2 MiB .. 128 MiB, as the tile sweep's halo buffers are) until
    // one covers the freed range; the hand-off then runs on exactly that range inside it
    std::vector<u64 *> held;
    u64 *b = nullptr, *blk = nullptr;
    size_t blk_bytes = 0;
    for (r.tries = 1; r.tries <= 64; ++r.tries) {
        // 2 .. 128 MiB, and sizes that straddle the block (the failing halo buffer was 4.4 MB)
        const size_t sz = (r.tries % 2) ? (BYTES << ((r.tries / 2) % 7)) : (BYTES + (BYTES / 5) * (size_t)(r.tries % 23));
        u64 *x = nullptr;
        CHK(hipMalloc((void **)&x, sz));
        if ((char *)x < (char *)a + BYTES && (char *)a < (char *)x + sz) {   // overlaps the freed range
            blk = x;
            blk_bytes = sz;
            // the part of the freed range inside the new block (at least one granule pair's chunk)
            b = (char *)a >= (char *)x ? a : x;
            if ((size_t)((char *)x + sz - (char *)b) < BYTES) b = (u64 *)((char *)x + sz - BYTES);
            break;
        }
        held.push_back(x);
    }
    r.reused = b != nullptr;
    if (!b) {   // the range was not handed out again: test a fresh block anyway
        CHK(hipMalloc((void **)&blk, BYTES));
        blk_bytes = BYTES;
        b = blk;
    }
    r.off = (size_t)((char *)b - (char *)blk);
    r.blk = blk_bytes;
    CHK(hipMemsetAsync(blk, 0, blk_bytes, 0));
    handoff(b, ep + 1, false, d_fail, &r.lostB, &r.badB);
    handoff(b, ep + 2, false, d_fail, &r.lostB2, &r.badB2);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, b, (u64)ep);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    std::vector<u64> h(NG);
    CHK(hipMemcpy(h.data(), b, BYTES, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < NG; ++i) r.fill_bad += h[i] != (((u64)ep << 32) ^ i);
    CHK(hipFree(blk));
    for (u64 *p : held) CHK(hipFree(p));
    return r;
}

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    unsigned *d_fail = nullptr;
    CHK(hipMalloc((void **)&d_fail, 2 * sizeof(unsigned)));
    hipDeviceProp_t pr;
    CHK(hipGetDeviceProperties(&pr, 0));
    printf("device %s, %d CUs; block %zu bytes, %d workgroups in pairs, spin budget %u polls per granule\n", pr.gcnArchName,
           pr.multiProcessorCount, BYTES, GRID, SPIN_MAX);
    unsigned ep = 1;
    int total_bad = 0;
    for (int k = 0; k < rounds; ++k)
        for (int v = 3; v >= 0; --v) {
            const int uc = v & 1;
            const bool adj = v & 2;
            const Res r = run(uc != 0, adj, d_fail, ep);
            ep += 4;
            const unsigned long long bad = (unsigned long long)r.lostB + r.badB + r.lostB2 + r.badB2 + r.fill_bad;
            total_bad += bad != 0;
            printf("round %d %-9s %s prime: lost %u bad %u | freed range handed out again: %s (try %d, inside a %zu MiB block at "
                   "offset %zu) | reuse hand-off: lost %u bad %u, again: lost %u bad %u | fill read-back wrong words %zu\n",
                   k, uc ? "uncached" : "plain", adj ? "+neighbour freed" : "alone          ", r.lostA, r.badA, r.reused ? "yes" : "no", r.tries, r.blk >> 20, r.off, r.lostB,
                   r.badB, r.lostB2, r.badB2, r.fill_bad);
            fflush(stdout);
        }
    printf("%s\n", total_bad ? "REPRODUCED: wrong data on a reused range" : "not reproduced: every reuse read back correct");
    return 0;
}
