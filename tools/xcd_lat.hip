// tools/xcd_lat.hip -- diagnostics only: latency of the memory operations a repair chain step is
// made of, between two workgroups on the SAME XCD (different CUs) and on DIFFERENT XCDs.
//   ping-pong of a flag: device-scope (sc1) store + sc1 load poll, vs plain store + nt load poll
//   (the nt variants read stale: the compiler may keep a non-volatile load out of the spin loop);
//   a dependent chain of returning atomics: agent scope vs workgroup scope;
//   a dependent chain of loads of one word: sc1 vs nt vs plain.
// Every spin is bounded; a variant whose value never arrives reports "stale".
// build: hipcc --offload-arch=gfx950 -O2 tools/xcd_lat.hip -o tools/xcd_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ unsigned xcc_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

enum { ROUNDS = 2000, SPIN = 1 << 22 };

struct Out {
    unsigned xcc[64];
    unsigned pair[16];   // XCC (+1) of the two blocks of each ping-pong slot
    unsigned long long t[16];
    unsigned fail[16];
};

template <int MODE>
__device__ __forceinline__ void st_flag(unsigned *p, unsigned v)
{
    if (MODE == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (MODE == 1) { *(volatile unsigned *)p = v; }
    else __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int MODE>
__device__ __forceinline__ unsigned ld_flag(unsigned *p)
{
    if (MODE == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_nontemporal_load(p);
}

// ping-pong between block a and block b; slot s of the output
template <int MODE>
__device__ void pingpong(unsigned *flags, Out *o, int a, int b, int s)
{
    if (threadIdx.x != 0) return;
    unsigned *f0 = flags + s * 64, *f1 = flags + s * 64 + 32;
    if ((int)blockIdx.x == a) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (unsigned r = 1; r <= ROUNDS; ++r) {
            st_flag<MODE>(f0, r);
            unsigned n = 0;
            while (ld_flag<MODE>(f1) != r)
                if (++n > SPIN) { o->fail[s] = r; return; }
        }
        o->t[s] = __builtin_amdgcn_s_memtime() - t0;
    } else if ((int)blockIdx.x == b) {
        for (unsigned r = 1; r <= ROUNDS; ++r) {
            unsigned n = 0;
            while (ld_flag<MODE>(f0) != r)
                if (++n > SPIN) { o->fail[s + 8] = r; return; }
            st_flag<MODE>(f1, r);
        }
    }
}

__global__ void k_xcc(Out *o) { if (threadIdx.x == 0) o->xcc[blockIdx.x] = xcc_id(); }

template <int MODE>
__global__ void k_pp(unsigned *flags, Out *o, int a, int b, int s)
{
    if (threadIdx.x == 0 && ((int)blockIdx.x == a || (int)blockIdx.x == b))
        o->pair[2 * s + ((int)blockIdx.x == b)] = xcc_id() + 1;
    pingpong<MODE>(flags, o, a, b, s);
}

// dependent chains in one lane of block 0
__global__ void k_chain(unsigned long long *w, unsigned *u, Out *o)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    unsigned long long t0, acc = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) acc += atomicAdd(w + (acc >> 62), 1ull);   // agent scope
    o->t[8] = __builtin_amdgcn_s_memtime() - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r)
        acc += __hip_atomic_fetch_add(w + 16 + (acc >> 62), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    o->t[9] = __builtin_amdgcn_s_memtime() - t0;
    unsigned x = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) x += __hip_atomic_load(u + (x >> 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    o->t[10] = __builtin_amdgcn_s_memtime() - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) x += __builtin_nontemporal_load(u + 32 + (x >> 31));
    o->t[11] = __builtin_amdgcn_s_memtime() - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < ROUNDS; ++r) x += *(volatile unsigned *)(u + 64 + (x >> 31));
    o->t[12] = __builtin_amdgcn_s_memtime() - t0;
    o->fail[15] = (unsigned)acc + x;
}

int main()
{
    Out *o;
    unsigned *flags;
    unsigned long long *w;
    CHK(hipMalloc(&o, sizeof(Out)));
    CHK(hipMalloc(&flags, 64 * 64 * 4));
    CHK(hipMalloc(&w, 4096));
    CHK(hipMemset(o, 0, sizeof(Out)));
    CHK(hipMemset(flags, 0, 64 * 64 * 4));
    CHK(hipMemset(w, 0, 4096));
    hipLaunchKernelGGL(k_xcc, dim3(64), dim3(64), 0, 0, o);
    Out h;
    CHK(hipMemcpy(&h, o, sizeof(Out), hipMemcpyDeviceToHost));
    // partner blocks: same XCC as block 0 (other than 0), and a different XCC
    int same = -1, other = -1;
    for (int b = 1; b < 64; ++b) {
        if (h.xcc[b] == h.xcc[0] && same < 0) same = b;
        if (h.xcc[b] != h.xcc[0] && other < 0) other = b;
    }
    printf("xcc of blocks 0..15:");
    for (int b = 0; b < 16; ++b) printf(" %u", h.xcc[b]);
    printf("\nsame-XCC partner %d, other-XCC partner %d\n", same, other);
    if (same < 0 || other < 0) return 1;
    // slots: 0 sc1/same 1 sc1/other 2 plain+nt/same 3 plain+nt/other 4 wg-xchg+nt/same 5 wg-xchg+nt/other
    // (placement is re-checked per launch: a block's XCC is read again)
    hipLaunchKernelGGL(k_pp<0>, dim3(64), dim3(64), 0, 0, flags, o, 0, same, 0);
    hipLaunchKernelGGL(k_pp<0>, dim3(64), dim3(64), 0, 0, flags, o, 0, other, 1);
    hipLaunchKernelGGL(k_pp<1>, dim3(64), dim3(64), 0, 0, flags, o, 0, same, 2);
    hipLaunchKernelGGL(k_pp<1>, dim3(64), dim3(64), 0, 0, flags, o, 0, other, 3);
    hipLaunchKernelGGL(k_pp<2>, dim3(64), dim3(64), 0, 0, flags, o, 0, same, 4);
    hipLaunchKernelGGL(k_pp<2>, dim3(64), dim3(64), 0, 0, flags, o, 0, other, 5);
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, w, flags + 2048, o);
    hipLaunchKernelGGL(k_xcc, dim3(64), dim3(64), 0, 0, o);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(&h, o, sizeof(Out), hipMemcpyDeviceToHost));
    const char *nm[6] = {"sc1 store / sc1 poll, same XCC", "sc1 store / sc1 poll, other XCC",
                         "plain store / nt poll, same XCC", "plain store / nt poll, other XCC",
                         "wg-scope xchg / nt poll, same XCC", "wg-scope xchg / nt poll, other XCC"};
    for (int s = 0; s < 6; ++s) {
        printf("[xcc %u,%u] ", h.pair[2 * s] - 1, h.pair[2 * s + 1] - 1);
        if (h.fail[s] || h.fail[s + 8])
            printf("%-36s stale (round %u / %u)\n", nm[s], h.fail[s], h.fail[s + 8]);
        else
            printf("%-36s %8.0f cycles per round trip\n", nm[s], (double)h.t[s] / ROUNDS);
    }
    const char *cn[5] = {"atomicAdd agent (returning)", "atomicAdd workgroup scope", "load sc1 (dependent)",
                         "load nt (dependent)", "load plain volatile (dependent)"};
    for (int s = 0; s < 5; ++s) printf("%-36s %8.0f cycles each\n", cn[s], (double)h.t[8 + s] / ROUNDS);
    return 0;
}
