// tools/hostreg_probe.cpp -- what the ROCm runtime remembers about host pages across register /
// unregister / munmap / mmap, and around its own pinning of large pageable copies (DESIGN.md §6,
// the round-3 host-map fault).  Host-side only: no kernel ever reads host memory here, so a stale
// mapping shows up as an attribute, not as a GPU fault.
//   build: hipcc -O2 -o tools/hostreg_probe tools/hostreg_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

static void attrs(const char *what, void *p)
{
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    hipError_t e = hipPointerGetAttributes(&a, p);
    void *dp = nullptr;
    hipError_t e2 = hipHostGetDevicePointer(&dp, p, 0);
    printf("%-44s %p: attr %-22s type %d devptr %p hostptr %p | hipHostGetDevicePointer %s %p\n", what, p,
           hipGetErrorName(e), (int)a.type, a.devicePointer, a.hostPointer, hipGetErrorName(e2), dp);
    (void)hipGetLastError();
}

static void *map(size_t n, void *hint)
{
    void *p = mmap(hint, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        perror("mmap");
        exit(1);
    }
    memset(p, 1, n);
    return p;
}

int main()
{
    const size_t small = 12u << 20, big = 537u << 20;
    float *dev = nullptr;
    if (hipMalloc((void **)&dev, big) != hipSuccess) return 1;
    // (1) register, unregister, unmap; a new mapping at the same address
    void *a = map(small, nullptr);
    printf("hipHostRegister(A, mapped): %s\n", hipGetErrorName(hipHostRegister(a, small, hipHostRegisterMapped)));
    attrs("A registered", a);
    printf("hipHostUnregister(A): %s\n", hipGetErrorName(hipHostUnregister(a)));
    attrs("A unregistered", a);
    munmap(a, small);
    void *b = map(small, a);
    printf("B mapped at %s address as A\n", b == a ? "the SAME" : "a different");
    attrs("B (never registered)", b);
    // (2) registered, then the pages go away WITHOUT unregister (a cached registration)
    printf("hipHostRegister(B, mapped): %s\n", hipGetErrorName(hipHostRegister(b, small, hipHostRegisterMapped)));
    attrs("B registered", b);
    munmap(b, small);
    void *c = map(small, b);
    printf("C mapped at %s address as B (B still registered)\n", c == b ? "the SAME" : "a different");
    attrs("C (new pages, B's registration alive)", c);
    printf("hipHostRegister(C, mapped): %s\n", hipGetErrorName(hipHostRegister(c, small, hipHostRegisterMapped)));
    attrs("C after its own register", c);
    printf("hipHostUnregister(C): %s\n", hipGetErrorName(hipHostUnregister(c)));
    (void)hipGetLastError();
    munmap(c, small);
    // (3) a large pageable copy out (the runtime pins the destination itself), then the pages go away
    void *d = map(big, nullptr);
    printf("hipMemcpy D2H into pageable D (%zu MB): %s\n", big >> 20, hipGetErrorName(hipMemcpy(d, dev, big, hipMemcpyDeviceToHost)));
    attrs("D after the runtime's own pinned copy", d);
    munmap(d, big);
    void *e = map(big, d);
    printf("E mapped at %s address as D\n", e == d ? "the SAME" : "a different");
    attrs("E (new pages where D was)", e);
    printf("hipMemcpy D2H into E: %s\n", hipGetErrorName(hipMemcpy(e, dev, big, hipMemcpyDeviceToHost)));
    printf("hipHostRegister(E part, mapped): %s\n", hipGetErrorName(hipHostRegister(e, small, hipHostRegisterMapped)));
    attrs("E part registered", e);
    printf("hipHostUnregister(E part): %s\n", hipGetErrorName(hipHostUnregister(e)));
    (void)hipGetLastError();
    munmap(e, big);
    (void)hipFree(dev);
    printf("done\n");
    return 0;
}
