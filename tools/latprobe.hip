// latprobe.hip -- load latency by cache-policy variant (not part of the
// product): one lane chases a random cycle through a table, each load
// depending on the previous.  Table sizes: 16 KB (L1), 1 MB (L2), 64 MB
// (Infinity Cache), 1 GB (HBM).  Tells whether the L1-bypassing variants the
// XCD-resident decoder uses (nt, sc1) are served by the L2.
//   hipcc --offload-arch=gfx950 -O3 -o tools/latprobe tools/latprobe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

template <int V>
__device__ __forceinline__ unsigned ldx(const unsigned* p)
{
    unsigned r;
    if constexpr (V == 0) asm volatile("global_load_dword %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 1) asm volatile("global_load_dword %0, %1, off nt\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 2) asm volatile("global_load_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 3) asm volatile("global_load_dword %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 4) asm volatile("global_load_dword %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}

template <int V>
__global__ void chase(const unsigned* t, int steps, unsigned long long* out)
{
    if (threadIdx.x != 0) return;
    unsigned i = 0;
    for (int s = 0; s < 64; s++) i = ldx<V>(t + i);  // warm
    const unsigned long long c0 = clock64();
    for (int s = 0; s < steps; s++) i = ldx<V>(t + i);
    const unsigned long long c1 = clock64();
    out[0] = (c1 - c0) / steps;
    out[1] = i;
}

int main()
{
    const size_t sizes[] = {16u << 10, 1u << 20, 64u << 20, 1024u << 20};
    unsigned* d;
    hipMalloc(&d, 1024u << 20);
    unsigned long long* o;
    hipMalloc(&o, 16);
    for (size_t sz : sizes) {
        // random cycle over 128-B-spaced slots
        const size_t n = sz / 128;
        std::vector<unsigned> perm(n), tab(sz / 4, 0);
        for (size_t i = 0; i < n; i++) perm[i] = (unsigned)i;
        srand(7);
        for (size_t i = n - 1; i > 0; i--) std::swap(perm[i], perm[(size_t)rand() % (i + 1)]);
        for (size_t i = 0; i < n; i++) tab[(size_t)perm[i] * 32] = perm[(i + 1) % n] * 32;
        hipMemcpy(d, tab.data(), sz, hipMemcpyHostToDevice);
        std::printf("%8zu KB:", sz >> 10);
        unsigned long long h[2];
        const int steps = 4000;
#define RUN(V)                                                                  \
        hipLaunchKernelGGL(chase<V>, dim3(1), dim3(64), 0, 0, d, steps, o);     \
        hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);                             \
        std::printf("  v%d %4llu", V, h[0]);
        RUN(0) RUN(1) RUN(2) RUN(3) RUN(4)
        std::printf("  cycles/load (v0 plain, v1 nt, v2 sc1, v3 sc0 sc1, v4 sc0)\n");
    }
    return 0;
}
