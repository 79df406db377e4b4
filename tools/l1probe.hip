// l1probe.hip -- L1 coherence between CUs of one XCD (not part of the product).
// Consumer block (XCD 0) caches a line in its L1, the producer block (same
// XCD) rewrites it and raises a flag (device atomic); the consumer then
// re-reads the line with each load variant and counts stale values.  Then the
// read rate of a 2 MB table (L2-resident for one XCD) per variant, to see
// which variants still hit the L2.
//   hipcc --offload-arch=gfx950 -O3 -o tools/l1probe tools/l1probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int V>
__device__ __forceinline__ unsigned long long ld(const unsigned long long* p)
{
    unsigned long long r;
    if constexpr (V == 0) asm volatile("global_load_dwordx2 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 1) asm volatile("global_load_dwordx2 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 2) asm volatile("global_load_dwordx2 %0, %1, off nt\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 3) asm volatile("global_load_dwordx2 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 4) asm volatile("global_load_dwordx2 %0, %1, off sc0 nt\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 5) asm volatile("buffer_inv sc0\n global_load_dwordx2 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 6) asm volatile("buffer_inv sc1\n global_load_dwordx2 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    if constexpr (V == 7) asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// block 0 = consumer, block 8 = producer (both XCD 0); rounds r = 0..R-1 on line r
template <int V>
__global__ void coh(unsigned long long* data, unsigned long long* flag, unsigned long long* stale, int R)
{
    if (threadIdx.x != 0) return;
    if (blockIdx.x == 0) {
        unsigned long long bad = 0;
        for (int r = 0; r < R; r++) {
            unsigned long long* p = data + (size_t)r * 16;
            const unsigned long long v0 = ld<0>(p);  // cache it in this CU's L1 (plain load)
            asm volatile("" ::"v"(v0));
            atomicAdd(flag, 1ull);  // ready: 2r+1
            while (atomicAdd(flag, 0ull) < 2ull * r + 2) __builtin_amdgcn_s_sleep(1);
            const unsigned long long v = ld<V>(p);
            bad += v != (unsigned long long)(r + 1) * 1000;
        }
        *stale = bad;
    } else if (blockIdx.x == 8) {
        for (int r = 0; r < R; r++) {
            unsigned long long* p = data + (size_t)r * 16;
            while (atomicAdd(flag, 0ull) < 2ull * r + 1) __builtin_amdgcn_s_sleep(1);
            *p = (unsigned long long)(r + 1) * 1000;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long o = atomicAdd(flag, 1ull);  // written: 2r+2
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");
        }
    }
}

// read rate: XCD 0's blocks (b % 8 == 0) sweep a 2 MB table `passes` times
template <int V>
__global__ __launch_bounds__(256) void rate(const unsigned long long* t, size_t n, int passes, unsigned long long* sink)
{
    if (blockIdx.x % 8 != 0) return;
    const size_t nb = gridDim.x / 8, b = blockIdx.x / 8;
    unsigned long long acc = 0;
    for (int p = 0; p < passes; p++)
        for (size_t i = b * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) acc += ld<V>(t + i);
    if (acc == 42) *sink = acc;
}

template <int V>
void run(unsigned long long* data, unsigned long long* flag, unsigned long long* d_stale, unsigned long long* tab,
         unsigned long long* sink)
{
    const int R = 2000;
    hipMemset(data, 0, (size_t)R * 128);
    hipMemset(flag, 0, 8);
    hipLaunchKernelGGL(coh<V>, dim3(16), dim3(64), 0, 0, data, flag, d_stale, R);
    unsigned long long st = 0;
    hipMemcpy(&st, d_stale, 8, hipMemcpyDeviceToHost);
    const size_t n = (2u << 20) / 8;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(rate<V>, dim3(256), dim3(256), 0, 0, tab, n, 2, sink);
    hipEventRecord(a);
    hipLaunchKernelGGL(rate<V>, dim3(256), dim3(256), 0, 0, tab, n, 50, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::printf("variant %d: stale %llu / %d   2 MB table x50 on one XCD: %.1f GB/s\n", V, st, R,
                50.0 * n * 8 / (ms * 1e-3) / 1e9);
}

int main()
{
    unsigned long long *data, *flag, *st, *tab, *sink;
    hipMalloc(&data, 2000 * 128);
    hipMalloc(&flag, 8);
    hipMalloc(&st, 8);
    hipMalloc(&tab, 2u << 20);
    hipMalloc(&sink, 8);
    hipMemset(tab, 1, 2u << 20);
    run<0>(data, flag, st, tab, sink);
    run<1>(data, flag, st, tab, sink);
    run<2>(data, flag, st, tab, sink);
    run<3>(data, flag, st, tab, sink);
    run<4>(data, flag, st, tab, sink);
    run<5>(data, flag, st, tab, sink);
    run<6>(data, flag, st, tab, sink);
    run<7>(data, flag, st, tab, sink);
    return 0;
}
