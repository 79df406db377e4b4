// membench.hip -- memory-pattern ceilings on MI355X for the decoder's access
// shapes (not part of the product).  Prints GB/s of moved bytes per pattern.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
//   tools/membench [GB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

template <bool NT>
__device__ __forceinline__ double ldd(const double* p) { if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; }
template <bool NT>
__device__ __forceinline__ void std_(double* p, double v) { if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v; }

// plain streaming copy, 8 B per lane
template <bool NT>
__global__ void copy_x2(const double* __restrict__ a, double* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        std_<NT>(b + i, ldd<NT>(a + i));
}

// 16 B per lane
__global__ void copy_x4(const double2* __restrict__ a, double2* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// check-kernel shape: one wave reads SEG x 512 B contiguous into registers,
// then writes SEG x 512 B contiguous (to a different buffer)
template <int SEG, bool NT>
__global__ __launch_bounds__(256) void rows_x2(const double* __restrict__ a, double* __restrict__ b, size_t nwaves)
{
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const int lane = threadIdx.x & 63;
    const double* src = a + w * SEG * 64 + lane;
    double* dst = b + w * SEG * 64 + lane;
    double x[SEG];
#pragma unroll
    for (int k = 0; k < SEG; k++) x[k] = ldd<NT>(src + k * 64);
    double s = 0;
#pragma unroll
    for (int k = 0; k < SEG; k++) s += x[k];
    asm volatile("" ::"v"(s));
#pragma unroll
    for (int k = 0; k < SEG; k++) std_<NT>(dst + k * 64, x[k] * 1.0000001);
}

// variable-kernel shape: one wave gathers 8 x 512 B segments at table
// positions and scatters 8 x 512 B segments to other table positions
template <bool NT>
__global__ __launch_bounds__(256) void cols_x2(const double* __restrict__ a, double* __restrict__ b,
                                               const int* __restrict__ idx, size_t nwaves, size_t nseg)
{
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const int lane = threadIdx.x & 63;
    const size_t tile = (w * 8) / nseg;  // segments grouped like [tile][E]
    double v[8];
#pragma unroll
    for (int s = 0; s < 8; s++) v[s] = a[((size_t)idx[(w * 8 + s) % nseg] + tile * nseg) * 64 + lane];
#pragma unroll
    for (int s = 0; s < 8; s++) std_<NT>(b + ((size_t)idx[(w * 8 + s) % nseg] + tile * nseg) * 64 + lane, v[s] * 1.5);
}

static float timeit(void (*fn)(void*), void* ctx, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    fn(ctx);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) fn(ctx);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

struct Ctx {
    double *a, *b;
    int* idx;
    size_t n, nseg;
};

// waves of the cols shape over the whole tiles of nseg segments the buffers hold
static size_t cols_waves(const Ctx* c)
{
    const size_t tiles = (c->n / 64) / c->nseg;
    return tiles * c->nseg / 8;
}

int main(int argc, char** argv)
{
    const double gb = argc > 1 ? std::atof(argv[1]) : 4.0;
    const size_t n = (size_t)(gb * 1e9 / 8) / (72 * 64) * (72 * 64);
    Ctx c;
    c.n = n;
    CK(hipMalloc(&c.a, n * 8));
    CK(hipMalloc(&c.b, n * 8));
    CK(hipMemset(c.a, 0, n * 8));
    CK(hipMemset(c.b, 0, n * 8));
    // a random permutation of the E = 147456 segment ids of one 64-codeword tile
    const size_t E = 147456;
    c.nseg = E;
    std::vector<int> h(E);
    for (size_t i = 0; i < E; i++) h[i] = (int)i;
    srand(1);
    for (size_t i = E - 1; i > 0; i--) { size_t j = (size_t)rand() % (i + 1); std::swap(h[i], h[j]); }
    CK(hipMalloc(&c.idx, E * 4));
    CK(hipMemcpy(c.idx, h.data(), E * 4, hipMemcpyHostToDevice));
    const double bytes = 2.0 * n * 8;
    struct T { const char* name; void (*fn)(void*); };
    T tests[] = {
        {"copy_x2", [](void* p) { auto* c = (Ctx*)p; hipLaunchKernelGGL(copy_x2<false>, dim3(8192), dim3(256), 0, 0, c->a, c->b, c->n); }},
        {"copy_x2_nt", [](void* p) { auto* c = (Ctx*)p; hipLaunchKernelGGL(copy_x2<true>, dim3(8192), dim3(256), 0, 0, c->a, c->b, c->n); }},
        {"copy_x4", [](void* p) { auto* c = (Ctx*)p; hipLaunchKernelGGL(copy_x4, dim3(8192), dim3(256), 0, 0, (const double2*)c->a, (double2*)c->b, c->n / 2); }},
        {"rows72_x2", [](void* p) { auto* c = (Ctx*)p; size_t nw = c->n / (72 * 64); hipLaunchKernelGGL((rows_x2<72, false>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, c->a, c->b, nw); }},
        {"rows72_x2_nt", [](void* p) { auto* c = (Ctx*)p; size_t nw = c->n / (72 * 64); hipLaunchKernelGGL((rows_x2<72, true>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, c->a, c->b, nw); }},
        {"rows8_x2", [](void* p) { auto* c = (Ctx*)p; size_t nw = c->n / (8 * 64); hipLaunchKernelGGL((rows_x2<8, false>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, c->a, c->b, nw); }},
        // whole tiles only: a segment id of the last, partial tile would address
        // past the buffers (round 6: a 16 GB run of the old bound faulted the GPU)
        {"cols8_x2", [](void* p) { auto* c = (Ctx*)p; size_t nw = cols_waves(c); hipLaunchKernelGGL((cols_x2<false>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, c->a, c->b, c->idx, nw, c->nseg); }},
        {"cols8_x2_nt", [](void* p) { auto* c = (Ctx*)p; size_t nw = cols_waves(c); hipLaunchKernelGGL((cols_x2<true>), dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, c->a, c->b, c->idx, nw, c->nseg); }},
    };
    std::printf("buffer %.2f GB each\n", n * 8 / 1e9);
    for (auto& t : tests) {
        const bool cols = t.name[0] == 'c' && t.name[1] == 'o' && t.name[2] == 'l';
        const double b = cols ? 2.0 * (double)cols_waves(&c) * 8 * 512 : bytes;
        float ms = timeit(t.fn, &c, 5);
        std::printf("%-14s %8.3f ms  %7.1f GB/s\n", t.name, ms, b / (ms * 1e-3) / 1e9);
    }
    // small working sets (Infinity Cache resident): rows/cols over 150 MB
    const size_t small = (size_t)(150e6 / 8) / (72 * 64) * (72 * 64);
    Ctx s = c;
    s.n = small;
    const double sbytes = 2.0 * small * 8;
    for (auto& t : tests) {
        const bool cols = t.name[0] == 'c' && t.name[1] == 'o' && t.name[2] == 'l';
        const double b = cols ? 2.0 * (double)cols_waves(&s) * 8 * 512 : sbytes;
        float ms = timeit(t.fn, &s, 20);
        std::printf("%-14s %8.4f ms  %7.1f GB/s  (150 MB working set)\n", t.name, ms, b / (ms * 1e-3) / 1e9);
    }
    return 0;
}
