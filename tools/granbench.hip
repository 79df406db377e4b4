// granbench.hip -- throughput of the variable phase's access pattern as a
// function of the contiguous block size: each "column" reads 8 blocks at
// random positions of a cache-sized buffer (the c2v scratch) and writes 8
// blocks at random positions of a large buffer (the d stream, nontemporal).
// A block is P x 512 B (P tiles of 64 fp64 lanes interleaved); the P waves of
// one column each move 512 B of it.
//   hipcc --offload-arch=gfx950 -O3 -o tools/granbench tools/granbench.hip
//   tools/granbench [big_GB=4] [small_MB=226]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

template <int P, int MODE>  // MODE 0: read+write, 1: read only, 2: write only, 3: read+write + the BP variable arithmetic
__global__ __launch_bounds__(256) void k_gran(const double* __restrict__ small_buf, double* __restrict__ big_buf,
                                              const int32_t* __restrict__ rperm, const int32_t* __restrict__ wperm,
                                              int64_t ncols, double* __restrict__ sink)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t col = (int64_t)blockIdx.x * (4 / P) + w / P;
    const int part = w % P;
    if (col >= ncols) return;
    double v[8];
    double acc = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (MODE != 2) {
            const int64_t b = rperm[col * 8 + s];
            v[s] = small_buf[(b * P + part) * 64 + lane];
        } else {
            v[s] = (double)s;
        }
        acc += v[s];
    }
    if (MODE == 3) {  // forward/backward products + 1 - 2/(1+v) per edge, as k_var_m
        double pr[8], p = 1.0 + acc * 1e-9, a2 = 1.0;
#pragma unroll
        for (int s = 0; s < 8; ++s) { pr[s] = p; p = p * (1.0 + v[s]); }
#pragma unroll
        for (int s = 7; s >= 0; --s) {
            double x = pr[s] * a2;
            if (__builtin_isnan(x)) x = 1.0;
            a2 = a2 * (1.0 + v[s]);
            v[s] = 1.0 - 2.0 / (1.0 + x);
        }
        acc = p;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (MODE != 1) {
            const int64_t b = wperm[col * 8 + s];
            __builtin_nontemporal_store(v[s] + acc, &big_buf[(b * P + part) * 64 + lane]);
        }
    }
    if (MODE == 1 && acc == 12345.678) sink[0] = acc;
}

template <int P, int MODE>
static float run(const double* sb, double* bb, const int32_t* rp, const int32_t* wp, int64_t ncols, double* sink)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned blocks = (unsigned)((ncols + (4 / P) - 1) / (4 / P));
    hipLaunchKernelGGL((k_gran<P, MODE>), dim3(blocks), dim3(256), 0, 0, sb, bb, rp, wp, ncols, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; r++)
        hipLaunchKernelGGL((k_gran<P, MODE>), dim3(blocks), dim3(256), 0, 0, sb, bb, rp, wp, ncols, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

template <int P>
static void sweep(double big_gb, double small_mb)
{
    const int64_t blk_bytes = 512LL * P;
    const int64_t nbig = (int64_t)(big_gb * 1e9) / blk_bytes;
    const int64_t nsmall = (int64_t)(small_mb * 1e6) / blk_bytes;
    // one column per 8 written blocks of the big buffer; reads cycle the small one
    const int64_t ncols = nbig / 8;
    std::mt19937_64 rng(1);
    std::vector<int32_t> wperm(nbig), rperm(ncols * 8);
    std::iota(wperm.begin(), wperm.end(), 0);
    std::shuffle(wperm.begin(), wperm.end(), rng);
    for (int64_t i = 0; i < ncols * 8; i++) rperm[i] = (int32_t)(rng() % nsmall);
    double *sb, *bb, *sink;
    int32_t *rp, *wp;
    CK(hipMalloc(&sb, nsmall * blk_bytes));
    CK(hipMalloc(&bb, nbig * blk_bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&rp, rperm.size() * 4));
    CK(hipMalloc(&wp, wperm.size() * 4));
    CK(hipMemcpy(rp, rperm.data(), rperm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wp, wperm.data(), wperm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(sb, 0, nsmall * blk_bytes));
    const double bytes_rw = (double)ncols * 8 * blk_bytes;
    const float t0 = run<P, 0>(sb, bb, rp, wp, ncols, sink);
    const float t1 = run<P, 1>(sb, bb, rp, wp, ncols, sink);
    const float t2 = run<P, 2>(sb, bb, rp, wp, ncols, sink);
    const float t3 = run<P, 3>(sb, bb, rp, wp, ncols, sink);
    std::printf("block %5lld B: read+write %7.1f GB/s   read-only %7.1f GB/s   write-only %7.1f GB/s   "
                "read+BP-arith+write %7.1f GB/s\n",
                (long long)blk_bytes, 2 * bytes_rw / (t0 * 1e-3) / 1e9, bytes_rw / (t1 * 1e-3) / 1e9,
                bytes_rw / (t2 * 1e-3) / 1e9, 2 * bytes_rw / (t3 * 1e-3) / 1e9);
    CK(hipFree(sb)); CK(hipFree(bb)); CK(hipFree(sink)); CK(hipFree(rp)); CK(hipFree(wp));
}

int main(int argc, char** argv)
{
    const double big = argc > 1 ? std::atof(argv[1]) : 4.0;
    const double small = argc > 2 ? std::atof(argv[2]) : 226.0;
    std::printf("random 8-block gathers from a %.0f MB buffer, 8-block scatters into %.1f GB (nontemporal)\n", small,
                big);
    sweep<1>(big, small);
    sweep<2>(big, small);
    sweep<4>(big, small);
    return 0;
}
