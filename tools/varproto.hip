// varproto.hip -- the variable phase's ingredients added one at a time to a
// plain gather/scatter stream, to find what separates k_var_m (~5.7 TB/s of
// algorithmic traffic) from the bare pattern (~6.6 TB/s, layoutbench):
//   F_PRIOR : contiguous 512 B prior read per column
//   F_ARITH : BP forward/backward products and 1 - 2/(1+v)
//   F_BALLOT: hard-decision ballot store (8 B per column by lane 0)
//   CPW     : columns per wave, all loads issued first
// Scratch (c2v) 226 MB, d stream / prior as large HBM buffers.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/varproto tools/varproto.hip
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

constexpr int DV = 8;

template <int CPW, bool F_PRIOR, bool F_ARITH, bool F_BALLOT, bool NTP = false>
__global__ __launch_bounds__(256) void k_proto(const double* __restrict__ c2v, double* __restrict__ d,
                                               const double* __restrict__ prior, uint64_t* __restrict__ hard,
                                               const int32_t* __restrict__ col_edge, int32_t ncols)
{
    const int lane = threadIdx.x & 63;
    const int32_t j0 = (int32_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * CPW;
    if (j0 >= ncols) return;
    int32_t eid[CPW][DV];
    double l[CPW][DV], pv[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int s = 0; s < DV; ++s) eid[c][s] = col_edge[(size_t)(j0 + c) * DV + s];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        pv[c] = F_PRIOR ? (NTP ? __builtin_nontemporal_load(&prior[(size_t)(j0 + c) * 64 + lane])
                               : prior[(size_t)(j0 + c) * 64 + lane])
                        : 1.0;
#pragma unroll
        for (int s = 0; s < DV; ++s) l[c][s] = c2v[(size_t)eid[c][s] * 64 + lane];
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        double dv[DV];
        bool h = false;
        if (F_ARITH) {
            double pr[DV], p = pv[c];
#pragma unroll
            for (int s = 0; s < DV; ++s) { pr[s] = p; p = p * l[c][s]; }
            if (__builtin_isnan(p)) p = 1.0;
            h = p <= 1.0;
            double acc = 1.0;
#pragma unroll
            for (int s = DV - 1; s >= 0; --s) {
                double v = pr[s] * acc;
                if (__builtin_isnan(v)) v = 1.0;
                acc = acc * l[c][s];
                dv[s] = 1.0 - 2.0 / (1.0 + v);
            }
        } else {
#pragma unroll
            for (int s = 0; s < DV; ++s) dv[s] = l[c][s] + pv[c];
        }
#pragma unroll
        for (int s = 0; s < DV; ++s) __builtin_nontemporal_store(dv[s], &d[(size_t)eid[c][s] * 64 + lane]);
        if (F_BALLOT) {
            const uint64_t m = __ballot(h);
            if (lane == 0) hard[j0 + c] = m;
        }
    }
}

template <int CPW, bool A, bool B, bool C, bool NTP = false>
static void run(const char* name, const double* c2v, double* d, const double* prior, uint64_t* hard, const int32_t* ce,
                int32_t ncols, double alg_bytes)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned blocks = (unsigned)((ncols / CPW + 3) / 4);
    hipLaunchKernelGGL((k_proto<CPW, A, B, C, NTP>), dim3(blocks), dim3(256), 0, 0, c2v, d, prior, hard, ce, ncols);
    CK(hipEventRecord(a));
    for (int r = 0; r < 10; r++)
        hipLaunchKernelGGL((k_proto<CPW, A, B, C, NTP>), dim3(blocks), dim3(256), 0, 0, c2v, d, prior, hard, ce, ncols);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 10;
    std::printf("%-40s %7.4f ms  %7.1f GB/s\n", name, ms, alg_bytes / (ms * 1e-3) / 1e9);
}

int main()
{
    // 3 tiles of the DNA code's shape: E = 147456 edges, N = 18432 columns per tile
    const int32_t N = 18432, E = 147456, T = 3;
    const int32_t ncols = N * T;
    std::mt19937_64 rng(5);
    std::vector<int32_t> perm((size_t)E * T);
    std::iota(perm.begin(), perm.end(), 0);
    // edges of a tile stay in that tile's block (as in the engine)
    for (int t = 0; t < T; t++) std::shuffle(perm.begin() + (size_t)t * E, perm.begin() + (size_t)(t + 1) * E, rng);
    double *c2v, *d, *prior;
    uint64_t* hard;
    int32_t* ce;
    CK(hipMalloc(&c2v, (size_t)E * T * 512));
    CK(hipMalloc(&d, (size_t)E * T * 512 * 40));  // d stream: the tiles sit inside a larger buffer
    CK(hipMalloc(&prior, (size_t)N * T * 512 * 40));
    CK(hipMalloc(&hard, (size_t)N * T * 8));
    CK(hipMalloc(&ce, perm.size() * 4));
    CK(hipMemcpy(ce, perm.data(), perm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(c2v, 0, (size_t)E * T * 512));
    CK(hipMemset(prior, 0, (size_t)N * T * 512));
    const double alg = (double)T * (16.0 * E + 8.0 * N + N / 8.0) * 64;  // the bench's per-tile algorithmic bytes
    std::printf("variable-phase prototypes on %d tiles (c2v %.0f MB); GB/s = algorithmic bytes / time\n", T,
                E * T * 512 / 1e6);
    run<1, false, false, false>("bare gather/scatter, 1 col/wave", c2v, d, prior, hard, ce, ncols, alg);
    run<1, true, false, false>("+prior", c2v, d, prior, hard, ce, ncols, alg);
    run<1, true, true, false>("+prior +arith", c2v, d, prior, hard, ce, ncols, alg);
    run<1, true, true, true>("+prior +arith +ballot (1 col/wave)", c2v, d, prior, hard, ce, ncols, alg);
    run<2, true, true, true>("full, 2 col/wave", c2v, d, prior, hard, ce, ncols, alg);
    run<4, true, true, true>("full, 4 col/wave", c2v, d, prior, hard, ce, ncols, alg);
    run<8, true, true, true>("full, 8 col/wave", c2v, d, prior, hard, ce, ncols, alg);
    run<4, false, false, false>("bare, 4 col/wave", c2v, d, prior, hard, ce, ncols, alg);
    run<1, true, false, false, true>("+prior (nontemporal)", c2v, d, prior, hard, ce, ncols, alg);
    run<4, true, true, true, true>("full, 4 col/wave, nontemporal prior", c2v, d, prior, hard, ce, ncols, alg);
    run<1, true, true, true, true>("full, 1 col/wave, nontemporal prior", c2v, d, prior, hard, ce, ncols, alg);
    return 0;
}
