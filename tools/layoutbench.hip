// layoutbench.hip -- the two decode phases' memory patterns under different
// edge layouts, as plain streams (no decode arithmetic):
//   check phase  : per row-wave, 72 blocks of 512 B read from the d stream
//                  (4 GB, HBM, nontemporal) and 72 blocks written to the c2v
//                  scratch (226 MB, Infinity-Cache sized)
//   variable     : per column-wave, 8 blocks read from the scratch and 8
//                  written to the d stream (nontemporal)
// Each side is either contiguous (CSR order for the check phase, CSC order
// for the variable phase) or scattered through a random permutation.
//   hipcc --offload-arch=gfx950 -O3 -o tools/layoutbench tools/layoutbench.hip
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

// DEG blocks per wave; read block k of wave w at rperm[w*DEG+k] (or w*DEG+k),
// write at wperm[...] (or w*DEG+k).  Reads are nontemporal from the big
// buffer (RBIG) or plain from the small one; writes the other way round.
template <int DEG, bool RSC, bool WSC, bool RBIG>
__global__ __launch_bounds__(256) void k_stream(const double* __restrict__ src, double* __restrict__ dst,
                                                const int32_t* __restrict__ rperm, const int32_t* __restrict__ wperm,
                                                int64_t nwaves, int64_t nsrc, int64_t ndst)
{
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    double v[DEG];
#pragma unroll
    for (int k = 0; k < DEG; ++k) {
        int64_t b = RSC ? rperm[w * DEG + k] : (w * DEG + k);  // < nsmall <= nsrc
        const double* p = src + b * 64 + lane;
        v[k] = RBIG ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < DEG; ++k) {
        int64_t b = WSC ? wperm[w * DEG + k] : (w * DEG + k);  // < nsmall <= ndst
        double* p = dst + b * 64 + lane;
        if (RBIG) *p = v[k] + 1.0;
        else __builtin_nontemporal_store(v[k] + 1.0, p);
    }
}

template <int DEG, bool RSC, bool WSC, bool RBIG>
static void run(const char* name, const double* src, double* dst, const int32_t* rp, const int32_t* wp, int64_t nwaves,
                int64_t nsrc, int64_t ndst)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned blocks = (unsigned)((nwaves + 3) / 4);
    hipLaunchKernelGGL((k_stream<DEG, RSC, WSC, RBIG>), dim3(blocks), dim3(256), 0, 0, src, dst, rp, wp, nwaves, nsrc, ndst);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; r++)
        hipLaunchKernelGGL((k_stream<DEG, RSC, WSC, RBIG>), dim3(blocks), dim3(256), 0, 0, src, dst, rp, wp, nwaves, nsrc,
                           ndst);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    const double bytes = 2.0 * nwaves * DEG * 512;
    std::printf("%-44s %7.3f ms  %7.1f GB/s (read+write)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv)
{
    const double big_gb = argc > 1 ? std::atof(argv[1]) : 4.0;
    const double small_mb = argc > 2 ? std::atof(argv[2]) : 226.0;
    const int64_t nbig = (int64_t)(big_gb * 1e9) / 512, nsmall = (int64_t)(small_mb * 1e6) / 512;
    double *big, *small;
    CK(hipMalloc(&big, nbig * 512));
    CK(hipMalloc(&small, nsmall * 512));
    CK(hipMemset(big, 0, nbig * 512));
    CK(hipMemset(small, 0, nsmall * 512));
    std::mt19937_64 rng(3);
    // one pass over the scratch per launch: nsmall blocks moved
    std::vector<int32_t> pbig(nsmall), psmall(nsmall);
    for (auto& x : pbig) x = (int32_t)(rng() % nbig);
    std::iota(psmall.begin(), psmall.end(), 0);
    std::shuffle(psmall.begin(), psmall.end(), rng);
    int32_t *d_pbig, *d_psmall;
    CK(hipMalloc(&d_pbig, nsmall * 4));
    CK(hipMalloc(&d_psmall, nsmall * 4));
    CK(hipMemcpy(d_pbig, pbig.data(), nsmall * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_psmall, psmall.data(), nsmall * 4, hipMemcpyHostToDevice));
    std::printf("d stream %.1f GB (HBM, nontemporal), scratch %.0f MB\n", big_gb, small_mb);
    const int64_t wc = nsmall / 72, wv = nsmall / 8;
    // check phase: read d (big) -> write scratch (small)
    run<72, false, false, true>("check: d contiguous -> scratch contiguous", big, small, d_pbig, d_psmall, wc, nbig, nsmall);
    run<72, true, false, true>("check: d scattered  -> scratch contiguous", big, small, d_pbig, d_psmall, wc, nbig, nsmall);
    run<72, false, true, true>("check: d contiguous -> scratch scattered", big, small, d_pbig, d_psmall, wc, nbig, nsmall);
    // variable phase: read scratch (small) -> write d (big)
    run<8, true, true, false>("var: scratch scattered -> d scattered", small, big, d_psmall, d_pbig, wv, nsmall, nbig);
    run<8, true, false, false>("var: scratch scattered -> d contiguous", small, big, d_psmall, d_pbig, wv, nsmall, nbig);
    run<8, false, true, false>("var: scratch contiguous -> d scattered", small, big, d_psmall, d_pbig, wv, nsmall, nbig);
    return 0;
}
