// fp64bench.hip -- the BP check row's arithmetic without memory traffic (not
// part of the product).  Is k_check_bp bound by its fp64 work at two waves
// per SIMD (its occupancy), or by memory?  Each lane holds a row's 72 d
// values in registers and runs check_bp_compute's operation sequence
// (prefix products with 8-edge checkpoints, backward suffix, 72 IEEE
// divisions (1+t)/(1-t)) R times; one wave per (row, tile) as the kernel.
// Reports ns per wave-row at the kernel's occupancy (launch_bounds(256, 2))
// and the same for the division alone and the products alone.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/fp64bench tools/fp64bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

constexpr int DC = 72;

template <int MODE>  // 0: the full row (check_bp_compute), 1: divisions only, 2: products only
__global__ __launch_bounds__(256, 2) void k_row(const double* __restrict__ in, double* __restrict__ out, int reps)
{
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    double x[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) x[k] = in[(g * 7 + k) & 4095];
    double acc = 0.0;
    for (int r = 0; r < reps; ++r) {
        // opaque: the row's values are "new" every repetition (nothing hoisted)
#pragma unroll
        for (int k = 0; k < DC; ++k) asm volatile("" : "+v"(x[k]));
        constexpr int SEG = 8, NSEG = DC / SEG;
        if constexpr (MODE == 0 || MODE == 2) {
            double cp[NSEG];
            double p = 1.0;
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                if (k % SEG == 0) cp[k / SEG] = p;
                p = p * x[k];
            }
            double s = 1.0;
#pragma unroll
            for (int gi = NSEG - 1; gi >= 0; --gi) {
                double pk[SEG];
                double q = cp[gi];
                asm volatile("" : "+v"(q));
#pragma unroll
                for (int i = 0; i < SEG; ++i) { pk[i] = q; q = q * x[gi * SEG + i]; }
#pragma unroll
                for (int i = SEG - 1; i >= 0; --i) {
                    const double tt = pk[i] * s;
                    if constexpr (MODE == 0) acc += (1.0 + tt) / (1.0 - tt);
                    else acc += (1.0 + tt) * (1.0 - tt);
                    s = s * x[gi * SEG + i];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                const double tt = x[k] * 0.5;
                acc += (1.0 + tt) / (1.0 - tt);
            }
        }
        asm volatile("" : "+v"(acc));
    }
    out[g] = acc;
}

template <int MODE>
static float run(const double* in, double* out, int blocks, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_row<MODE>, dim3(blocks), dim3(256), 0, 0, in, out, 1);  // warm-up
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_row<MODE>, dim3(blocks), dim3(256), 0, 0, in, out, reps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main()
{
    double *in, *out;
    const int blocks = 256 * 2 * 4;  // 2 waves per SIMD on every SIMD: 8192 waves
    CK(hipMalloc(&in, 4096 * 8));
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    double h[4096];
    for (int i = 0; i < 4096; i++) h[i] = 0.9 - 1.8 * ((i * 2654435761u) % 1000) / 1000.0;  // d in (-0.9, 0.9]
    CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
    const int reps = 64;
    const double waves = (double)blocks * 4;
    const char* names[] = {"check row (72 div + products)", "72 divisions only", "products, no division"};
    float ms[3] = {run<0>(in, out, blocks, reps), run<1>(in, out, blocks, reps), run<2>(in, out, blocks, reps)};
    for (int m = 0; m < 3; m++) {
        // wave-rows per SIMD in flight: 2; ns per wave-row = time / (wave-rows per SIMD)
        const double per_simd = waves * reps / 1024.0;
        std::printf("%-32s %8.3f ms  %7.1f ns per wave-row per SIMD  (%.1f us for the 6 wave-rows per SIMD of a 3-tile check launch)\n",
                    names[m], ms[m], ms[m] * 1e6 / per_simd, ms[m] * 1e6 / per_simd * 6 / 1e3);
    }
    return 0;
}
