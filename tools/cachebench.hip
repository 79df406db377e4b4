// cachebench.hip -- where in-place message traffic is served from on MI355X
// (not part of the product).  The resident pool runs every phase as an
// in-place read-modify-write of the pool's messages; this measures the rate
// of that access shape against the working-set size, to find the size below
// which the L2 (4 MB per XCD) or the Infinity Cache (256 MB) serves it.
//
//   rows : one wave reads 72 x 512 B contiguous segments, then rewrites them
//          (the check kernel's shape)
//   cols : one wave reads 8 x 512 B segments at random positions of its
//          64-codeword tile, then rewrites them (the variable kernel's shape)
//   launch  : one pass per kernel launch, launches back to back
//   persist : one launch making R passes (a block always touches the same
//             data, so its XCD's L2 could keep it between passes)
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/cachebench tools/cachebench.hip
//   tools/cachebench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

template <int SEG>
__global__ __launch_bounds__(256, 2) void rows_rmw(double* a, size_t nwaves, int passes)
{
    const int lane = threadIdx.x & 63;
    for (int p = 0; p < passes; p++) {
        for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < nwaves; w += (size_t)gridDim.x * 4) {
            double* s = a + w * SEG * 64 + lane;
            double x[SEG];
#pragma unroll
            for (int k = 0; k < SEG; k++) x[k] = s[k * 64];
#pragma unroll
            for (int k = 0; k < SEG; k++) s[k * 64] = x[k] * 1.0000001 + 1e-300;
        }
    }
}

// the same shapes with two codewords per lane (16 B per lane, 1024 B per
// wave-segment): half the memory instructions per byte
template <int SEG>
__global__ __launch_bounds__(256, 2) void rows_rmw2(double2* a, size_t nwaves)
{
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    double2* s = a + w * SEG * 64 + lane;
    double2 x[SEG];
#pragma unroll
    for (int k = 0; k < SEG; k++) x[k] = s[k * 64];
#pragma unroll
    for (int k = 0; k < SEG; k++) s[k * 64] = make_double2(x[k].x * 1.0000001 + 1e-300, x[k].y * 1.0000001 + 1e-300);
}

__global__ __launch_bounds__(256) void cols_rmw2(double2* a, const int* __restrict__ idx, size_t nwaves, size_t nseg)
{
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const size_t tile = (w * 8) / nseg;
    double2 v[8];
    size_t o[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        o[s] = ((size_t)idx[(w * 8 + s) % nseg] + tile * nseg) * 64 + lane;
        v[s] = a[o[s]];
    }
#pragma unroll
    for (int s = 0; s < 8; s++) a[o[s]] = make_double2(v[s].x * 1.5 + 1e-300, v[s].y * 1.5 + 1e-300);
}

// var shape: segment ids of one tile are a random permutation; wave w of a
// tile takes 8 of them
__global__ __launch_bounds__(256) void cols_rmw(double* a, const int* __restrict__ idx, size_t nwaves, size_t nseg,
                                                int passes)
{
    const int lane = threadIdx.x & 63;
    for (int p = 0; p < passes; p++) {
        for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < nwaves; w += (size_t)gridDim.x * 4) {
            const size_t tile = (w * 8) / nseg;
            double v[8];
            size_t o[8];
#pragma unroll
            for (int s = 0; s < 8; s++) {
                o[s] = ((size_t)idx[(w * 8 + s) % nseg] + tile * nseg) * 64 + lane;
                v[s] = a[o[s]];
            }
#pragma unroll
            for (int s = 0; s < 8; s++) a[o[s]] = v[s] * 1.5 + 1e-300;
        }
    }
}

int main(int argc, char** argv)
{
    const size_t maxb = (size_t)2048 << 20;
    double* a;
    CK(hipMalloc(&a, maxb));
    CK(hipMemset(a, 0, maxb));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // per-"tile" segment permutation (as the 64-codeword tile's E edges), scaled to the buffer
    const size_t E = 147456;
    std::vector<int> h(E);
    for (size_t i = 0; i < E; i++) h[i] = (int)i;
    srand(1);
    for (size_t i = E - 1; i > 0; i--) { size_t j = (size_t)rand() % (i + 1); std::swap(h[i], h[j]); }
    int* idx;
    CK(hipMalloc(&idx, E * 4));
    CK(hipMemcpy(idx, h.data(), E * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (argc > 1 && std::string(argv[1]) == "calib") {
        // PMC calibration (tools/gpu_pmc_r2.sh): one in-place pass of the check
        // kernel's shape (72 x 512 B read, then rewritten, per wave) over 2048 MB
        // (HBM) and over 64 MB (Infinity Cache after the first pass): known
        // bytes, 2048 / 64 MB read and the same written, per dispatch
        for (double mb : {2048.0, 64.0}) {
            const size_t nw = (size_t)(mb * (1 << 20)) / 512 / 72;
            for (int r = 0; r < 3; r++)
                hipLaunchKernelGGL(rows_rmw<72>, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, a, nw, 1);
            CK(hipDeviceSynchronize());
            std::printf("calib %.0f MB: %zu waves, %.0f bytes read + written per dispatch\n", mb, nw, (double)nw * 72 * 512);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "wide") {
        // one pass per launch, 8 B vs 16 B per lane, same bytes
        std::printf("%8s %10s %10s %10s %10s\n", "MB", "rows72x8", "rows72x16", "cols8x8", "cols8x16");
        for (double mb : {96.0, 128.0, 160.0, 192.0, 224.0, 256.0, 2048.0}) {
            const size_t nseg_tot = (size_t)(mb * (1 << 20)) / 512;
            double gbs[4];
            for (int v = 0; v < 4; v++) {
                const bool wide = v & 1, rows = v < 2;
                const size_t segs = wide ? nseg_tot / 2 : nseg_tot;  // 1024 B segments when wide
                const size_t nseg = segs < E ? segs : E;
                const size_t nw = rows ? segs / 72 : (segs / nseg) * nseg / 8;
                const double bytes = 2.0 * (double)nw * (rows ? 72 : 8) * (wide ? 1024 : 512);
                const unsigned grid = (unsigned)((nw + 3) / 4);
                auto go = [&]() {
                    if (rows && !wide) hipLaunchKernelGGL(rows_rmw<72>, dim3(grid), dim3(256), 0, 0, a, nw, 1);
                    else if (rows) hipLaunchKernelGGL(rows_rmw2<72>, dim3(grid), dim3(256), 0, 0, (double2*)a, nw);
                    else if (!wide) hipLaunchKernelGGL(cols_rmw, dim3(grid), dim3(256), 0, 0, a, idx, nw, nseg, 1);
                    else hipLaunchKernelGGL(cols_rmw2, dim3(grid), dim3(256), 0, 0, (double2*)a, idx, nw, nseg);
                };
                const int reps = 30;
                go(); go();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (int r = 0; r < reps; r++) go();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                gbs[v] = bytes * reps / (ms * 1e-3) / 1e9;
            }
            std::printf("%8.0f %10.1f %10.1f %10.1f %10.1f\n", mb, gbs[0], gbs[1], gbs[2], gbs[3]);
            std::fflush(stdout);
        }
        return 0;
    }
    const double mbs[] = {4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 512, 2048};
    std::printf("cus %d\n", cus);
    std::printf("%8s %10s %10s %10s %10s %10s %10s\n", "MB", "rows72_l", "rows72_p", "rows8_l", "rows8_p", "cols_l",
                "cols_p");
    for (double mb : mbs) {
        // rows: whole 72-segment waves; cols: the segment ids of a tile are
        // [0, E): use nseg = min(E, segments in the buffer)
        const size_t nseg_tot = (size_t)(mb * (1 << 20)) / 512;
        const size_t nw_r72 = nseg_tot / 72, nw_r8 = nseg_tot / 8;
        const size_t nseg = nseg_tot < E ? nseg_tot : E;
        const size_t ntiles = nseg_tot / nseg;
        const size_t nw_cols = ntiles * nseg / 8;
        double gbs[6];
        for (int v = 0; v < 6; v++) {
            const int shape = v / 2;  // 0 rows72, 1 rows8, 2 cols
            const bool pers = v & 1;
            const size_t nw = shape == 0 ? nw_r72 : shape == 1 ? nw_r8 : nw_cols;
            const double bytes = 2.0 * (double)nw * (shape == 0 ? 72 : 8) * 512;
            const unsigned grid = pers ? (unsigned)(cus * (shape == 0 ? 2 : 4)) : (unsigned)((nw + 3) / 4);
            const int reps = 20;
            auto go = [&](int passes) {
                if (shape == 0) hipLaunchKernelGGL(rows_rmw<72>, dim3(grid), dim3(256), 0, 0, a, nw, passes);
                else if (shape == 1) hipLaunchKernelGGL(rows_rmw<8>, dim3(grid), dim3(256), 0, 0, a, nw, passes);
                else hipLaunchKernelGGL(cols_rmw, dim3(grid), dim3(256), 0, 0, a, idx, nw, nseg, passes);
            };
            if (pers) go(2); else { go(1); go(1); }
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            if (pers) go(reps); else for (int r = 0; r < reps; r++) go(1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            gbs[v] = bytes * reps / (ms * 1e-3) / 1e9;
        }
        std::printf("%8.0f %10.1f %10.1f %10.1f %10.1f %10.1f %10.1f\n", mb, gbs[0], gbs[1], gbs[2], gbs[3], gbs[4],
                    gbs[5]);
        std::fflush(stdout);
    }
    return 0;
}
