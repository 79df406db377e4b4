// xccprobe.hip -- which XCD a workgroup runs on (not part of the product):
// HW_REG_XCC_ID per block against blockIdx % 8, for a 1-block-per-CU grid
// (150 KB of LDS per block, as the XCD-resident decoder) and a 2048-block grid.
//   hipcc --offload-arch=gfx950 -O3 -o tools/xccprobe tools/xccprobe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256, 1) void big(unsigned* out)
{
    __shared__ double s[18000];
    unsigned x, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    s[threadIdx.x] = x;
    __syncthreads();
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = (unsigned)s[0]; out[2 * blockIdx.x + 1] = hw; }
}
__global__ void small(unsigned* out)
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) out[2 * blockIdx.x] = x;
}

int main()
{
    unsigned* d;
    hipMalloc(&d, 2 * 4096 * 4);
    std::vector<unsigned> h(2 * 4096);
    for (int mode = 0; mode < 2; mode++) {
        const int nb = mode == 0 ? 256 : 2048;
        if (mode == 0) hipLaunchKernelGGL(big, dim3(nb), dim3(256), 0, 0, d);
        else hipLaunchKernelGGL(small, dim3(nb), dim3(64), 0, 0, d);
        hipMemcpy(h.data(), d, 2 * nb * 4, hipMemcpyDeviceToHost);
        int hist[16] = {0}, match = 0;
        for (int b = 0; b < nb; b++) {
            hist[h[2 * b] & 15]++;
            match += (int)((h[2 * b] & 15) == (unsigned)(b % 8));
        }
        std::printf("grid %d: raw[0..3] %#x %#x %#x %#x  hist", nb, h[0], h[2], h[4], h[6]);
        for (int i = 0; i < 16; i++) std::printf(" %d", hist[i]);
        std::printf("  xcc == block %% 8: %d / %d\n", match, nb);
        if (mode == 0) {
            std::printf("  hw_id of blocks 0..15:");
            for (int b = 0; b < 16; b++) std::printf(" %#x", h[2 * b + 1]);
            std::printf("\n");
        }
    }
    return 0;
}
