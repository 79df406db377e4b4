// wrbench.hip -- write/read shape ceilings for the min-sum v2c stream
// (not part of the product).  The compressed min-sum keeps only v2c in fp64
// (8 B per edge and codeword, [tile][edge][64 lanes]); this measures, over a
// v2c-sized buffer, the two ways of laying it out:
//   CSR order (today): the variable kernel scatters a column's 8 segments of
//     512 B to random rows; the check kernel reads a row's 72 segments
//     contiguously (36 KB);
//   CSC order (the compressed min-sum's since round 4): the variable kernel
//     writes a column's 8 segments contiguously (4 KB; 8 KB per 2-column
//     wave); the check kernel gathers its 72 segments from random columns.
//   row-block-major (the compressed min-sum's on the DNA code since round 4,
//     at a 604 MB size = 8 tiles of the DNA code, E = 147456 segments each):
//     edge s of column j at s * N + j of its tile; the variable kernel's
//     wave order (1-D grid, block L -> tile L % 8, two columns per wave,
//     stores in (column, s) order) and the check kernel's (grid (M / 4, 8),
//     row r of row block s = r / 256 gathering its 72 columns ascending, a
//     random partition of the N columns into the block's 256 rows).
// Prints GB/s of moved bytes per pattern, nontemporal and plain.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/wrbench tools/wrbench.hip
//   tools/wrbench [MB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

template <bool NT>
__device__ __forceinline__ void stv(double* p, double v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__device__ __forceinline__ double ldv(const double* p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// one wave per group of SEG segments: segment k of wave w goes to seg[w*SEG+k]
// (a permutation of all segments: random or identity)
template <int SEG, bool NT>
__global__ __launch_bounds__(256) void write_segs(double* __restrict__ b, const int* __restrict__ seg, size_t nwaves, double v)
{
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < SEG; k++) stv<NT>(b + (size_t)seg[w * SEG + k] * 64 + lane, v + k);
}

template <int SEG, bool NT>
__global__ __launch_bounds__(256) void read_segs(const double* __restrict__ a, const int* __restrict__ seg, size_t nwaves,
                                                 double* __restrict__ out)
{
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const int lane = threadIdx.x & 63;
    double x[SEG];
#pragma unroll
    for (int k = 0; k < SEG; k++) x[k] = ldv<NT>(a + (size_t)seg[w * SEG + k] * 64 + lane);
    double s = 0;
#pragma unroll
    for (int k = 0; k < SEG; k++) s = s < x[k] ? x[k] : s;
    if (s == 12345.0) out[lane] = s;
}

template <typename F>
static float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv)
{
    const double mb = argc > 1 ? std::atof(argv[1]) : 1208.0;
    const size_t nseg = (size_t)(mb * 1e6 / 512) / 72 * 72;
    const size_t bytes = nseg * 512;
    double *buf, *out;
    int *ident, *rnd;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64 * 8));
    CK(hipMalloc(&ident, nseg * 4));
    CK(hipMalloc(&rnd, nseg * 4));
    CK(hipMemset(buf, 0, bytes));
    std::vector<int> h(nseg);
    for (size_t i = 0; i < nseg; i++) h[i] = (int)i;
    CK(hipMemcpy(ident, h.data(), nseg * 4, hipMemcpyHostToDevice));
    uint64_t x = 88172645463325252ull;
    for (size_t i = nseg - 1; i > 0; i--) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        std::swap(h[i], h[x % (i + 1)]);
    }
    CK(hipMemcpy(rnd, h.data(), nseg * 4, hipMemcpyHostToDevice));
    // row-block-major shapes of the DNA code (N = 18432, M = 2048, 8 row blocks), 8 tiles
    constexpr int NC = 18432, MR = 2048, DV = 8, DC = 72, RB = MR / DV;
    constexpr size_t ET = (size_t)NC * DV;
    int *rbw = nullptr, *rbr = nullptr;
    const bool rb = nseg % ET == 0;
    if (rb) {
        const size_t tiles = nseg / ET;
        std::vector<int> w(nseg), r(nseg);
        // variable kernel: wave v = block L * 4 + w4; tile L % tiles, columns j0, j0 + 1
        for (size_t v = 0; v < nseg / 16; v++) {
            const size_t L = v / 4, w4 = v % 4, ty = L % tiles, cb = L / tiles;
            const size_t j0 = (cb * 4 + w4) * 2;
            for (int c = 0; c < 2; c++)
                for (int sb = 0; sb < DV; sb++) w[v * 16 + c * DV + sb] = (int)(ty * ET + (size_t)sb * NC + j0 + c);
        }
        // check kernel: wave v = tile * M + row; row r of block r / RB reads its 72 columns ascending
        std::vector<int> perm(NC);
        std::vector<int> cols((size_t)MR * DC);
        for (int sb = 0; sb < DV; sb++) {
            for (int j = 0; j < NC; j++) perm[j] = j;
            for (int j = NC - 1; j > 0; j--) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                std::swap(perm[j], perm[x % (j + 1)]);
            }
            for (int u = 0; u < RB; u++) {
                int* c = cols.data() + ((size_t)sb * RB + u) * DC;
                for (int k = 0; k < DC; k++) c[k] = perm[u * DC + k];
                std::sort(c, c + DC);
            }
        }
        for (size_t v = 0; v < nseg / DC; v++) {
            const size_t t = v / MR, row = v % MR, sb = row / RB;
            for (int k = 0; k < DC; k++) r[v * DC + k] = (int)(t * ET + sb * NC + (size_t)cols[row * DC + k]);
        }
        CK(hipMalloc(&rbw, nseg * 4));
        CK(hipMalloc(&rbr, nseg * 4));
        CK(hipMemcpy(rbw, w.data(), nseg * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rbr, r.data(), nseg * 4, hipMemcpyHostToDevice));
    }
    const int reps = 10;
    auto run_w = [&](const char* name, auto kern, int SEG, const int* seg) {
        const size_t nw = nseg / SEG;
        const float ms = timeit([&] { kern<<<dim3((unsigned)((nw + 3) / 4)), dim3(256)>>>(buf, seg, nw, 1.0); }, reps);
        std::printf("%-44s %8.1f GB/s  (%.1f us)\n", name, bytes / (ms * 1e-3) / 1e9, ms * 1e3);
    };
    auto run_r = [&](const char* name, auto kern, int SEG, const int* seg) {
        const size_t nw = nseg / SEG;
        const float ms = timeit([&] { kern<<<dim3((unsigned)((nw + 3) / 4)), dim3(256)>>>(buf, seg, nw, out); }, reps);
        std::printf("%-44s %8.1f GB/s  (%.1f us)\n", name, bytes / (ms * 1e-3) / 1e9, ms * 1e3);
    };
    std::printf("buffer %.1f MB, %zu segments of 512 B\n", bytes / 1e6, nseg);
    run_w("write 8 random segments / wave, nt", write_segs<8, true>, 8, rnd);
    run_w("write 8 random segments / wave, plain", write_segs<8, false>, 8, rnd);
    run_w("write 32 contiguous segments / wave, nt", write_segs<32, true>, 32, ident);
    run_w("write 32 contiguous segments / wave, plain", write_segs<32, false>, 32, ident);
    run_w("write 8 contiguous segments / wave, nt", write_segs<8, true>, 8, ident);
    run_w("write 16 contiguous segments / wave, nt", write_segs<16, true>, 16, ident);
    run_w("write 16 contiguous segments / wave, plain", write_segs<16, false>, 16, ident);
    run_r("read 72 contiguous segments / wave, nt", read_segs<72, true>, 72, ident);
    run_r("read 72 contiguous segments / wave, plain", read_segs<72, false>, 72, ident);
    run_r("read 72 random segments / wave, nt", read_segs<72, true>, 72, rnd);
    run_r("read 72 random segments / wave, plain", read_segs<72, false>, 72, rnd);
    if (rb) {
        run_w("write rb, variable kernel's order, nt", write_segs<16, true>, 16, rbw);
        run_r("read rb, check kernel's order, nt", read_segs<72, true>, 72, rbr);
    }
    return 0;
}
