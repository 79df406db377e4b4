// xr2probe.hip -- round-5 go / no-go probe for an L2-resident BP decoder on
// MI355X (not part of the product).
//
// The tiled decoder keeps 192 codewords in flight and streams their messages
// through the Infinity Cache (~6.8 TB/s for its access shape).  Only the
// XCDs' L2s (4 MB each) are faster, and they can hold ~3 codewords per XCD.
// This probe runs the BP iteration of the DNA code for C codewords per XCD
// inside ONE persistent launch, with the phases separated by XCD-local
// barriers, and reports microseconds per codeword-iteration:
//
//   messages  msg[c][t][b][i] fp64: the edge of column i of column block b
//             in row block t (the code's 8 x 72 array of 256 x 256
//             permutations, ldpc_graph_blocks); in place, d between the
//             phases after a variable phase, lr after a check phase
//   check     task (codeword, row block t): one 256-thread workgroup (1 per
//             CU: 147 KB LDS) loads the block's 147 KB contiguously into LDS,
//             lane = row, reads its 72 edges in the row's own (reference)
//             order through a u16 index table, runs dec.cpp:646-662's
//             prefix / suffix arithmetic, writes lr back into LDS, and the
//             workgroup stores the 147 KB back; plus the row parity of the
//             previous decisions (a 2.3 KB bitmap in LDS)
//   variable  task (codeword, column block b): lane = column, its 8 edges
//             (one per row block, ascending row) coalesced, dec.cpp:667-693,
//             the decision ballots
//   parts     (C = 3) the check task without its 147 KB load / store, and
//             with only them
//   barrier   per XCD: every wave drains its stores, one agent-scope atomic
//             add per workgroup, a bounded relaxed poll; message loads are
//             agent-scope (sc1: they miss the CU's L1 and hit the XCD's L2)
//
// The workgroup -> XCD mapping is read from HW_REG_XCC_ID; a workgroup whose
// XCD differs from blockIdx % 8 is counted (the probe assumes round-robin
// placement for its work split -- timing only, results are not used).  Every
// spin is bounded: a timeout sets err and ends the launch.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/xr2probe tools/xr2probe.hip \
//         -Ldna-ldpc-codes_amd/lib -lldpc_amd -Wl,-rpath,$PWD/dna-ldpc-codes_amd/lib
//   tools/xr2probe tests/golden/decode_n18432_m2048_final.pchk
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/ldpc_amd.h"

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
    } while (0)

constexpr int Q = 256, RB = 8, CB = 72, DC = 72, DV = 8;
constexpr int NCOL = Q * CB, NROW = Q * RB, EDGES = NCOL * DV;
constexpr int NXCD = 8;
constexpr unsigned kSpinMax = 1u << 22;

struct Args {
    double* msg;            // [cw][RB][CB][Q]
    const int8_t* pcode;    // [cw][CB][Q]
    const double* ptab;     // [256]
    const uint16_t* ridx;   // [RB][DC][Q]: b * Q + i of row (t, r)'s k-th edge
    uint64_t* hard;         // [cw][NCOL / 64]
    unsigned* bar;          // [NXCD * 32] (one 128-B line per XCD)
    unsigned* err;          // [0] timeouts, [1] XCC mismatches
    int C;                  // codewords per XCD
    int iters;
    int mode;               // 1 check, 2 variable, 3 both (0: barriers only)
};

// Loads that miss the CU's L1 and are served by the XCD's L2: buffer loads
// with the sc1 cache-policy bit (aux 16 on gfx950).  Plain loads, so the
// compiler keeps many in flight -- agent-scope atomic loads (the round-2 XR
// decoder's LDM 2) each wait for the previous one (s_waitcnt vmcnt(0)).
constexpr int kSc1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                            (int)(bytes < 0x7fffffffull ? bytes : 0x7fffffffull), 0x00020000);
}
__device__ __forceinline__ double ld_l2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, kSc1));
}

// XCD-local barrier, epoch e (1, 2, ...): nwg workgroups of XCD x
__device__ bool xcd_barrier(const Args& a, int x, unsigned nwg, unsigned e)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        unsigned* c = a.bar + x * 32;
        const unsigned o = atomicAdd(c, 1u);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");
        const unsigned want = nwg * e;
        unsigned spins = 0;
        int ok = 1;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins >= kSpinMax || __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                atomicAdd(a.err, 1u);
                ok = 0;
                break;
            }
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// dec.cpp:646-662 on one row, in registers (the product's check_bp_compute);
// x[k] receives lr_k once d_k has had its last use
__device__ __forceinline__ void check_row(double (&x)[DC])
{
    constexpr int SEG = 8, NSEG = DC / SEG;
    double cp[NSEG];
    double p = 1.0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k % SEG == 0) cp[k / SEG] = p;
        p = p * x[k];
    }
    double s = 1.0;
#pragma unroll
    for (int g = NSEG - 1; g >= 0; --g) {
        double pk[SEG];
        double q = cp[g];
        asm volatile("" : "+v"(q));
#pragma unroll
        for (int i = 0; i < SEG; ++i) { pk[i] = q; q = q * x[g * SEG + i]; }
#pragma unroll
        for (int i = SEG - 1; i >= 0; --i) {
            const int k = g * SEG + i;
            const double tt = pk[i] * s;
            const double lr = (1.0 + tt) / (1.0 - tt);
            s = s * x[k];
            x[k] = lr;
        }
    }
}

__global__ __launch_bounds__(256, 1) void k_xr2(Args a)
{
    __shared__ double s_blk[RB == 8 ? CB * Q : 1];  // 147 456 B
    __shared__ uint64_t s_hb[NCOL / 64];            // 2 304 B
    __shared__ unsigned s_any;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int x = (int)(blockIdx.x % NXCD), w = (int)(blockIdx.x / NXCD);
    const unsigned nwg = gridDim.x / NXCD;
    if (threadIdx.x == 0 && (int)(xcc & 0xfu) != x) atomicAdd(a.err + 1, 1u);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned e = 0;
    for (int it = 0; it < a.iters; ++it) {
        // ---- check phase: tasks (codeword, row block), one per workgroup ----
        if ((a.mode & 1) && w < a.C * RB) {
            const int c = x * a.C + w / RB, t = w % RB;
            double* blk = a.msg + ((size_t)c * RB + t) * CB * Q;
            const auto rb = rsrc(blk, (uint64_t)CB * Q * 8);
            // the block's 147 KB: thread tid loads elements tid + 256 q (512-B wave segments)
            if (!(a.mode & 4)) {
#pragma unroll 24
                for (int q = 0; q < CB * Q / 256; ++q) s_blk[tid + 256 * q] = ld_l2(rb, (uint32_t)(tid + 256 * q) * 8);
            }
            const auto rh = rsrc(a.hard + (size_t)c * (NCOL / 64), NCOL / 8);
            for (int q = tid; q < NCOL / 64; q += 256)
                s_hb[q] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rh, q * 8, 0, kSc1));
            if (tid == 0) s_any = 0;
            __syncthreads();
            if (!(a.mode & 8)) {
                const uint16_t* ix = a.ridx + (size_t)t * DC * Q + tid;
                uint16_t id[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) id[k] = ix[(size_t)k * Q];
                double xv[DC];
                unsigned par = 0;
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    xv[k] = s_blk[id[k]];
                    par ^= (unsigned)(s_hb[id[k] >> 6] >> (id[k] & 63)) & 1u;
                }
                check_row(xv);
                if (__ballot(par) && lane == 0) atomicOr(&s_any, 1u);
#pragma unroll
                for (int k = 0; k < DC; ++k) s_blk[id[k]] = xv[k];
            }
            __syncthreads();
            if (!(a.mode & 4)) {
#pragma unroll 8
                for (int q = 0; q < CB * Q / 256; ++q) blk[tid + 256 * q] = s_blk[tid + 256 * q];
            }
        }
        if (!xcd_barrier(a, x, nwg, ++e)) return;
        // ---- variable phase: tasks (codeword, column block), strided over the XCD's workgroups ----
        if (a.mode & 2) {
            for (int task = w; task < a.C * CB; task += (int)nwg) {
                const int c = x * a.C + task / CB, b = task % CB;
                const int i = tid;
                double l[DV];
                const auto rm = rsrc(a.msg + (size_t)c * EDGES, (uint64_t)EDGES * 8);
#pragma unroll
                for (int t = 0; t < DV; ++t) l[t] = ld_l2(rm, (uint32_t)(((t * CB) + b) * Q + i) * 8);
                const double LR = a.ptab[a.pcode[((size_t)c * CB + b) * Q + i] + 128];
                double pr[DV], d[DV];
                double p = LR;
#pragma unroll
                for (int t = 0; t < DV; ++t) { pr[t] = p; p = p * l[t]; }
                if (__builtin_isnan(p)) p = 1.0;
                const bool h = p <= 1.0;
                double acc = 1.0;
#pragma unroll
                for (int t = DV - 1; t >= 0; --t) {
                    double v = pr[t] * acc;
                    if (__builtin_isnan(v)) v = 1.0;
                    acc = acc * l[t];
                    d[t] = 1.0 - 2.0 / (1.0 + v);
                }
#pragma unroll
                for (int t = 0; t < DV; ++t) a.msg[(((size_t)c * RB + t) * CB + b) * Q + i] = d[t];
                const uint64_t m = __ballot(h);
                if (lane == 0) a.hard[(size_t)c * (NCOL / 64) + b * (Q / 64) + wave] = m;
            }
        }
        if (!xcd_barrier(a, x, nwg, ++e)) return;
    }
}

int main(int argc, char** argv)
{
    const char* pchk = argc > 1 ? argv[1] : "tests/golden/decode_n18432_m2048_final.pchk";
    int err = 0;
    ldpc_graph* g = ldpc_graph_load(pchk, &err);
    if (!g) { std::printf("load %s: %s\n", pchk, ldpc_last_error()); return 1; }
    int32_t M, N, dv, rdv, dc, rdc;
    int64_t E;
    ldpc_graph_info(g, &M, &N, &E, &dv, &rdv, &dc, &rdc);
    int32_t q = 0, rb = 0, cb = 0;
    std::vector<int32_t> colblk(N);
    if (ldpc_graph_blocks(g, &q, &rb, &cb, colblk.data()) || q != Q || rb != RB || cb != CB || N != NCOL ||
        M != NROW || E != EDGES) {
        std::printf("not the (8,72) array code: Q %d, %d x %d blocks\n", q, rb, cb);
        return 1;
    }
    std::vector<int32_t> rp(M + 1), ci(E);
    ldpc_graph_edges(g, rp.data(), ci.data(), nullptr, nullptr);
    std::vector<int32_t> inblk(N), cnt(CB, 0);
    for (int j = 0; j < N; j++) inblk[j] = cnt[colblk[j]]++;
    std::vector<uint16_t> ridx((size_t)RB * DC * Q);
    for (int r = 0; r < M; r++) {
        const int t = r / Q, rr = r % Q;
        std::vector<int> seen(CB, 0);
        for (int k = 0; k < DC; k++) {
            const int j = ci[rp[r] + k];
            seen[colblk[j]]++;
            ridx[((size_t)t * DC + k) * Q + rr] = (uint16_t)(colblk[j] * Q + inblk[j]);
        }
        for (int b = 0; b < CB; b++)
            if (seen[b] != 1) { std::printf("row %d: %d edges in column block %d\n", r, seen[b], b); return 1; }
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    if (prop.multiProcessorCount != 256) { std::printf("%d CUs: the probe needs all 256 resident\n", prop.multiProcessorCount); return 1; }
    const int cmax = 4;
    const int ncw = NXCD * cmax;
    double* d_msg;
    int8_t* d_pc;
    double* d_tab;
    uint16_t* d_ridx;
    uint64_t* d_hard;
    unsigned *d_bar, *d_err;
    CK(hipMalloc(&d_msg, (size_t)ncw * EDGES * 8));
    CK(hipMalloc(&d_pc, (size_t)ncw * NCOL));
    CK(hipMalloc(&d_tab, 256 * 8));
    CK(hipMalloc(&d_ridx, ridx.size() * 2));
    CK(hipMalloc(&d_hard, (size_t)ncw * NCOL / 8));
    CK(hipMalloc(&d_bar, NXCD * 32 * 4));
    CK(hipMalloc(&d_err, 64));
    CK(hipMemcpy(d_ridx, ridx.data(), ridx.size() * 2, hipMemcpyHostToDevice));
    std::vector<double> tab(256);
    for (int k = 0; k < 256; k++) tab[k] = std::exp((k - 128) * std::log(49.0));
    CK(hipMemcpy(d_tab, tab.data(), 256 * 8, hipMemcpyHostToDevice));
    // BSC(0.02)-like codes (+1 / -1), d = 1 - 2 / (1 + LR) on every edge
    std::vector<int8_t> pc((size_t)ncw * NCOL);
    uint64_t s = 12345;
    for (auto& v : pc) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = ((s >> 33) % 50 == 0) ? -1 : 1; }
    CK(hipMemcpy(d_pc, pc.data(), pc.size(), hipMemcpyHostToDevice));
    std::vector<double> msg((size_t)ncw * EDGES);
    for (int c = 0; c < ncw; c++)
        for (int t = 0; t < RB; t++)
            for (int b = 0; b < CB; b++)
                for (int i = 0; i < Q; i++) {
                    const double LR = tab[pc[((size_t)c * CB + b) * Q + i] + 128];
                    msg[(((size_t)c * RB + t) * CB + b) * Q + i] = 1.0 - 2.0 / (1.0 + LR);
                }
    CK(hipMemcpy(d_msg, msg.data(), msg.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(d_hard, 0, (size_t)ncw * NCOL / 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("xr2probe: %d codewords max, %zu B LDS per workgroup\n", ncw, (size_t)(CB * Q * 8 + NCOL / 8 + 4));
    // mode bits: 1 check phase, 2 variable phase; 4: the check task without
    // its 147 KB load and store (LDS reads, arithmetic, LDS writes only),
    // 8: the check task's load and store only
    const char* mname[] = {"barriers", "check", "variable", "both", "", "chk-lds+arith", "", "", "", "chk-ld/st"};
    for (int C : {1, 2, 3, 4}) {
        for (int mode : {0, 1, 2, 3, 5, 9}) {
            if ((mode == 5 || mode == 9) && C != 3) continue;
            float ms[2];
            const int its[2] = {4, 24};
            for (int r = 0; r < 2; r++) {
                CK(hipMemset(d_bar, 0, NXCD * 32 * 4));
                CK(hipMemset(d_err, 0, 64));
                Args a{d_msg, d_pc, d_tab, d_ridx, d_hard, d_bar, d_err, C, its[r], mode};
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_xr2, dim3(256), dim3(256), 0, 0, a);
                CK(hipGetLastError());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[r], e0, e1));
                unsigned he[2];
                CK(hipMemcpy(he, d_err, 8, hipMemcpyDeviceToHost));
                if (he[0] || he[1]) { std::printf("C %d mode %s: %u timeouts, %u XCC mismatches\n", C, mname[mode], he[0], he[1]); if (he[0]) return 2; }
            }
            const double us_it = (ms[1] - ms[0]) * 1e3 / (its[1] - its[0]);
            const int cw = NXCD * C;
            std::printf("C %d (%2d codewords)  %-9s  %8.2f us per iteration  %6.3f us per codeword-iteration", C, cw,
                        mname[mode], us_it, us_it / cw);
            if (mode == 3) std::printf("  -> %6.0f cw/s at 50 iterations", cw / (us_it * 50 * 1e-6));
            std::printf("\n");
            std::fflush(stdout);
        }
    }
    return 0;
}
