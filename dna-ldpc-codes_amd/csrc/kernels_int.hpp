// kernels_int.hpp -- integer-message decoders of dec.cpp on the same tiled
// layout as the fp64 kernels (tile = 64 codewords = one wave, lane =
// codeword, messages [tile][E][64], prior [tile][N][64], hard ballots
// [tile][N]).  All arithmetic is integer, so totals-minus-own replaces the
// reference's O(d^2) "all other edges" loops exactly.
//
//   quantized / offset min-sum  Run_MSA_Decoder dec.cpp:1174-1210 with
//     Init_MSA :1256-1298, Check_Update_MSA :1357-1396 (offset beta, clip at
//     0), Variable_Update_MSA :1438-1477 (its bSave_word_state trapping-set
//     post-processing branch is unreachable in the reference build: the flag
//     is set FALSE at DNA_main.cpp:697 and never TRUE, :724 is commented out),
//     Decision_MSA :1624-1656, Set_MSA :1683-1701, Cal_MSA_Q :1708-1746,
//     Cal_MSA_Clip :1748-1764.
//   Gallager A / B1 / B2        Run_Gallager_Decoder dec.cpp:699-723,
//     Init_Gallager :725-739, Check_Update_Gallager :748-769,
//     Variable_Update_Gallager :771-802, Decision_Gallager :804-832.
//
// Ties (a zero posterior in quantized min-sum) are broken in the reference
// by rand_int(2) from Intel MKL (dec.cpp:1273, :1647), which does not exist
// here; they are broken by tie_bit(seed, codeword, stage, bit), a
// counter-based hash shared with the oracle.  Outside ties the decoders are
// deterministic and follow the reference exactly.
#pragma once
#include "kernels.hpp"

namespace ldpc {
namespace dev {

__device__ __forceinline__ uint64_t smix(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// stage 0 = Init_MSA, stage n+1 = Decision_MSA of iteration n
__device__ __forceinline__ bool tie_bit(uint64_t seed, int64_t b, int32_t stage, int32_t j)
{
    uint64_t x = smix(seed);
    x = smix(x ^ (uint64_t)b);
    x = smix(x ^ (((uint64_t)(uint32_t)stage << 32) | (uint32_t)j));
    return (x & 1ull) != 0;
}

struct IntParams {
    int32_t algo;       // LDPC_ALGO_QMSA / GALLAGER_*
    int32_t max_value;  // Set_MSA: 2^(q-1) - 1
    int32_t min_value;  // -(2^(q-1) - 1)
    int32_t beta;       // offset (0 or 1 in the reference)
    double step;        // quantizer step
    uint64_t seed;      // tie-break seed
    int32_t b_var;      // Gallager: variable threshold
    int32_t b_dec;      // Gallager: decision threshold
};

// int32 arithmetic with the reference's wrap-around.  The reference is an
// x86 build: (int) of a double outside the int32 range -- an infinite or NaN
// LLR, or |LLR| / step >= 2^31 -- converts (cvttsd2si) to INT32_MIN, the
// "integer indefinite" value, which its sign step, abs() and sums then carry
// with two's-complement wrap.  In C++ all of these are undefined and the
// device's own conversion saturates, so the cases are spelled out here (and
// identically in oracle/ldpc_oracle.c).
__device__ __forceinline__ int32_t wrap_neg(int32_t v) { return (int32_t)(0u - (uint32_t)v); }
__device__ __forceinline__ int32_t wrap_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int32_t wrap_sub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

// Cal_MSA_Q(x, 0): uniform quantizer with clipping (dec.cpp:1708-1746)
__device__ __forceinline__ int32_t quantize(double x, const IntParams& p)
{
    const double mag = __builtin_fabs(x);
    const double q = mag / p.step + 0.5;
    int32_t k = q < 2147483648.0 ? (int32_t)q : INT32_MIN;  // (NaN fails the compare)
    if (x >= 0) {
        if (k > p.max_value) k = p.max_value;
    } else {
        if (k > -p.min_value) k = -p.min_value;
        k = wrap_neg(k);  // k *= sign
    }
    return k;
}

// init: prior (qLLR or recv = +-1) and v2c for every edge of the column;
// hard decision of the reference's Init_*.  in: [Bc][N] LLR, fp64.
__global__ __launch_bounds__(256) void k_init_int(const double* __restrict__ in, int64_t Bc, int64_t b_base,
                                                  int32_t N, int64_t E, const int32_t* __restrict__ col_ptr,
                                                  const int32_t* __restrict__ col_edge, IntParams p,
                                                  int32_t* __restrict__ prior, int32_t* __restrict__ v2c,
                                                  uint64_t* __restrict__ hard, uint64_t* __restrict__ active,
                                                  int32_t* __restrict__ iters, uint8_t* __restrict__ valid)
{
    __shared__ double s[TILE][TILE + 1];
    const int lane = lane_id(), w = wave_id();
    const int64_t t = blockIdx.y;
    const int32_t j0 = blockIdx.x * TILE;
    for (int r = w; r < TILE; r += 4) {
        const int64_t b = t * TILE + r;
        const int32_t j = j0 + lane;
        double v = 1.0;  // pad lanes: never active
        if (b < Bc && j < N) v = in[(size_t)b * N + j];
        s[r][lane] = v;
    }
    __syncthreads();
    const int64_t b = t * TILE + lane;
    const bool inb = b < Bc;
    for (int c = w; c < TILE; c += 4) {
        const int32_t j = j0 + c;
        if (j >= N) break;
        const double x = s[lane][c];
        int32_t m;
        bool h;
        if (p.algo == LDPC_ALGO_QMSA) {
            m = quantize(x, p);
            h = m > 0 ? false : (m < 0 ? true : tie_bit(p.seed, b_base + b, 0, j));
        } else {
            m = x < 0 ? -1 : 1;  // hard decision of the soft input (channel_BSC's recv)
            h = m < 0;
        }
        prior[((size_t)t * N + j) * TILE + lane] = m;
        const int32_t a = col_ptr[j], e1 = col_ptr[j + 1];
        for (int32_t q = a; q < e1; ++q) v2c[((size_t)t * E + col_edge[q]) * TILE + lane] = m;
        const uint64_t hm = __ballot(h && inb);
        if (lane == 0) hard[(size_t)t * N + j] = hm;
    }
    if (blockIdx.x == 0 && w == 0) {
        const uint64_t am = __ballot(inb);
        if (lane == 0) active[t] = am;
        if (inb) { iters[b] = 0; valid[b] = 0; }
    }
}

// check phase, one wave per (row, tile): quantized min-sum with offset, or
// the Gallager product of the other +-1 messages.
__global__ __launch_bounds__(256) void k_check_int(const int32_t* __restrict__ v2c, int32_t* __restrict__ c2v,
                                                   const uint64_t* __restrict__ active,
                                                   const int32_t* __restrict__ row_ptr, int32_t M, int64_t E,
                                                   int64_t t0, IntParams p)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (row >= M) return;
    if (!((active[t] >> lane) & 1ull)) return;
    const int32_t a = row_ptr[row], b = row_ptr[row + 1];
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    if (b == a) return;
    if (p.algo != LDPC_ALGO_QMSA) {
        int32_t prod = 1;
        for (int32_t e = a; e < b; ++e) prod *= v2c[(tb + e) * TILE + lane];
        for (int32_t e = a; e < b; ++e) c2v[(tl + e) * TILE + lane] = prod * v2c[(tb + e) * TILE + lane];
        return;
    }
    int32_t m1 = 0x7fffffff, m2 = 0x7fffffff, i1 = -1;
    uint32_t neg = 0;
    for (int32_t e = a; e < b; ++e) {
        const int32_t x = v2c[(tb + e) * TILE + lane];
        const int32_t ax = x < 0 ? wrap_neg(x) : x;  // abs(), INT32_MIN stays INT32_MIN
        neg ^= x >= 0 ? 0u : 1u;
        if (ax < m1) { m2 = m1; m1 = ax; i1 = e; }
        else if (ax < m2) m2 = ax;
    }
    for (int32_t e = a; e < b; ++e) {
        const int32_t x = v2c[(tb + e) * TILE + lane];
        // mag_min over the other edges; -1 sentinel when there are none
        int32_t mag = (b - a == 1) ? -1 : (e == i1 ? m2 : m1);
        mag = wrap_sub(mag, p.beta);
        if (mag < 0) mag = 0;
        const int32_t sign = ((neg ^ (x >= 0 ? 0u : 1u)) & 1u) ? -1 : 1;
        c2v[(tl + e) * TILE + lane] = sign * mag;
    }
}

// variable phase + decision, one wave per (column, tile).  post (optional,
// fp64 [t][N][64]) receives L_Q (min-sum) or the decided +-1 (Gallager).
__global__ __launch_bounds__(256) void k_var_int(const int32_t* __restrict__ c2v, int32_t* __restrict__ v2c,
                                                 const int32_t* __restrict__ prior, uint64_t* __restrict__ hard,
                                                 const uint64_t* __restrict__ active,
                                                 const int32_t* __restrict__ col_ptr,
                                                 const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                 int32_t N, int64_t E, int64_t t0, int64_t b_base, int32_t iter,
                                                 IntParams p)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (j >= N) return;
    const uint64_t act = active[t];
    if (act == 0) return;
    const bool live = (act >> lane) & 1ull;
    const int32_t a = col_ptr[j], b = col_ptr[j + 1];
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    bool h = false;
    if (live) {
        const size_t pj = ((size_t)t * N + j) * TILE + lane;
        const int32_t pr = prior[pj];
        if (p.algo == LDPC_ALGO_QMSA) {
            // the reference's sequential sum prior + the other edges, in wrapping
            // int32 (associative, so prior + all - own is the same value)
            int32_t tot = 0;
            for (int32_t s = a; s < b; ++s) tot = wrap_add(tot, c2v[(tl + col_edge[s]) * TILE + lane]);
            for (int32_t s = a; s < b; ++s) {
                int32_t sum = wrap_sub(wrap_add(pr, tot), c2v[(tl + col_edge[s]) * TILE + lane]);
                if (sum > p.max_value) sum = p.max_value;
                else if (sum < p.min_value) sum = p.min_value;
                v2c[(tb + col_edge[s]) * TILE + lane] = sum;
            }
            const int32_t L = wrap_add(pr, tot);
            h = L > 0 ? false : (L < 0 ? true : tie_bit(p.seed, b_base + t * TILE + lane, iter + 1, j));
            if (post) post[pj] = (double)L;
        } else {
            const int32_t msg = -pr;
            int32_t cnt = 0;
            for (int32_t s = a; s < b; ++s) cnt += c2v[(tl + col_edge[s]) * TILE + lane] == msg;
            for (int32_t s = a; s < b; ++s) {
                const int32_t num = cnt - (c2v[(tl + col_edge[s]) * TILE + lane] == msg);
                v2c[(tb + col_edge[s]) * TILE + lane] = num >= p.b_var ? msg : pr;
            }
            const int32_t temp = cnt >= p.b_dec ? msg : pr;
            h = temp < 0;
            if (post) post[pj] = (double)temp;
        }
    }
    const uint64_t m = __ballot(h);
    if (lane == 0) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (act == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~act) | (m & act);
    }
}

// posterior rows [b][N]: the last decision's value, or the prior at iters 0
__global__ __launch_bounds__(256) void k_finalize_int(const double* __restrict__ post_t,
                                                      const int32_t* __restrict__ prior,
                                                      const int32_t* __restrict__ iters, double* __restrict__ out,
                                                      int64_t Bc, int32_t N)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = blockIdx.y;
    const int64_t b = t * TILE + lane;
    if (j >= N || b >= Bc) return;
    const size_t pj = ((size_t)t * N + j) * TILE + lane;
    out[(size_t)b * N + j] = iters[b] == 0 ? (double)prior[pj] : post_t[pj];
}

}  // namespace dev
}  // namespace ldpc
