// kernels.hpp -- HIP device kernels for batched LDPC decoding on MI355X (gfx950).
//
// Layout in HBM (one engine = one chunk of C codewords, C a multiple of 64):
//   tile t = 64 consecutive codewords; lane l of a wavefront = codeword 64t+l.
//   v2c [t][E][64] fp64  BP: d = 1 - 2/(1+pr) of the variable->check message
//                        MSA: msg_v_to_c_fp
//   c2v [t][E][64] fp64  BP: lr (check->variable likelihood ratio)
//                        MSA: msg_c_to_v_fp
//   prior [t][N][64] fp64  BP: LR = exp(LLR);  MSA: LLR
//   hard [t][N] u64     bit l = hard decision of codeword 64t+l (a ballot)
//   active [t] u64      bit l = codeword 64t+l still iterating
// Every message access of a wave is one 512-B contiguous segment (64 lanes x
// 8 B) in BOTH phases, and the graph indices (CSR row offsets, CSC edge ids)
// are wave-uniform scalar loads.  Each lane runs the reference's sequential
// per-row / per-column loops, which is what bit-exactness with the
// reference's fp64 operation order requires (no tree reductions of the
// products/sums; only the order-free XOR/OR syndrome uses cross-lane ops).
//
// Compiled with -ffp-contract=off and without fast-math: fp64 '/' lowers to
// the correctly-rounded IEEE division, no FMA contraction, isnan() honoured.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "kargs.hpp"

namespace ldpc {
namespace dev {

constexpr int TILE = 64;

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// XCD-aware block order (cdna_hip_programming.md T1): blocks b and b+8 share an
// XCD under round-robin dispatch, so give each b % 8 group a contiguous range
// of logical blocks (bijective for any grid size).  Speed only, never
// correctness: neighbouring column groups then share the XCD's L2 (refill
// input rows, hard-bit words).
__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb)
{
    const unsigned q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m)
{
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = (uint32_t)__shfl_xor((int)lo, m);
    hi = (uint32_t)__shfl_xor((int)hi, m);
    return ((uint64_t)hi << 32) | lo;
}

// A fault found where the codeword index is no longer at hand: the report
// carries another index (the lane's pool slot).  Each kind has its own word
// (fault[kind]), so reports of different kinds never overwrite each other.
__device__ __forceinline__ void lane_fault(unsigned long long* fault, unsigned kind, int64_t idx)
{
    if (fault)
        __hip_atomic_store(fault + kind, kFaultTag | ((unsigned long long)kind << 48) | ((unsigned long long)idx & kFaultIndex),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A lane's codeword index b addresses the decode's outputs / input rows
// only when 0 <= b < B.  Outside, the caller skips the access and the
// fault word (kargs.hpp kFaultTag) records the kind and index for the host,
// so broken lane bookkeeping ends as LDPC_ERR_DEVICE, not as an
// out-of-bounds write.
__device__ __forceinline__ bool lane_index_ok(int64_t b, int64_t B, unsigned long long* fault, unsigned kind)
{
    if (b >= 0 && b < B) return true;
    lane_fault(fault, kind, b);
    return false;
}

// The variable kernels' two lane-indexed accesses, checked by plain compares
// whose faults are reported at the end of the kernel (lane_fault, by the
// lane's pool slot): a report branch between a refilled lane's lane_b load
// and its input-row load cost config 5 2 % (profiles/r5/README.md).
//   refill_row: a refilled lane's input row, row 0 when b is out of range
//   out_ok:     the finished codeword's index bounds at its output stores
__device__ __forceinline__ int64_t refill_row(int64_t b, const Refill& rf, bool& bad)
{
    const bool ok = (uint64_t)b < (uint64_t)rf.nb;
    bad = !ok;
    return ok ? b : 0;
}
__device__ __forceinline__ bool out_ok(int64_t fb, const Refill& rf) { return (uint64_t)fb < (uint64_t)rf.nb; }

// streaming access to the v2c ("d") array, optionally nontemporal
template <bool NT>
__device__ __forceinline__ double ld(const double* p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(double* p, double v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Message pointers of the phase kernels: __restrict__ when the input and
// output messages are distinct buffers; plain pointers when they are the same
// buffer (the resident pool runs in place: a row's check messages overwrite
// the variable messages they are computed from, a column's variable messages
// its check messages).  In place, the order "every load of a row's / column's
// edges before its first store" is then the source's, which the compiler must
// keep for possibly aliasing accesses -- it does not rest on the generated ISA.
template <bool INPLACE>
struct Msg {
    using in = const double* __restrict__;
    using out = double* __restrict__;
};
template <>
struct Msg<true> {
    using in = const double*;
    using out = double*;
};

// Whole-line lane policy: a lane with no codeword, or a
// finished one, still runs when its 16-lane group -- one 128-byte line of
// every 512-byte message segment -- holds a lane that is being decoded, so
// message stores cover whole lines; lines without one are neither read nor
// written (a partly filled last tile, a draining pool).  Their values are
// never read.
__device__ __forceinline__ bool line_occupied(uint64_t m, int lane)
{
    return ((m >> (lane & ~15)) & 0xFFFFull) != 0ull;
}

// The finished codeword's hard bits of the wave's CPW consecutive columns
// (pre-update ballots), one CPW-byte store per lane when the output is
// aligned for it (Refill::hard_vec), else byte stores.
template <int CPW>
__device__ __forceinline__ void store_fin_hard(const Refill& rf, const uint64_t* __restrict__ hw, int64_t fb,
                                               int32_t N, int32_t j0, int lane)
{
    uint64_t v = 0;
#pragma unroll
    for (int c = 0; c < CPW; ++c) v |= ((hw[c] >> lane) & 1ull) << (8 * c);
    uint8_t* p = rf.hard_out + (size_t)fb * N + j0;
    if (rf.hard_vec && (CPW == 8 || CPW == 4 || CPW == 2 || CPW == 1)) {
        if constexpr (CPW == 8) *reinterpret_cast<uint64_t*>(p) = v;
        else if constexpr (CPW == 4) *reinterpret_cast<uint32_t*>(p) = (uint32_t)v;
        else if constexpr (CPW == 2) *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
        else *p = (uint8_t)v;
    } else {
#pragma unroll
        for (int c = 0; c < CPW; ++c) p[c] = (uint8_t)(v >> (8 * c));
    }
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Lane bookkeeping of tile t once its syndrome word U is known (threads 0..63
// of the block; lane = threadIdx.x).  Shared with k_syndrome_res.
// ln0 / b0: the lane's cs.lane_n / cs.lane_b, loaded by the caller (only
// meaningful for occupied lanes).  probe: read the claim counter before
// claiming (avoids atomics on it once the input is exhausted).
__device__ __forceinline__ void cont_lanes(int64_t t, uint64_t occ, uint64_t U, int32_t max_iter, const ContState& cs,
                                           const ContOut& co, int64_t* s_b, int32_t* s_n, uint64_t* s_fin,
                                           int32_t ln0, int64_t b0, bool probe)
{
    const int lane = lane_id();
    {
        const size_t li = (size_t)t * TILE + lane;
        const bool o = (occ >> lane) & 1ull;
        const int32_t ln = o ? ln0 : 0;
        const bool unsat = (U >> lane) & 1ull;
        const bool fin = o && (!unsat || ln == max_iter);
        const bool cont = o && !fin;
        const int64_t b = o ? b0 : -1;
        if (fin && lane_index_ok(b, cs.B, cs.fault, kFaultIters)) { co.iters[b] = ln; co.valid[b] = unsat ? 0 : 1; }
        s_b[lane] = b;
        s_n[lane] = ln;
        const uint64_t F = __ballot(fin), Cm = __ballot(cont);
        // refill every lane that is not continuing
        const uint64_t freem = ~Cm;
        const int nfree = __popcll(freem);
        unsigned long long base = 0;
        if (lane == 0 && nfree > 0) {
            if (probe) {
                const unsigned long long nb = __hip_atomic_load(cs.next_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                base = (nb < (unsigned long long)cs.B) ? atomicAdd(cs.next_b, (unsigned long long)nfree) : nb;
            } else {
                base = atomicAdd(cs.next_b, (unsigned long long)nfree);
            }
        }
        base = __shfl(base, 0);
        const int rank = __popcll(freem & ((1ull << lane) - 1ull));
        const bool fresh = !cont && (base + (unsigned long long)rank < (unsigned long long)cs.B);
        const uint64_t Fr = __ballot(fresh);
        if (cont) cs.lane_n[li] = ln + 1;
        if (fresh) {
            int64_t nbv = (int64_t)(base + rank);
            if (cs.debug_bad_lane && nbv == 0) nbv = cs.B + 4096;  // tests only (LDPC_SCHED_DEBUG_BAD_LANE)
            cs.lane_b[li] = nbv;
            cs.lane_n[li] = 0;
        }
        if (lane == 0) {
            cs.active[t] = Cm;
            cs.fresh[t] = Fr;
            cs.occupied[t] = Cm | Fr;
            *s_fin = F;
            if (cs.occ_count) {
                const unsigned long long add = (1ull << kOccTileShift) | (unsigned long long)__popcll(Cm | Fr);
                const unsigned long long old = atomicAdd(cs.occ_count, add);
                if (cs.poll_host && (int64_t)(old >> kOccTileShift) + 1 == cs.ntiles)
                    __hip_atomic_store(cs.poll_host, (cs.poll_tag << kOccTileShift) | ((old + add) & kOccMask),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (t == 0 && cs.occ_clear) *cs.occ_clear = 0ull;
        }
    }
}

// Resident pool (ResStep): the parity of one row over the ballots of the
// previous variable phase, one gathered ballot per lane (DC / 64 rounds)
// and an XOR across the wave; the result is wave-uniform.
template <int DC>
__device__ __forceinline__ uint64_t row_parity(const uint64_t* __restrict__ h, const int32_t* __restrict__ cols)
{
    const int lane = lane_id();
    uint64_t p = 0;
#pragma unroll
    for (int k0 = 0; k0 < DC; k0 += TILE)
        if (k0 + lane < DC) p ^= h[cols[k0 + lane]];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) p ^= shfl_xor_u64(p, off);
    return p;
}

// Resident pool epilogue of a check block (all 256 threads): OR the block's
// row parities into unsat[t]; the last of the tile's nblk blocks to arrive runs the
// lane bookkeeping for the step (cont_lanes: iters / valid, refill claims,
// active / fresh / occupied masks) and hands the finished lanes to the
// variable kernel, which writes their outputs before refilling them.
__device__ __forceinline__ void res_arrive(int64_t t, uint64_t occ, uint64_t p, const ResStep& rs, int32_t ln0,
                                           int64_t b0, uint32_t nblk)
{
    __shared__ uint64_t red[4];
    __shared__ int64_t s_b[TILE];
    __shared__ int32_t s_n[TILE];
    __shared__ uint64_t s_fin;
    __shared__ int s_last;
    const int lane = lane_id(), w = wave_id();
    if (lane == 0) red[w] = p;
    __syncthreads();
    // No fences: an agent-scope release would write back the L2 in every
    // block.  Only device-coherent atomics carry data between the blocks; the
    // arrival is issued after the OR has returned (its value is consumed), and
    // the last block reads the word back with an RMW.  Everything else the
    // bookkeeping reads was written by earlier kernels.
    if (threadIdx.x == 0) {
        const uint64_t U = red[0] | red[1] | red[2] | red[3];
        unsigned long long o = 0;
        if (U) o = atomicOr(rs.unsat + t, (unsigned long long)U);
        asm volatile("" ::"v"(o) : "memory");
        s_last = atomicAdd(rs.done + t, 1u) == nblk - 1;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x < TILE) {
        const uint64_t U = occ ? (uint64_t)atomicOr(rs.unsat + t, 0ull) : 0ull;
        cont_lanes(t, occ, U, rs.max_iter, rs.cs, rs.co, s_b, s_n, &s_fin, ln0, b0, false);
        const size_t li = (size_t)t * TILE + lane;
        rs.fin_b[li] = s_b[lane];
        rs.fin_n[li] = s_n[lane];
        if (lane == 0) {
            rs.fin[t] = s_fin;
            atomicExch(rs.unsat + t, 0ull);
            atomicExch(rs.done + t, 0u);
        }
    }
}

// ---------------------------------------------------------------------------
// init: transpose a [b][N] input chunk into the tiled layout, set the initial
// messages and hard decisions.
//   BP  : Init_Belief_Propagation dec.cpp:608-629  (pr = LR, lr = 1, dblk = LR < 1);
//         d = 1 - 2/(1+pr) is what the check phase consumes (dec.cpp:652,660).
//   MSA : Init_MSA_INF dec.cpp:1300-1329 (v2c = LLR, dblk = !(LLR > 0)).
// grid (ceil(N/64), tiles), block 256; LDS 64x65 fp64 transpose tile.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_init(const double* __restrict__ in, int in_is_llr, int algo_msa,
                                              int64_t Bc, int32_t N, int64_t E,
                                              const int32_t* __restrict__ col_ptr, const int32_t* __restrict__ col_edge,
                                              double* __restrict__ prior, double* __restrict__ v2c,
                                              uint64_t* __restrict__ hard, uint64_t* __restrict__ active,
                                              int32_t* __restrict__ iters, uint8_t* __restrict__ valid,
                                              uint8_t* __restrict__ sgn, int32_t vpa, int32_t vpb)
{
    __shared__ double s[TILE][TILE + 1];
    const int lane = lane_id(), w = wave_id();
    const int64_t t = blockIdx.y;
    const int32_t j0 = blockIdx.x * TILE;
    for (int r = w; r < TILE; r += 4) {
        const int64_t b = t * TILE + r;
        const int32_t j = j0 + lane;
        double v = in_is_llr ? 0.0 : 1.0;  // pad lanes: LLR 0 / LR 1 (never active)
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
        double pv, m;
        bool h;
        if (algo_msa) {
            pv = x;  // LLR
            m = x;
            h = !(x > 0);
        } else {
            pv = in_is_llr ? exp(x) : x;  // LR (ocml exp when the input is LLR)
            m = 1.0 - 2.0 / (1.0 + pv);
            h = (pv < 1.0);
        }
        prior[((size_t)t * N + j) * TILE + lane] = pv;
        const int32_t a = col_ptr[j], e1 = col_ptr[j + 1];
        // (the compressed min-sum -- sgn set -- keeps v2c in column order:
        // edge s of column j at j * vpa + s * vpb, see k_var_msa_c)
        for (int32_t q = a; q < e1; ++q)
            v2c[((size_t)t * E + (sgn ? j * vpa + (q - a) * vpb : col_edge[q])) * TILE + lane] = m;
        // compressed min-sum without codes: sign bits of the stored v2c (all edges alike)
        if (sgn) sgn[((size_t)t * N + j) * TILE + lane] = (m >= 0) ? 0u : 0xffu;
        const uint64_t hm = __ballot(h && inb);
        if (lane == 0) hard[(size_t)t * N + j] = hm;
    }
    if (blockIdx.x == 0 && w == 0) {
        const uint64_t am = __ballot(inb);
        if (lane == 0) active[t] = am;
        if (inb) { iters[b] = 0; valid[b] = 0; }
    }
}

// ---------------------------------------------------------------------------
// syndrome + termination bookkeeping for iteration n (one block per tile).
// check() check.cpp:28-45 / mod2sparse_mulvec mod2sparse.cpp:855-881 on the
// 64 codewords of the tile at once: row parity = XOR of the column ballots.
// Run_*_Decoder loop control dec.cpp:594-599 / 1223-1246:
//   c == 0            -> stop, iters = n, valid = 1
//   n == max_iter     -> stop, iters = n, valid = (c == 0)
// ---------------------------------------------------------------------------
template <int DC>
__global__ __launch_bounds__(1024) void k_syndrome(const uint64_t* __restrict__ hard, uint64_t* __restrict__ active,
                                                   int32_t* __restrict__ iters, uint8_t* __restrict__ valid,
                                                   const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col_idx,
                                                   const int32_t* __restrict__ col_idx_T, int32_t M, int32_t N,
                                                   int32_t n, int32_t max_iter)
{
    __shared__ uint64_t red[16];
    const int64_t t = blockIdx.x;
    const uint64_t act = active[t];
    if (act == 0) return;
    const uint64_t* h = hard + (size_t)t * N;
    uint64_t u = 0;
    for (int32_t i = threadIdx.x; i < M; i += blockDim.x) {
        uint64_t p = 0;
        if (DC > 0) {
#pragma unroll 24
            for (int k = 0; k < DC; ++k) p ^= h[col_idx_T[(size_t)k * M + i]];
        } else {
            for (int32_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) p ^= h[col_idx[e]];
        }
        u |= p;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) u |= shfl_xor_u64(u, off);
    const int lane = lane_id(), w = wave_id();
    if (lane == 0) red[w] = u;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint64_t U = 0;
        const int nw = blockDim.x >> 6;
        for (int q = 0; q < nw; ++q) U |= red[q];
        if ((act >> lane) & 1ull) {
            const size_t b = (size_t)t * TILE + lane;
            if (!((U >> lane) & 1ull)) { iters[b] = n; valid[b] = 1; }
            else if (n == max_iter) { iters[b] = n; valid[b] = 0; }
        }
        if (lane == 0) active[t] = (n == max_iter) ? 0ull : (act & U);
    }
}

// ---------------------------------------------------------------------------
// BP check-node phase, regular row degree DC (Iter_Belief_Propagation
// dec.cpp:646-662).  Per row and lane:
//   forward  lr_k <- p_k = (((1*d_0)*d_1)*...)*d_{k-1}
//   backward s = 1; for k = DC-1..0: t = p_k*s; lr_k = (1+t)/(1-t); s *= d_k
// d_k (= 1 - 2/(1+pr_k), stored by the variable phase) stays in registers;
// the prefix products are kept as checkpoints every SEG edges and recomputed
// segment by segment in the backward pass (same operations in the same order
// -> identical values), which keeps the kernel at 2 waves/SIMD.
// grid (ceil(M/4), tiles), block 256: one wave per (row, tile).
// ---------------------------------------------------------------------------
template <int DC, bool NT, bool INPLACE>
__device__ __forceinline__ void check_bp_load(double (&x)[DC], typename Msg<INPLACE>::in src)
{
#pragma unroll
    for (int k = 0; k < DC; ++k) x[k] = ld<NT>(src + (size_t)k * TILE);
}

// dst: the row's first c2v message (CSR order, row-contiguous)
template <int DC, bool INPLACE>
__device__ __forceinline__ void check_bp_compute(const double (&x)[DC], typename Msg<INPLACE>::out dst)
{
    constexpr int SEG = 8;
    constexpr int NSEG = (DC + SEG - 1) / SEG;
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
        // opaque copy: stops the compiler from CSE-ing the recomputed prefixes
        // with the forward pass (which would keep all DC prefixes live)
        asm volatile("" : "+v"(q));
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const int k = g * SEG + i;
            if (k < DC) { pk[i] = q; q = q * x[k]; }
        }
#pragma unroll
        for (int i = SEG - 1; i >= 0; --i) {
            const int k = g * SEG + i;
            if (k < DC) {
                const double tt = pk[i] * s;
                dst[(size_t)k * TILE] = (1.0 + tt) / (1.0 - tt);
                s = s * x[k];
            }
        }
    }
}

// RES (resident pool, ResStep): messages in place (lr == dmsg, see Msg), the
// lanes run are the tile's occupied ones, every wave also takes its row's
// parity over the previous variable phase's ballots, and every block ends in
// res_arrive (no early exit).
// Block rb of nrb row blocks of tile t; lr_t = the tile's c2v messages.
template <int DC, bool NT, bool RES>
__device__ __forceinline__ void check_bp_block(typename Msg<RES>::in dmsg, typename Msg<RES>::out lr_t,
                                               const uint64_t* __restrict__ active, int32_t M, int64_t E,
                                               int64_t t, uint32_t rb, uint32_t nrb, const ResStep& rs)
{
    const int lane = lane_id();
    const int32_t row = (int32_t)rb * 4 + wave_id();
    const uint64_t act = RES ? rs.cs.occupied[t] : active[t];
    const auto src = dmsg + ((size_t)t * E + (size_t)row * DC) * TILE + lane;
    const auto dst = lr_t + (size_t)row * DC * TILE + lane;
    if constexpr (!RES) {
        // whole-line policy: converged / empty lanes of an active tile run
        // along on their stale state so every c2v store covers whole lines
        // (their values are never read)
        if (!(row < M && line_occupied(act, lane))) return;
        double x[DC];
        check_bp_load<DC, NT, false>(x, src);
        check_bp_compute<DC, false>(x, dst);
    } else {
        // Issue order inside one wave-uniform arm: the row's column indices,
        // its DC message loads, the parity's ballot gathers (which need the
        // indices), the arithmetic, then the XOR reduction -- the gathers'
        // latency hides behind the messages instead of preceding them.  All
        // lanes of an occupied tile run (whole-line stores; unoccupied lanes'
        // values are never read): a lane-masked arm, or a join between the
        // loads and their uses, makes the compiler wait for every outstanding
        // load there.
        static_assert(DC <= 2 * TILE, "row parity: two gathers per lane");
        const bool occ_l = (act >> lane) & 1ull;
        // the lane state for res_arrive's bookkeeping (the tile's last block,
        // on an occupied tile only), loaded up front off the tail's chain
        const int32_t ln0 = rs.cs.lane_n[t * TILE + lane];
        const int64_t b0 = rs.cs.lane_b[t * TILE + lane];
        uint64_t par = 0;
        if (row < M && act != 0) {
            const int32_t* __restrict__ cols = rs.col_idx + (size_t)row * DC;
            const int32_t c0 = cols[lane < DC ? lane : DC - 1];
            const int32_t c1 = cols[TILE + lane < DC ? TILE + lane : DC - 1];
            double x[DC];
            check_bp_load<DC, NT, true>(x, src);
            // opaque copies: the gather addresses (and the wait for the
            // index loads) stay behind the message loads
            int32_t d0 = c0, d1 = c1;
            asm volatile("" : "+v"(d0), "+v"(d1));
            const uint64_t* __restrict__ h = rs.hard + (size_t)t * rs.N;
            const uint64_t g0 = h[d0];
            const uint64_t g1 = h[d1];
            check_bp_compute<DC, true>(x, dst);
            uint64_t p = (lane < DC ? g0 : 0ull) ^ (TILE + lane < DC ? g1 : 0ull);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) p ^= shfl_xor_u64(p, off);
            par = p;
        }
        res_arrive(t, act, par, rs, occ_l ? ln0 : 0, occ_l ? b0 : 0, nrb);
    }
}

// The first check of a single-fill decode (every occupied lane in its first
// iteration; the refill stored only the prior, Refill::prior_only): each
// edge's d0 = 1 - 2/(1+LR) of its column -- the expression and operands of
// the refill (Init_Belief_Propagation dec.cpp:608-629 + the stored d of
// dec.cpp:652) -- gathered from the tile's [N][64] prior instead of read from
// E stored copies; then k_check_bp's arithmetic.  Same grid as k_check_bp.
// PC: the prior is the lanes' int8 codes (pcode) and the LR table (ptab).
template <int DC, bool PC = false>
__global__ __launch_bounds__(256, 2) void k_check_bp_first(const double* __restrict__ prior,
                                                           const int8_t* __restrict__ pcode,
                                                           const double* __restrict__ ptab,
                                                           const int32_t* __restrict__ col_idx,
                                                           double* __restrict__ lr, const uint64_t* __restrict__ active,
                                                           int32_t M, int32_t N, int64_t E, int64_t t0)
{
    const int lane = lane_id();
    const int32_t row = (int32_t)blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    const uint64_t act = active[t];
    if (!(row < M && line_occupied(act, lane))) return;
    const size_t pt = (size_t)t * N * TILE + lane;
    const int32_t* __restrict__ cols = col_idx + (size_t)row * DC;
    double x[DC];
    if constexpr (PC) {
        int8_t k8[DC];
#pragma unroll
        for (int k = 0; k < DC; ++k) k8[k] = pcode[pt + (size_t)cols[k] * TILE];
#pragma unroll
        for (int k = 0; k < DC; ++k) x[k] = ptab[k8[k] + kCodeBias];
    } else {
#pragma unroll
        for (int k = 0; k < DC; ++k) x[k] = prior[pt + (size_t)cols[k] * TILE];
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) x[k] = 1.0 - 2.0 / (1.0 + x[k]);
    check_bp_compute<DC, false>(x, lr + ((size_t)blockIdx.y * E + (size_t)row * DC) * TILE + lane);
}

// Step 0 of a single-fill coded BP decode (the DNA batch): every occupied
// lane was just refilled (Refill::prior_only), so the refill is a transpose
// of the claimed codewords' input rows ([b][N] int8) into the tiles' lane
// codes ([t][N][64], Refill::pcode) plus the ballots of Init_Belief_
// Propagation's decisions LR < 1 (dec.cpp:608-629; LR = ptab[code + 128]).
// Through LDS, 64 columns x 64 lanes per block: each input row segment is
// read as 64 contiguous bytes and each lane-code segment written as 64 --
// instead of the variable kernel's per-lane byte gathers.  N % 64 == 0;
// grid (N / 64, tiles), block 256.
// It replaces the variable kernel of that step only because no lane of the
// tile is live (active) or finished (fin) then: it neither updates nor
// writes outputs.  A tile that breaks this is reported (kFaultSchedule) and
// left alone.
__global__ __launch_bounds__(256) void k_fill_codes(const int8_t* __restrict__ in_code,
                                                    const int64_t* __restrict__ lane_b,
                                                    const uint64_t* __restrict__ fresh, int8_t* __restrict__ pcode,
                                                    const double* __restrict__ ptab, uint64_t* __restrict__ hard,
                                                    int32_t N, int64_t B, unsigned long long* fault,
                                                    const uint64_t* __restrict__ active,
                                                    const uint64_t* __restrict__ fin)
{
    __shared__ int8_t sc[TILE][TILE + 4];
    __shared__ int64_t sb[TILE];
    const int64_t t = blockIdx.y;
    const uint64_t frm = fresh[t];
    if (frm == 0ull) return;  // block-uniform
    if (active[t] != 0ull || fin[t] != 0ull) {  // block-uniform
        if (threadIdx.x == 0) lane_index_ok(-1 - t, 0, fault, kFaultSchedule);
        return;
    }
    const int lane = lane_id(), w = wave_id();
    const int32_t j0 = (int32_t)blockIdx.x * TILE;
    if (threadIdx.x < TILE) {
        int64_t b = ((frm >> lane) & 1ull) ? lane_b[t * TILE + lane] : -1;
        if (b >= 0 && !lane_index_ok(b, B, fault, kFaultRefill)) b = -1;
        sb[lane] = b;
    }
    __syncthreads();
    for (int l = w; l < TILE; l += 4) {
        const int64_t b = sb[l];
        sc[l][lane] = b >= 0 ? in_code[(size_t)b * N + j0 + lane] : (int8_t)0;
    }
    __syncthreads();
    const bool fr = (frm >> lane) & 1ull;
    for (int c = w; c < TILE; c += 4) {
        const int8_t k = sc[lane][c];
        const size_t o = (size_t)t * N + j0 + c;
        pcode[o * TILE + lane] = k;
        const uint64_t m = __ballot(fr && ptab[k + kCodeBias] < 1.0);
        if (lane == 0) hard[o] = (frm == ~0ull) ? m : ((hard[o] & ~frm) | m);
    }
}

// grid (ceil(M/4), tiles t0 .. t0+gridDim.y-1); lr: the group's c2v scratch
// ([t - t0][E][64]), or with RES the pool's messages themselves (in place).
template <int DC, bool NT, bool RES>
__global__ __launch_bounds__(256, 2) void k_check_bp(typename Msg<RES>::in dmsg, typename Msg<RES>::out lr,
                                                     const uint64_t* __restrict__ active, int32_t M, int64_t E,
                                                     int64_t t0, ResStep rs)
{
    check_bp_block<DC, NT, RES>(dmsg, lr + (size_t)blockIdx.y * E * TILE, active, M, E, t0 + blockIdx.y, blockIdx.x,
                                gridDim.x, rs);
}

// Generic row degree: the prefix products go through the lr array exactly as
// the reference does (e->lr = dl in the forward pass, dec.cpp:650-653).
__global__ __launch_bounds__(256) void k_check_bp_gen(const double* __restrict__ dmsg, double* __restrict__ lr,
                                                      const uint64_t* __restrict__ active,
                                                      const int32_t* __restrict__ row_ptr, int32_t M, int64_t E,
                                                      int64_t t0)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (row >= M) return;
    const uint64_t act = active[t];
    if (!((act >> lane) & 1ull)) return;
    const int32_t a = row_ptr[row], b = row_ptr[row + 1];
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    double dl = 1.0;
    for (int32_t e = a; e < b; ++e) {
        lr[(tl + e) * TILE + lane] = dl;
        dl = dl * dmsg[(tb + e) * TILE + lane];
    }
    dl = 1.0;
    for (int32_t e = b - 1; e >= a; --e) {
        const size_t o = (tl + e) * TILE + lane;
        const double tt = lr[o] * dl;
        lr[o] = (1.0 + tt) / (1.0 - tt);
        dl = dl * dmsg[(tb + e) * TILE + lane];
    }
}

// A lane's prior at [tile][N][64] index i: the fp64 value, or with PC (coded
// input) the table value of its int8 code -- 1 byte per column and lane moves
// instead of 8; the table (2 KB) stays in the L1 / L2.
template <bool PC>
__device__ __forceinline__ double prior_at(const double* __restrict__ prior, const Refill& rf, size_t i)
{
    if constexpr (PC) return rf.ptab[rf.pcode[i] + kCodeBias];
    else return prior[i];
}

// ---------------------------------------------------------------------------
// Variable-node phase, regular column degree DV, CPW consecutive columns per
// wave (every c2v load of the wave's columns is issued before the first
// column's arithmetic -- fewer, longer-lived waves).  Requires N % (4 * CPW)
// == 0 (CPW = 1: any N).  Per column and lane:
//   BP (MSA = false, dec.cpp:667-693):
//     forward  pr_s = P_s; P_{s+1} = P_s * lr_s; P_0 = LR
//     P = P_DV; NaN -> 1; dblk = (P <= 1)
//     backward acc = 1; s = DV-1..0: pr_s *= acc; NaN -> 1; acc *= lr_s
//     then stores d_s = 1 - 2/(1+pr_s) for the next check phase
//   min-sum (MSA = true, Variable_Update_MSA_INF dec.cpp:1597-1619 +
//   Decision_MSA_INF dec.cpp:1659-1678):
//     v2c_s = ((LLR + c_0) + c_1) ... skipping c_s, ascending row order
//     L = LLR + c_0 + ... + c_{DV-1};  dblk = !(L > 0)
// and the ballot of the hard decisions; post (optional) receives P / L.
// CONT: refilled lanes (Refill::fresh) get Init_Belief_Propagation
// (dec.cpp:608-629) / Init_MSA_INF (dec.cpp:1300-1329) through the same
// stores, and finished lanes (Refill::fin) get their outputs written first.
// INPLACE: v2c == c2v (resident pool), see Msg.  PC (coded input, CONT
// only): the lanes' priors are int8 codes (Refill::pcode / ptab), refills
// read the input's codes (Refill::in_code).
// Column block cb (4 waves x CPW columns) of tile t; c2v_t = the tile's c2v messages.
template <bool MSA, int DV, bool NT, bool CONT, int CPW, bool INPLACE, bool PC = false>
__device__ __forceinline__ void var_m_block(typename Msg<INPLACE>::in c2v_t, typename Msg<INPLACE>::out v2c,
                                            double* __restrict__ prior, uint64_t* __restrict__ hard,
                                            const uint64_t* __restrict__ active, const int32_t* __restrict__ col_edge,
                                            double* __restrict__ post, int32_t N, int64_t E, int64_t t, uint32_t cb,
                                            const Refill& rf)
{
    const int lane = lane_id();
    const int32_t j0 = ((int32_t)cb * 4 + wave_id()) * CPW;
    if (j0 >= N) return;
    const uint64_t act = active[t];
    const uint64_t frm = CONT ? rf.fresh[t] : 0ull;
    const uint64_t touched = act | frm;
    // resident pool: lanes whose codeword finished at this step's syndrome
    // (their outputs are written here, before a refill overwrites the lane)
    const uint64_t fm = (CONT && rf.fin) ? rf.fin[t] : 0ull;
    if (touched == 0 && fm == 0) return;
    const bool live = (act >> lane) & 1ull;
    const bool fr = CONT && ((frm >> lane) & 1ull);
    const bool fl = (fm >> lane) & 1ull;
    int64_t fb = 0;
    int32_t fn = 0;
    if (fl) {
        fb = rf.fin_b[t * TILE + lane];
        fn = rf.fin_n[t * TILE + lane];
    }
    const size_t tb = (size_t)t * E;
    int32_t eid[CPW][DV];
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int s = 0; s < DV; ++s) eid[c][s] = col_edge[(size_t)(j0 + c) * DV + s];
    double l[CPW][DV], pv[CPW], xin[CPW];
    int8_t kin[CPW];  // PC: the refilled lane's input codes
    // a refilled lane's out-of-range index, reported at the end: held in a
    // VGPR (opaque copy below), as a lane mask in SGPRs it pushed
    // k_var_msa_c past 96 SGPRs (6 instead of 7 waves per SIMD, config 5 -3 %)
    bool bad_in = false;
    int bad_v = 0;
    if (fr) {  // refilled lane: its input row, prefetched with the c2v loads
        const size_t rb = (size_t)refill_row(rf.lane_b[t * TILE + lane], rf, bad_in) * N;
        bad_v = bad_in ? 1 : 0;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            if constexpr (PC) kin[c] = rf.in_code[rb + j0 + c];
            else xin[c] = rf.in[rb + j0 + c];
        }
    }
    if (live) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            pv[c] = prior_at<PC>(prior, rf, ((size_t)t * N + j0 + c) * TILE + lane);
#pragma unroll
            for (int s = 0; s < DV; ++s) l[c][s] = c2v_t[(size_t)eid[c][s] * TILE + lane];
        }
    }
    if constexpr (PC) {
        if (fr) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) xin[c] = rf.ptab[kin[c] + kCodeBias];
        }
    }
    // the finished codeword's index bounds: a plain compare at the stores
    // (a check with its fault report where fin_b is loaded makes every wave
    // wait for that load before its message loads: config 5 -2.4 %); the
    // report itself comes last (lane_fault_report)
    const bool fok = out_ok(fb, rf);
    if (CONT && fl && fok) {  // finished codeword: hard bits of its exit (ballots before this step's update)
        uint64_t hw[CPW];
#pragma unroll
        for (int c = 0; c < CPW; ++c) hw[c] = hard[(size_t)t * N + j0 + c];
        store_fin_hard<CPW>(rf, hw, fb, N, j0, lane);
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int32_t j = j0 + c;
        const size_t pj = ((size_t)t * N + j) * TILE + lane;
        if (CONT && fl && fok && rf.post_out) {  // finished codeword: posterior of its exit
            const size_t ob = (size_t)fb * N + j;
            const double pv = fn > 0 ? post[pj] : prior_at<PC>(prior, rf, pj);
            if (MSA) rf.post_out[ob] = pv;
            else {
                const double P = __builtin_isnan(pv) ? 1.0 : pv;
                rf.post_out[ob] = rf.post_ratio ? P : log(P);
            }
        }
        bool h = false;
        double dv[DV];
#pragma unroll
        for (int s = 0; s < DV; ++s) dv[s] = 0.0;
        double np = 0.0;  // the prior this lane holds after the step (refill: its new one)
        if (live) np = pv[c];
        if (fr) {  // Init_Belief_Propagation / Init_MSA_INF for a refilled lane
            const double x = xin[c];
            if (MSA) {
                np = x;
#pragma unroll
                for (int s = 0; s < DV; ++s) dv[s] = x;
                h = !(x > 0);
            } else {
                // PC: the table holds LR already (the host exp of the caller's LLR table)
                const double LR0 = (!PC && rf.in_is_llr) ? exp(x) : x;
                np = LR0;
                const double d0 = 1.0 - 2.0 / (1.0 + LR0);
#pragma unroll
                for (int s = 0; s < DV; ++s) dv[s] = d0;
                h = (LR0 < 1.0);
            }
        } else if (live) {
            if (MSA) {  // v2c_s = LLR + c_0 + ... (skipping c_s); L = LLR + all
#pragma unroll
                for (int s = 0; s < DV; ++s) {
                    double sum = pv[c];
#pragma unroll
                    for (int r = 0; r < DV; ++r)
                        if (r != s) sum = sum + l[c][r];
                    dv[s] = sum;
                }
                double L = pv[c];
#pragma unroll
                for (int s = 0; s < DV; ++s) L = L + l[c][s];
                h = !(L > 0);
                if (post) post[pj] = L;
            } else {
                double pr[DV];
                double p = pv[c];
#pragma unroll
                for (int s = 0; s < DV; ++s) { pr[s] = p; p = p * l[c][s]; }
                if (__builtin_isnan(p)) p = 1.0;
                h = (p <= 1.0);
                if (post) post[pj] = p;
                double acc = 1.0;
#pragma unroll
                for (int s = DV - 1; s >= 0; --s) {
                    double v = pr[s] * acc;
                    if (__builtin_isnan(v)) v = 1.0;
                    acc = acc * l[c][s];
                    dv[s] = 1.0 - 2.0 / (1.0 + v);
                }
            }
        }
        if (CONT && fr) {
            if constexpr (PC) rf.pcode[pj] = kin[c];
            else prior[pj] = np;
        }
        // whole-line stores (others write 0, never read) -- not in a tile that
        // only hands out finished codewords (no live or refilled lane), nor
        // for refills whose first check reads the prior (Refill::prior_only)
        const bool skip_init = CONT && rf.prior_only && !live;
        if (!skip_init && (line_occupied(touched, lane) || fr || live)) {
#pragma unroll
            for (int s = 0; s < DV; ++s) st<NT>(v2c + (tb + eid[c][s]) * TILE + lane, dv[s]);
        }
        const uint64_t m = __ballot(h);
        if (lane == 0 && touched) {
            const size_t o = (size_t)t * N + j;
            const uint64_t old = (touched == ~0ull) ? 0ull : hard[o];
            hard[o] = (old & ~touched) | (m & touched);
        }
    }
    // the reports of skipped accesses: the lane's pool slot (the indices need
    // not stay live; cont_lanes reports an out-of-range index itself)
    if (CONT && fl && !fok) lane_fault(rf.fault, kFaultOutput, t * TILE + lane);
    asm volatile("" : "+v"(bad_v));
    if (bad_v) lane_fault(rf.fault, kFaultRefill, t * TILE + lane);
}

template <bool MSA, int DV, bool NT, bool CONT, int CPW, bool INPLACE, bool PC = false>
__global__ __launch_bounds__(256) void k_var_m(typename Msg<INPLACE>::in c2v, typename Msg<INPLACE>::out v2c,
                                               double* __restrict__ prior, uint64_t* __restrict__ hard,
                                               const uint64_t* __restrict__ active,
                                               const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                               int32_t N, int64_t E, int64_t t0, Refill rf)
{
    static_assert(CONT || !PC, "coded priors come with continuous refills");
    var_m_block<MSA, DV, NT, CONT, CPW, INPLACE, PC>(c2v + (size_t)blockIdx.y * E * TILE, v2c, prior, hard, active,
                                                 col_edge, post, N, E, t0 + blockIdx.y,
                                                 xcd_block(blockIdx.x, gridDim.x), rf);
}

// Generic column degree: the partial products go through the v2c array
// exactly as the reference keeps them in e->pr.
__global__ __launch_bounds__(256) void k_var_bp_gen(const double* __restrict__ lr, double* __restrict__ dmsg,
                                                    const double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                    const uint64_t* __restrict__ active, const int32_t* __restrict__ col_ptr,
                                                    const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                    int32_t N, int64_t E, int64_t t0)
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
        double p = prior[pj];
        for (int32_t q = a; q < b; ++q) {
            const int32_t e = col_edge[q];
            dmsg[(tb + e) * TILE + lane] = p;
            p = p * lr[(tl + e) * TILE + lane];
        }
        if (__builtin_isnan(p)) p = 1.0;
        h = (p <= 1.0);
        if (post) post[pj] = p;
        double acc = 1.0;
        for (int32_t q = b - 1; q >= a; --q) {
            const int32_t e = col_edge[q];
            const size_t o = (tb + e) * TILE + lane;
            double v = dmsg[o] * acc;
            if (__builtin_isnan(v)) v = 1.0;
            acc = acc * lr[(tl + e) * TILE + lane];
            dmsg[o] = 1.0 - 2.0 / (1.0 + v);
        }
    }
    const uint64_t m = __ballot(h);
    if (lane == 0) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (act == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~act) | (m & act);
    }
}

// ---------------------------------------------------------------------------
// Min-sum check-node phase (Check_Update_MSA_INF dec.cpp:1398-1433) in O(dc):
// for edge k the reference scans the other edges o in order with
//   if (mag == -1 || mag > |x_o|) mag = |x_o|;   sign *= (x_o >= 0 ? 1 : -1)
// which equals: |x_f| if it is NaN (f = first other edge: 1 for k = 0, else 0
// -- a NaN first value sticks because every later comparison is false),
// otherwise the minimum over the non-NaN others = (k == argmin ? min2 : min1)
// with argmin the FIRST index of the minimum.  sign = product over others of
// (x >= 0 ? +1 : -1) (NaN counts -1).  c2v = (double)sign * mag.
// dc == 1: mag stays -1 -> 0, sign 1 -> 0.0 (dec.cpp:1427-1430).
// ---------------------------------------------------------------------------
template <int DC, bool NT, bool INPLACE>
__device__ __forceinline__ void check_msa_row(typename Msg<INPLACE>::in src, typename Msg<INPLACE>::out dst)
{
    double x[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) x[k] = ld<NT>(src + (size_t)k * TILE);
    if constexpr (DC == 1) {
        dst[0] = 0.0;
        return;
    }
    double m1 = __builtin_inf(), m2 = __builtin_inf();
    int i1 = -1;
    uint32_t neg = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const double a = __builtin_fabs(x[k]);
        neg ^= (x[k] >= 0) ? 0u : 1u;
        if (a < m1) { m1 = a; i1 = k; }  // NaN never compares less; first index kept
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const double a = __builtin_fabs(x[k]);
        if (k != i1 && a < m2) m2 = a;
    }
    const double a0 = __builtin_fabs(x[0]), a1 = __builtin_fabs(x[DC > 1 ? 1 : 0]);
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const double af = (k == 0) ? a1 : a0;
        double mag = (k == i1) ? m2 : m1;
        if (__builtin_isnan(af)) mag = af;
        const uint32_t nk = (x[k] >= 0) ? 0u : 1u;
        const int sign = ((neg ^ nk) & 1u) ? -1 : 1;
        dst[(size_t)k * TILE] = (double)sign * mag;
    }
}

// RES: resident pool, as k_check_bp's (in place, row parity, res_arrive).
template <int DC, bool NT, bool RES>
__global__ __launch_bounds__(256) void k_check_msa(typename Msg<RES>::in v2c, typename Msg<RES>::out c2v,
                                                   const uint64_t* __restrict__ active, int32_t M, int64_t E,
                                                   int64_t t0, ResStep rs)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    const uint64_t act = RES ? rs.cs.occupied[t] : active[t];
    // whole-line policy: converged / empty lanes of an active tile run along on
    // their stale state so every c2v store covers whole lines (never read)
    const bool run = row < M && line_occupied(act, lane);
    if constexpr (!RES) {
        if (!run) return;
    }
    uint64_t par = 0;
    int32_t ln0 = 0;
    int64_t b0 = 0;
    if (RES && act != 0) {
        // the lane state for res_arrive's bookkeeping (used by the tile's last
        // block only), loaded up front so it is not on the tail's chain
        if (threadIdx.x < TILE && ((act >> lane) & 1ull)) {
            ln0 = rs.cs.lane_n[t * TILE + lane];
            b0 = rs.cs.lane_b[t * TILE + lane];
        }
        if (row < M) par = row_parity<DC>(rs.hard + (size_t)t * rs.N, rs.col_idx + (size_t)row * DC);
    }
    if (run)
        check_msa_row<DC, NT, RES>(v2c + ((size_t)t * E + (size_t)row * DC) * TILE + lane,
                                   c2v + ((size_t)blockIdx.y * E + (size_t)row * DC) * TILE + lane);
    if constexpr (RES) res_arrive(t, act, par, rs, ln0, b0, gridDim.x);
}

__global__ __launch_bounds__(256) void k_check_msa_gen(const double* __restrict__ v2c, double* __restrict__ c2v,
                                                       const uint64_t* __restrict__ active,
                                                       const int32_t* __restrict__ row_ptr, int32_t M, int64_t E,
                                                       int64_t t0)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (row >= M) return;
    const uint64_t act = active[t];
    if (!((act >> lane) & 1ull)) return;
    const int32_t a = row_ptr[row], b = row_ptr[row + 1];
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    if (b - a == 0) return;
    if (b - a == 1) { c2v[(tl + a) * TILE + lane] = 0.0; return; }
    double m1 = __builtin_inf(), m2 = __builtin_inf();
    int32_t i1 = -1;
    uint32_t neg = 0;
    for (int32_t e = a; e < b; ++e) {
        const double xv = v2c[(tb + e) * TILE + lane];
        const double av = __builtin_fabs(xv);
        neg ^= (xv >= 0) ? 0u : 1u;
        if (av < m1) { m1 = av; i1 = e; }
    }
    for (int32_t e = a; e < b; ++e) {
        const double av = __builtin_fabs(v2c[(tb + e) * TILE + lane]);
        if (e != i1 && av < m2) m2 = av;
    }
    const double a0 = __builtin_fabs(v2c[(tb + a) * TILE + lane]);
    const double a1 = __builtin_fabs(v2c[(tb + a + 1) * TILE + lane]);
    for (int32_t e = a; e < b; ++e) {
        const double xv = v2c[(tb + e) * TILE + lane];
        const double af = (e == a) ? a1 : a0;
        double mag = (e == i1) ? m2 : m1;
        if (__builtin_isnan(af)) mag = af;
        const uint32_t nk = (xv >= 0) ? 0u : 1u;
        const int sign = ((neg ^ nk) & 1u) ? -1 : 1;
        c2v[(tl + e) * TILE + lane] = (double)sign * mag;
    }
}

__global__ __launch_bounds__(256) void k_var_msa_gen(const double* __restrict__ c2v, double* __restrict__ v2c,
                                                     const double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                     const uint64_t* __restrict__ active, const int32_t* __restrict__ col_ptr,
                                                     const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                     int32_t N, int64_t E, int64_t t0)
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
        const double llr = prior[pj];
        // v2c is written only after all sums are formed, c2v is read-only here
        for (int32_t s = a; s < b; ++s) {
            double sum = llr;
            for (int32_t r = a; r < b; ++r)
                if (r != s) sum = sum + c2v[(tl + col_edge[r]) * TILE + lane];
            v2c[(tb + col_edge[s]) * TILE + lane] = sum;
        }
        double L = llr;
        for (int32_t s = a; s < b; ++s) L = L + c2v[(tl + col_edge[s]) * TILE + lane];
        h = !(L > 0);
        if (post) post[pj] = L;
    }
    const uint64_t m = __ballot(h);
    if (lane == 0) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (act == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~act) | (m & act);
    }
}

// ---------------------------------------------------------------------------
// Generic degrees staged in registers (codes other than the (8, 72)-regular
// one; fixed passes).  A row / column of degree d <= D keeps its messages in
// VGPRs: one load and one store per edge, where the *_gen kernels above take
// their partial products through memory (about 40 B per edge per phase
// instead of 16).  D is the engine's bucket for the graph's maximum degree
// (engine.hip kGenBuckets); every loop runs the same operations in the same
// order as the *_gen kernels (and the reference), guarded by k < d.
template <int D, bool INPLACE = false>
__device__ __forceinline__ void check_bp_compute_rt(const double (&x)[D], int32_t d, typename Msg<INPLACE>::out dst)
{
    constexpr int SEG = 8;
    constexpr int NSEG = (D + SEG - 1) / SEG;
    double cp[NSEG];
    double p = 1.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        if (k < d) {
            if (k % SEG == 0) cp[k / SEG] = p;
            p = p * x[k];
        }
    }
    double s = 1.0;
#pragma unroll
    for (int g = NSEG - 1; g >= 0; --g) {
        if (g * SEG >= d) continue;
        double pk[SEG];
        double q = cp[g];
        asm volatile("" : "+v"(q));  // (as check_bp_compute: no CSE with the forward pass)
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const int k = g * SEG + i;
            if (k < D && k < d) { pk[i] = q; q = q * x[k]; }
        }
#pragma unroll
        for (int i = SEG - 1; i >= 0; --i) {
            const int k = g * SEG + i;
            if (k < D && k < d) {
                const double tt = pk[i] * s;
                dst[(size_t)k * TILE] = (1.0 + tt) / (1.0 - tt);
                s = s * x[k];
            }
        }
    }
}

// BP check phase (dec.cpp:646-662), rows of degree <= D in registers
template <int D>
__global__ __launch_bounds__(256) void k_check_bp_gr(const double* __restrict__ dmsg, double* __restrict__ lr,
                                                     const uint64_t* __restrict__ active,
                                                     const int32_t* __restrict__ row_ptr, int32_t M, int64_t E,
                                                     int64_t t0)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (row >= M) return;
    if (!((active[t] >> lane) & 1ull)) return;
    const int32_t a = row_ptr[row], d = row_ptr[row + 1] - a;
    const double* src = dmsg + ((size_t)t * E + a) * TILE + lane;
    double* dst = lr + ((size_t)blockIdx.y * E + a) * TILE + lane;
    double x[D];
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (k < d) x[k] = src[(size_t)k * TILE];
    check_bp_compute_rt<D>(x, d, dst);
}

// min-sum check phase (dec.cpp:1398-1433, as k_check_msa_gen), rows of
// degree <= D in registers
template <int D>
__global__ __launch_bounds__(256) void k_check_msa_gr(const double* __restrict__ v2c, double* __restrict__ c2v,
                                                      const uint64_t* __restrict__ active,
                                                      const int32_t* __restrict__ row_ptr, int32_t M, int64_t E,
                                                      int64_t t0)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (row >= M) return;
    if (!((active[t] >> lane) & 1ull)) return;
    const int32_t a = row_ptr[row], d = row_ptr[row + 1] - a;
    double* dst = c2v + ((size_t)blockIdx.y * E + a) * TILE + lane;
    if (d == 0) return;
    if (d == 1) { dst[0] = 0.0; return; }
    const double* src = v2c + ((size_t)t * E + a) * TILE + lane;
    double x[D];
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (k < d) x[k] = src[(size_t)k * TILE];
    double m1 = __builtin_inf(), m2 = __builtin_inf();
    int32_t i1 = -1;
    uint32_t neg = 0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        if (k < d) {
            const double av = __builtin_fabs(x[k]);
            neg ^= (x[k] >= 0) ? 0u : 1u;
            if (av < m1) { m1 = av; i1 = k; }
        }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        if (k < d) {
            const double av = __builtin_fabs(x[k]);
            if (k != i1 && av < m2) m2 = av;
        }
    }
    const double a0 = __builtin_fabs(x[0]), a1 = __builtin_fabs(x[1]);
#pragma unroll
    for (int k = 0; k < D; ++k) {
        if (k < d) {
            const double af = (k == 0) ? a1 : a0;
            double mag = (k == i1) ? m2 : m1;
            if (__builtin_isnan(af)) mag = af;
            const uint32_t nk = (x[k] >= 0) ? 0u : 1u;
            const int sign = ((neg ^ nk) & 1u) ? -1 : 1;
            dst[(size_t)k * TILE] = (double)sign * mag;
        }
    }
}

// BP variable phase + decision (dec.cpp:667-693, as k_var_bp_gen), columns
// of degree <= D in registers
template <int D>
__global__ __launch_bounds__(256) void k_var_bp_gr(const double* __restrict__ lr, double* __restrict__ dmsg,
                                                   const double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                   const uint64_t* __restrict__ active,
                                                   const int32_t* __restrict__ col_ptr,
                                                   const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                   int32_t N, int64_t E, int64_t t0)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (j >= N) return;
    const uint64_t act = active[t];
    if (act == 0) return;
    const bool live = (act >> lane) & 1ull;
    const int32_t a = col_ptr[j], d = col_ptr[j + 1] - a;
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    bool h = false;
    if (live) {
        int32_t eid[D];
        double l[D], pr[D];
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) eid[s] = col_edge[a + s];
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) l[s] = lr[(tl + eid[s]) * TILE + lane];
        const size_t pj = ((size_t)t * N + j) * TILE + lane;
        double p = prior[pj];
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) { pr[s] = p; p = p * l[s]; }
        if (__builtin_isnan(p)) p = 1.0;
        h = (p <= 1.0);
        if (post) post[pj] = p;
        double acc = 1.0;
#pragma unroll
        for (int s = D - 1; s >= 0; --s) {
            if (s < d) {
                double v = pr[s] * acc;
                if (__builtin_isnan(v)) v = 1.0;
                acc = acc * l[s];
                dmsg[(tb + eid[s]) * TILE + lane] = 1.0 - 2.0 / (1.0 + v);
            }
        }
    }
    const uint64_t m = __ballot(h);
    if (lane == 0) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (act == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~act) | (m & act);
    }
}

// min-sum variable phase + decision (dec.cpp:1597-1619, 1659-1678, as
// k_var_msa_gen), columns of degree <= D in registers
template <int D>
__global__ __launch_bounds__(256) void k_var_msa_gr(const double* __restrict__ c2v, double* __restrict__ v2c,
                                                    const double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                    const uint64_t* __restrict__ active,
                                                    const int32_t* __restrict__ col_ptr,
                                                    const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                    int32_t N, int64_t E, int64_t t0)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (j >= N) return;
    const uint64_t act = active[t];
    if (act == 0) return;
    const bool live = (act >> lane) & 1ull;
    const int32_t a = col_ptr[j], d = col_ptr[j + 1] - a;
    const size_t tb = (size_t)t * E, tl = (size_t)blockIdx.y * E;
    bool h = false;
    if (live) {
        int32_t eid[D];
        double c[D];
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) eid[s] = col_edge[a + s];
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) c[s] = c2v[(tl + eid[s]) * TILE + lane];
        const size_t pj = ((size_t)t * N + j) * TILE + lane;
        const double llr = prior[pj];
#pragma unroll
        for (int s = 0; s < D; ++s) {
            if (s < d) {
                double sum = llr;
#pragma unroll
                for (int r = 0; r < D; ++r)
                    if (r < d && r != s) sum = sum + c[r];
                v2c[(tb + eid[s]) * TILE + lane] = sum;
            }
        }
        double L = llr;
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) L = L + c[s];
        h = !(L > 0);
        if (post) post[pj] = L;
    }
    const uint64_t m = __ballot(h);
    if (lane == 0) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (act == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~act) | (m & act);
    }
}

// Resident pool for row degrees <= D (codes other than the (8, 72)-regular
// one): k_check_bp_gr / k_check_msa_gr in place over the pool tile
// blockIdx.y, plus the fused syndrome of the previous variable phase (the
// row's parity over its ballots, CSR row_ptr / col_idx) and the tile's lane
// bookkeeping by its last block (res_arrive), as k_check_bp<72, ., true>.
// Every lane of an occupied 16-lane line runs (whole-line stores); no early
// return (res_arrive synchronises the block).
template <bool MSA, int D>
__global__ __launch_bounds__(256) void k_check_gr_res(double* msg, const int32_t* __restrict__ row_ptr, int32_t M,
                                                      int64_t E, ResStep rs)
{
    const int lane = lane_id();
    const int32_t row = blockIdx.x * 4 + wave_id();
    const int64_t t = blockIdx.y;
    const uint64_t act = rs.cs.occupied[t];
    uint64_t par = 0;
    int32_t ln0 = 0;
    int64_t b0 = 0;
    int32_t a = 0, d = 0;
    if (row < M) {
        a = row_ptr[row];
        d = row_ptr[row + 1] - a;
    }
    if (act != 0) {
        if (threadIdx.x < TILE && ((act >> lane) & 1ull)) {
            ln0 = rs.cs.lane_n[t * TILE + lane];
            b0 = rs.cs.lane_b[t * TILE + lane];
        }
        if (row < M) {
            const uint64_t* __restrict__ h = rs.hard + (size_t)t * rs.N;
            for (int32_t k0 = 0; k0 < d; k0 += TILE)
                if (k0 + lane < d) par ^= h[rs.col_idx[a + k0 + lane]];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) par ^= shfl_xor_u64(par, off);
        }
    }
    if (row < M && line_occupied(act, lane) && d > 0) {
        double* p = msg + ((size_t)t * E + a) * TILE + lane;
        if (MSA && d == 1) {
            p[0] = 0.0;
        } else {
            double x[D];
#pragma unroll
            for (int k = 0; k < D; ++k)
                if (k < d) x[k] = p[(size_t)k * TILE];
            if constexpr (MSA) {
                double m1 = __builtin_inf(), m2 = __builtin_inf();
                int32_t i1 = -1;
                uint32_t neg = 0;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    if (k < d) {
                        const double av = __builtin_fabs(x[k]);
                        neg ^= (x[k] >= 0) ? 0u : 1u;
                        if (av < m1) { m1 = av; i1 = k; }
                    }
                }
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    if (k < d) {
                        const double av = __builtin_fabs(x[k]);
                        if (k != i1 && av < m2) m2 = av;
                    }
                }
                const double a0 = __builtin_fabs(x[0]), a1 = __builtin_fabs(x[1]);
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    if (k < d) {
                        const double af = (k == 0) ? a1 : a0;
                        double mag = (k == i1) ? m2 : m1;
                        if (__builtin_isnan(af)) mag = af;
                        const uint32_t nk = (x[k] >= 0) ? 0u : 1u;
                        const int sign = ((neg ^ nk) & 1u) ? -1 : 1;
                        p[(size_t)k * TILE] = (double)sign * mag;
                    }
                }
            } else {
                check_bp_compute_rt<D, true>(x, d, p);
            }
        }
    }
    res_arrive(t, act, par, rs, ln0, b0, gridDim.x);
}

// Continuous mode for column degrees <= D (codes other than the
// (8, 72)-regular one; INPLACE: the resident pool, v2c == c2v, every load of
// the column's edges ahead of its first store): var_m_block's lane handling -- finished lanes' outputs
// first, refilled lanes' Init_Belief_Propagation (dec.cpp:608-629) /
// Init_MSA_INF (dec.cpp:1300-1329), live lanes' update as k_var_bp_gr /
// k_var_msa_gr -- for one column per wave with the degree read from col_ptr.
// PC: coded priors (Refill::pcode / ptab, refills from Refill::in_code).
template <bool MSA, int D, bool PC, bool INPLACE = false>
__global__ __launch_bounds__(256) void k_var_gr_cont(typename Msg<INPLACE>::in c2v, typename Msg<INPLACE>::out v2c,
                                                     double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                     const uint64_t* __restrict__ active,
                                                     const int32_t* __restrict__ col_ptr,
                                                     const int32_t* __restrict__ col_edge, double* __restrict__ post,
                                                     int32_t N, int64_t E, int64_t t0, Refill rf)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = t0 + blockIdx.y;
    if (j >= N) return;
    const uint64_t act = active[t];
    const uint64_t frm = rf.fresh[t];
    const uint64_t touched = act | frm;
    const uint64_t fm = rf.fin ? rf.fin[t] : 0ull;
    if (touched == 0 && fm == 0) return;
    const bool live = (act >> lane) & 1ull;
    const bool fr = (frm >> lane) & 1ull;
    const bool fl = (fm >> lane) & 1ull;
    int64_t fb = 0;
    int32_t fn = 0;
    if (fl) {
        fb = rf.fin_b[t * TILE + lane];
        fn = rf.fin_n[t * TILE + lane];
    }
    const int32_t a = col_ptr[j], d = col_ptr[j + 1] - a;
    const size_t tb = (size_t)t * E;
    typename Msg<INPLACE>::in c2v_t = c2v + (size_t)blockIdx.y * E * TILE;
    int32_t eid[D];
#pragma unroll
    for (int s = 0; s < D; ++s)
        if (s < d) eid[s] = col_edge[a + s];
    bool bad_in = false;
    int bad_v = 0;
    double xin = 0.0;
    int8_t kin = 0;
    if (fr) {  // refilled lane: its input value, loaded with the c2v loads
        const size_t rb = (size_t)refill_row(rf.lane_b[t * TILE + lane], rf, bad_in) * N;
        bad_v = bad_in ? 1 : 0;
        if constexpr (PC) kin = rf.in_code[rb + j];
        else xin = rf.in[rb + j];
    }
    const size_t pj = ((size_t)t * N + j) * TILE + lane;
    double l[D];
    double pv = 0.0;
    if (live) {
        pv = prior_at<PC>(prior, rf, pj);
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) l[s] = c2v_t[(size_t)eid[s] * TILE + lane];
    }
    if constexpr (PC) {
        if (fr) xin = rf.ptab[kin + kCodeBias];
    }
    const bool fok = out_ok(fb, rf);
    if (fl && fok) {  // finished codeword: hard bits of its exit (ballots before this step's update)
        const uint64_t hw[1] = {hard[(size_t)t * N + j]};
        store_fin_hard<1>(rf, hw, fb, N, j, lane);
        if (rf.post_out) {  // and its posterior
            const double q = fn > 0 ? post[pj] : prior_at<PC>(prior, rf, pj);
            if (MSA) rf.post_out[(size_t)fb * N + j] = q;
            else {
                const double P = __builtin_isnan(q) ? 1.0 : q;
                rf.post_out[(size_t)fb * N + j] = rf.post_ratio ? P : log(P);
            }
        }
    }
    bool h = false;
    double dv[D];
#pragma unroll
    for (int s = 0; s < D; ++s) dv[s] = 0.0;
    double np = live ? pv : 0.0;
    if (fr) {
        const double x = xin;
        if (MSA) {
            np = x;
#pragma unroll
            for (int s = 0; s < D; ++s) dv[s] = x;
            h = !(x > 0);
        } else {
            const double LR0 = (!PC && rf.in_is_llr) ? exp(x) : x;
            np = LR0;
            const double d0 = 1.0 - 2.0 / (1.0 + LR0);
#pragma unroll
            for (int s = 0; s < D; ++s) dv[s] = d0;
            h = (LR0 < 1.0);
        }
    } else if (live) {
        if (MSA) {
#pragma unroll
            for (int s = 0; s < D; ++s) {
                if (s < d) {
                    double sum = pv;
#pragma unroll
                    for (int r = 0; r < D; ++r)
                        if (r < d && r != s) sum = sum + l[r];
                    dv[s] = sum;
                }
            }
            double L = pv;
#pragma unroll
            for (int s = 0; s < D; ++s)
                if (s < d) L = L + l[s];
            h = !(L > 0);
            if (post) post[pj] = L;
        } else {
            double pr[D];
            double p = pv;
#pragma unroll
            for (int s = 0; s < D; ++s)
                if (s < d) { pr[s] = p; p = p * l[s]; }
            if (__builtin_isnan(p)) p = 1.0;
            h = (p <= 1.0);
            if (post) post[pj] = p;
            double acc = 1.0;
#pragma unroll
            for (int s = D - 1; s >= 0; --s) {
                if (s < d) {
                    double v = pr[s] * acc;
                    if (__builtin_isnan(v)) v = 1.0;
                    acc = acc * l[s];
                    dv[s] = 1.0 - 2.0 / (1.0 + v);
                }
            }
        }
    }
    if (fr) {
        if constexpr (PC) rf.pcode[pj] = kin;
        else prior[pj] = np;
    }
    // whole-line stores, as var_m_block (others write 0, never read)
    if (line_occupied(touched, lane) || fr || live) {
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < d) v2c[(tb + eid[s]) * TILE + lane] = dv[s];
    }
    const uint64_t m = __ballot(h);
    if (lane == 0 && touched) {
        const size_t o = (size_t)t * N + j;
        const uint64_t old = (touched == ~0ull) ? 0ull : hard[o];
        hard[o] = (old & ~touched) | (m & touched);
    }
    if (fl && !fok) lane_fault(rf.fault, kFaultOutput, t * TILE + lane);
    asm volatile("" : "+v"(bad_v));
    if (bad_v) lane_fault(rf.fault, kFaultRefill, t * TILE + lane);
}

// Raw buffer resource over [base, base + bytes) (gfx9 data format, no
// swizzle, stride 0).  A wave's gathers and scatters then take a
// wave-uniform byte offset in an SGPR (soffset) and one shared per-lane
// offset in a VGPR: no per-edge 64-bit address arithmetic on the VALU.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBufNT = 2;  // cache-policy bits of a buffer access: nt (gfx950), as __builtin_nontemporal_store
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                            (int)(bytes < 0x7fffffffull ? bytes : 0x7fffffffull), 0x00020000);
}

// ---------------------------------------------------------------------------
// Compressed min-sum check->variable messages ("MSA-C", (DC, DV)-regular
// graphs with E < 2^18).  A row's DC outgoing messages take only four
// magnitudes -- min1, min2 and, in the NaN cases derived above k_check_msa,
// |x_0| or |x_1| -- and a sign, so the check phase writes per (row, lane):
//   rec  [group tile][M][4][64] fp64 planes m1, m2, n0 = |x_0|, n1 = |x_1|
//        (n0 / n1 written only when NaN)
//   meta [group tile][M][64] u16: bit 15 the row's sign parity, bit 14 NaN at
//        x_1, bit 13 NaN at x_0, bit 12 no minimum (every |x| inf or NaN),
//        bits 0-6 the low 7 bits of min1's edge id row * DC + i1 (unique
//        within a row: DC <= 128 consecutive ids)
// and nothing per edge.  The variable phase rebuilds each c2v from the meta
// word, its own edge id and the sign bit of the v2c it stored itself (sgn,
// !(x >= 0) of exactly that value -- the check's sign rule):
//   sign = parity ^ own; mag = (edge == min1 edge) ? min2 : min1, or the NaN
//   plane (|x_1| for the row's first edge, |x_0| for the others)
//   c2v = mag with its sign bit flipped when sign is negative
// which is k_check_msa's (double)sign * mag for every non-NaN mag (+-0, +-inf
// included); a NaN's sign is never observed downstream (comparisons, fabs and
// sums only), so every sum and decision is unchanged.  Per edge and codeword
// the c2v stream shrinks from 16 B (fp64 write + read) to the records, which
// the row's DC columns re-read from the XCD's L2 (see k_var_msa_c).  Planes,
// not {m1, m2} pairs: a wave needs m2 only in the lanes whose codeword has
// its row minimum at this edge (1 in DC), so one load per edge from the plane
// each lane needs fetches the m1 plane's 512 B and only the m2 lines holding
// such a lane -- a pair layout fetches 1 KB per edge, which measured 16 %
// slower (profiles/r3).
// ---------------------------------------------------------------------------
constexpr int MSA_REC_PLANES = 4;
constexpr uint32_t MSA_META_ID = 0x7fu;      // meta bits 0-6: low bits of min1's edge id
constexpr uint32_t MSA_META_NONE = 0x1000u;  // meta bit 12: no min1 (never equals an edge's low bits)

// 1-D grid of gt * ceil(M/4) blocks, block 256: one wave per (row, tile);
// block L works on group tile L % gt, so with gt | 8 each XCD writes the
// records of the one tile whose variable blocks it runs next (k_var_msa_c's
// mapping) and they are read back from its own L2.  The v2c group is
// streamed once (NT: nontemporal loads).
template <int DC, bool NT>
__global__ __launch_bounds__(256) void k_check_msa_c(const double* __restrict__ v2c, double* __restrict__ rec,
                                                     uint16_t* __restrict__ meta, const uint64_t* __restrict__ active,
                                                     const int32_t* __restrict__ row_pos, int32_t M, int64_t E,
                                                     int64_t t0, uint32_t gt)
{
    static_assert(DC >= 2 && DC <= 96, "row degree");
    const int lane = lane_id();
    const uint32_t ty = blockIdx.x % gt;
    const int32_t row = (int32_t)(blockIdx.x / gt) * 4 + wave_id();
    const int64_t t = t0 + ty;
    const uint64_t act = active[t];
    // whole-line policy (as k_check_msa)
    if (!(row < M && line_occupied(act, lane))) return;
    // the row's DC segments through a buffer resource: per-edge offsets in
    // the instructions, one per-lane VGPR offset (no 64-bit addresses)
    // v2c is in column (CSC) order: the row's DC segments are gathered
    // through the CSR -> CSC position table (wave-uniform: scalar loads)
    const auto rv2c = buf_rsrc(v2c + (size_t)t * E * TILE, (uint64_t)E * TILE * 8);
    const int32_t* __restrict__ pos = row_pos + (size_t)row * DC;
    double x[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k)
        x[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rv2c, lane * 8, pos[k] * (TILE * 8),
                                                                               NT ? kBufNT : 0));
    // one pass: min1 with its FIRST index, min2 = minimum over the other
    // indices (a tie with min1 gives min2 == min1), NaN never compares less.
    // Without NaN as min / max (each returns one operand, bit for bit):
    //   m2 = min(m2, max(m1, a)), m1 = min(m1, a), i1 by the strict a < m1
    // -- the selects below, in a third of the VALU work; the sign parity
    // and the NaN flag as lane masks.  A lane with a NaN redoes the row with
    // the selects (max(m1, NaN) would drop the NaN and shrink m2).
    double m1 = __builtin_inf(), m2 = __builtin_inf();
    int i1 = -1;
    bool neg = false, anynan = false;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const double a = __builtin_fabs(x[k]);
        neg ^= !(x[k] >= 0);
        anynan |= __builtin_isnan(a);
        i1 = (a < m1) ? k : i1;
        m2 = __builtin_fmin(m2, __builtin_fmax(m1, a));
        m1 = __builtin_fmin(m1, a);
    }
    if (__builtin_expect(__ballot(anynan) != 0ull, 0) && anynan) {
        m1 = __builtin_inf();
        m2 = __builtin_inf();
        i1 = -1;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            // if (a < m1) { m2 = m1; m1 = a; i1 = k; } else if (a < m2) m2 = a;
            // as selects (no per-edge lane-masked branch); NaN compares false
            const double a = __builtin_fabs(x[k]);
            const bool lt1 = a < m1, lt2 = a < m2;
            m2 = lt1 ? m1 : (lt2 ? a : m2);
            m1 = lt1 ? a : m1;
            i1 = lt1 ? k : i1;
        }
    }
    const double a0 = __builtin_fabs(x[0]), a1 = __builtin_fabs(x[1]);
    const bool nan0 = __builtin_isnan(a0), nan1 = __builtin_isnan(a1);
    double* __restrict__ r = rec + ((size_t)ty * M + row) * (MSA_REC_PLANES * TILE) + lane;
    r[0] = m1;
    r[TILE] = m2;
    if (nan0) r[2 * TILE] = a0;
    if (nan1) r[3 * TILE] = a1;
    meta[((size_t)ty * M + row) * TILE + lane] =
        (uint16_t)(((neg ? 1u : 0u) << 15) | ((nan1 ? 1u : 0u) << 14) | ((nan0 ? 1u : 0u) << 13) |
                   (i1 < 0 ? MSA_META_NONE : ((uint32_t)(row * DC + i1) & MSA_META_ID)));
}

__device__ __forceinline__ double flip_sign(double v, uint32_t neg)
{
    return __longlong_as_double(__double_as_longlong(v) ^ ((long long)(neg & 1u) << 63));
}

// MSA-C column table: per CSC position q (column j's edges, ascending row),
// (row of edge << 18) | edge id -- one wave-uniform word per edge (E < 2^18,
// M < 2^14), so a wave's CPW x DV edges take CPW x DV SGPRs
constexpr int MSA_ER_SHIFT = 18;
constexpr uint32_t MSA_ER_EDGE = (1u << MSA_ER_SHIFT) - 1;
// position of a packed column-table edge in its row (edges are numbered
// row-major: id = row * DC + position); wave-uniform, scalar arithmetic
__device__ __forceinline__ uint32_t er_pos(uint32_t er, int DC)
{
    return (er & MSA_ER_EDGE) - (er >> MSA_ER_SHIFT) * (uint32_t)DC;
}

// Min-sum variable phase on compressed messages (the arithmetic of k_var_m<MSA>).
// 1-D grid of gt * (N / (4 CPW)) blocks; block L works on group tile L % gt.
// Workgroups are dispatched to the 8 XCDs round-robin, so when gt divides 8
// every XCD only ever touches the records of one tile (2.5 MB for the DNA
// code), which stay in its 4 MB L2 while the tile's DC columns per row re-read
// them.  The meta loads of the wave's CPW columns go out together, then the
// record loads (their plane depends on the meta word), all through buffer
// resources (per-edge offsets in SGPRs); NT: nontemporal v2c stores (the
// group's v2c is read back once, by the next check phase).  PC: coded
// priors, as k_var_m.
template <int DC, int DV, bool CONT, int CPW, bool NT, bool PC = false>
__global__ __launch_bounds__(256) void k_var_msa_c(const double* __restrict__ rec, const uint16_t* __restrict__ meta,
                                                   double* __restrict__ v2c,
                                                   double* __restrict__ prior, uint64_t* __restrict__ hard,
                                                   uint8_t* __restrict__ sgn, const uint64_t* __restrict__ active,
                                                   const uint32_t* __restrict__ col_er, double* __restrict__ post,
                                                   int32_t N, int32_t M, int64_t E, int64_t t0, uint32_t gt,
                                                   int32_t vpa, int32_t vpb, Refill rf)
{
    const int lane = lane_id();
    const uint32_t ty = blockIdx.x % gt;
    const int32_t j0 = (int32_t)((blockIdx.x / gt) * 4 + wave_id()) * CPW;
    const int64_t t = t0 + ty;
    if (j0 >= N) return;
    const uint64_t act = active[t];
    const uint64_t frm = CONT ? rf.fresh[t] : 0ull;
    const uint64_t touched = act | frm;
    // lanes whose codeword finished at this step's syndrome (outputs written
    // here, before a refill overwrites the lane; as k_var_m)
    const uint64_t fm = (CONT && rf.fin) ? rf.fin[t] : 0ull;
    if (touched == 0 && fm == 0) return;
    const bool live = (act >> lane) & 1ull;
    const bool fr = CONT && ((frm >> lane) & 1ull);
    const bool fl = (fm >> lane) & 1ull;
    int64_t fb = 0;
    int32_t fn = 0;
    if (fl) {
        fb = rf.fin_b[t * TILE + lane];
        fn = rf.fin_n[t * TILE + lane];
    }
    uint32_t er[CPW][DV];
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int s = 0; s < DV; ++s) er[c][s] = col_er[(size_t)(j0 + c) * DV + s];
    const auto rrec = buf_rsrc(rec + (size_t)ty * M * (MSA_REC_PLANES * TILE), (uint64_t)M * MSA_REC_PLANES * TILE * 8);
    const auto rmeta = buf_rsrc(meta + (size_t)ty * M * TILE, (uint64_t)M * TILE * sizeof(uint16_t));
    const auto rv2c = buf_rsrc(v2c + (size_t)t * E * TILE, (uint64_t)E * TILE * sizeof(double));
    static_assert(CONT || !PC, "coded priors come with continuous refills");
    double l[CPW][DV], pv[CPW], xin[CPW];
    int8_t kin[CPW];  // PC: the refilled lane's input codes
    bool bad_in = false;  // as k_var_m
    int bad_v = 0;
    if (fr) {
        const size_t rb = (size_t)refill_row(rf.lane_b[t * TILE + lane], rf, bad_in) * N;
        bad_v = bad_in ? 1 : 0;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            if constexpr (PC) kin[c] = rf.in_code[rb + j0 + c];
            else xin[c] = rf.in[rb + j0 + c];
        }
    }
    uint32_t cpk[CPW];  // per edge: c2v sign (bit 0) and record plane (bits 1-2), 4 bits each
    if (live) {
        // the meta words first; from them, per edge a 4-bit code (bit 0: the
        // c2v sign = parity ^ own sign, bits 1-2: the record plane -- m2 at the
        // row's min1 edge, a NaN plane when x_0 / x_1 is NaN, else m1), packed
        // 8 to a register; then one record load per edge from the plane each
        // lane needs: the wave fetches the m1 plane's lines plus only the m2
        // lines holding a lane that needs them
        constexpr int PB = TILE * 8;  // bytes per record plane of one row
        uint32_t sb[CPW], mw[CPW][DV];  // mw: the u16 meta words
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            pv[c] = prior_at<PC>(prior, rf, ((size_t)t * N + j0 + c) * TILE + lane);
            sb[c] = sgn[((size_t)t * N + j0 + c) * TILE + lane];
#pragma unroll
            for (int s = 0; s < DV; ++s) {
                const int rid = (int)(er[c][s] >> MSA_ER_SHIFT);
                mw[c][s] = __builtin_amdgcn_raw_buffer_load_b16(rmeta, lane * 2, rid * (TILE * 2), 0);
            }
        }
        uint32_t anynan = 0;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            cpk[c] = 0;
#pragma unroll
            for (int s = 0; s < DV; ++s) {
                const uint32_t m = mw[c][s];
                anynan |= m;
                const uint32_t q = (((m >> 15) ^ (sb[c] >> s)) & 1u) |
                                   ((m & (MSA_META_NONE | MSA_META_ID)) == (er[c][s] & MSA_META_ID) ? 2u : 0u);
                cpk[c] |= q << (4 * s);
            }
        }
        if (__builtin_expect(__ballot((anynan >> 13) & 3u) != 0ull, 0)) {
            // a row with NaN at x_0 / x_1: plane 3 (|x_1|) for the row's first edge, 2 (|x_0|) for the others
#pragma unroll
            for (int c = 0; c < CPW; ++c)
#pragma unroll
                for (int s = 0; s < DV; ++s) {
                    const bool first = er_pos(er[c][s], DC) == 0;
                    if ((mw[c][s] >> (first ? 14 : 13)) & 1u)
                        cpk[c] = (cpk[c] & ~(6u << (4 * s))) | ((first ? 3u : 2u) << (4 * s + 1));
                }
        }
#pragma unroll
        for (int c = 0; c < CPW; ++c)
#pragma unroll
            for (int s = 0; s < DV; ++s) {
                const int rid = (int)(er[c][s] >> MSA_ER_SHIFT);
                const int sp = (int)((cpk[c] >> (4 * s + 1)) & 3u);
                l[c][s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                         rrec, lane * 8 + sp * PB, rid * (MSA_REC_PLANES * PB), 0));
            }
    }
    // a refill's prior value: its table lookup goes out behind the record
    // loads (waiting only for its code), so the two latencies overlap
    if constexpr (PC) {
        if (fr) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) xin[c] = rf.ptab[kin[c] + kCodeBias];
        }
    }
    if (live) {
#pragma unroll
        for (int c = 0; c < CPW; ++c)
#pragma unroll
            for (int s = 0; s < DV; ++s) l[c][s] = flip_sign(l[c][s], cpk[c] >> (4 * s));
    }
    const bool fok = out_ok(fb, rf);  // index bounds, as k_var_m
    if (CONT && fl && fok) {  // finished codeword: hard bits of its exit (ballots before this step's update)
        uint64_t hw[CPW];
#pragma unroll
        for (int c = 0; c < CPW; ++c) hw[c] = hard[(size_t)t * N + j0 + c];
        store_fin_hard<CPW>(rf, hw, fb, N, j0, lane);
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int32_t j = j0 + c;
        const size_t pj = ((size_t)t * N + j) * TILE + lane;
        if (CONT && fl && fok && rf.post_out) {  // finished codeword: posterior L of its exit
            const size_t ob = (size_t)fb * N + j;
            rf.post_out[ob] = fn > 0 ? post[pj] : prior_at<PC>(prior, rf, pj);
        }
        bool h = false;
        double dv[DV];
#pragma unroll
        for (int s = 0; s < DV; ++s) dv[s] = 0.0;
        if (fr) {  // Init_MSA_INF for a refilled lane
            const double x = xin[c];
#pragma unroll
            for (int s = 0; s < DV; ++s) dv[s] = x;
            h = !(x > 0);
        } else if (live) {
            // v2c_s = LLR + c_0 + ... (skipping c_s), L = LLR + all, in the
            // reference's left-to-right order: v2c_s continues the shared
            // prefix P_s = LLR + c_0 + ... + c_{s-1} with c_{s+1} .. c_{DV-1}
            double P = pv[c];
#pragma unroll
            for (int s = 0; s < DV; ++s) {
                double sum = P;
#pragma unroll
                for (int q = s + 1; q < DV; ++q) sum = sum + l[c][q];
                dv[s] = sum;
                P = P + l[c][s];
            }
            h = !(P > 0);
            if (post) post[pj] = P;
        }
        if (CONT && fr) {
            if constexpr (PC) rf.pcode[pj] = kin[c];
            else prior[pj] = xin[c];
        }
        if (line_occupied(touched, lane) || fr || live) {  // whole-line stores, as k_var_m
            uint32_t sbn = 0;
#pragma unroll
            for (int s = 0; s < DV; ++s) {
                // v2c in column order: edge s of column j at j * vpa + s * vpb
                // (vpa = DV, vpb = 1: the wave's stores are one contiguous run;
                // vpa = 1, vpb = N: row-block-major, one run per row block)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, dv[s]), rv2c, lane * 8,
                                                      ((j0 + c) * vpa + s * vpb) * (TILE * 8), NT ? kBufNT : 0);
                sbn |= (dv[s] >= 0 ? 0u : 1u) << s;
            }
            sgn[pj] = (uint8_t)sbn;
        }
        const uint64_t m = __ballot(h);
        if (lane == 0 && touched) {
            const size_t o = (size_t)t * N + j;
            const uint64_t old = (touched == ~0ull) ? 0ull : hard[o];
            hard[o] = (old & ~touched) | (m & touched);
        }
    }
    // the reports of skipped accesses: the lane's pool slot (the indices need
    // not stay live; cont_lanes reports an out-of-range index itself)
    if (CONT && fl && !fok) lane_fault(rf.fault, kFaultOutput, t * TILE + lane);
    asm volatile("" : "+v"(bad_v));
    if (bad_v) lane_fault(rf.fault, kFaultRefill, t * TILE + lane);
}

// ---------------------------------------------------------------------------
// finalize: posterior per codeword/bit, written row-major [b][N].  The
// variable phase leaves the posterior of its iteration in post_t ([t][N][64]):
//   BP : P = LR * prod lr (ascending row, dec.cpp:669-674), NaN -> 1
//        (dec.cpp:676-677); iters == 0 -> P = LR (lr still 1 from init).
//        out = log(P) (LDPC_POST_LLR) or P (LDPC_POST_RATIO).
//   MSA: L = LLR + sum c2v (Decision_MSA_INF order); iters == 0 -> LLR.
// A codeword that stopped at iteration n > 0 was last updated by variable
// phase n-1, so post_t holds exactly its exit posterior.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ post_t, const double* __restrict__ prior,
                                                  const int32_t* __restrict__ iters, double* __restrict__ post,
                                                  int algo_msa, int post_ratio, int64_t Bc, int32_t N)
{
    const int lane = lane_id();
    const int32_t j = blockIdx.x * 4 + wave_id();
    const int64_t t = blockIdx.y;
    if (j >= N) return;
    const int64_t b = t * TILE + lane;
    if (b >= Bc) return;
    const size_t pj = ((size_t)t * N + j) * TILE + lane;
    double out;
    if (algo_msa) {
        out = iters[b] > 0 ? post_t[pj] : prior[pj];
    } else {
        double P = iters[b] > 0 ? post_t[pj] : prior[pj];
        if (__builtin_isnan(P)) P = 1.0;
        out = post_ratio ? P : log(P);
    }
    post[(size_t)b * N + j] = out;
}

// ---------------------------------------------------------------------------
// Continuous-batching syndrome step (one block per tile).  For every occupied
// lane (a codeword after lane_n iterations, or just initialised: lane_n = 0):
//   c == 0 or lane_n == max_iter  -> finished (Run_*_Decoder loop control,
//       dec.cpp:594-599 / 1223-1246): iters = lane_n, valid = (c == 0), hard
//       bits (and posterior) written to the codeword's output row; lane freed;
//   otherwise                    -> lane_n += 1, stays active.
// Free lanes claim the next codeword indices from a global counter (atomic)
// and are initialised by the following variable kernel (`fresh` mask).
// Which lane decodes which codeword varies run to run; each codeword's
// arithmetic does not.
// ---------------------------------------------------------------------------
// Start of a continuous decode: the lane masks, the claim counter, the
// occupancy ring and the split syndrome's words in one launch (instead of a
// memset launch each).
__global__ __launch_bounds__(256) void k_cont_reset(uint64_t* __restrict__ active, uint64_t* __restrict__ fresh,
                                                    uint64_t* __restrict__ occupied, unsigned long long* __restrict__ ctr,
                                                    int32_t nctr, unsigned long long* __restrict__ unsat,
                                                    unsigned* __restrict__ done, int64_t tiles)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tiles; i += (int64_t)gridDim.x * blockDim.x) {
        active[i] = 0;
        fresh[i] = 0;
        occupied[i] = 0;
        if (unsat) unsat[i] = 0;
        if (done) done[i] = 0;
    }
    if (blockIdx.x == 0 && (int32_t)threadIdx.x < nctr) ctr[threadIdx.x] = 0;
}

// Continuous-batching syndrome spread over gridDim.x blocks per tile (the
// k_syndrome_cont step with the resident pool's last-block bookkeeping,
// res_arrive): 16 tiles' syndromes in one block per tile left 240 of the 256
// CUs idle for ~64 us per step.  A wave takes 8 rows, lane (part, row) XORs
// the ballots of edges part*KP .. part*KP+KP-1 of its row (KP = ceil(DC/8)),
// the parts are XOR-combined across lanes, and the rows OR-combined; the
// tile's last block runs cont_lanes and hands the finished lanes to the
// variable kernel (Refill::fin), which writes their outputs.
// 1-D grid of nblk blocks per tile for `tiles` tiles: block L works on tile
// L % tiles, so with 8 | tiles each XCD gathers the ballots its own variable
// blocks just wrote (k_var_msa_c's tile-per-XCD mapping) from its L2.
template <int DC>
__global__ __launch_bounds__(256) void k_syndrome_split(int32_t M, ResStep rs, uint32_t tiles)
{
    constexpr int KP = (DC + 7) / 8;
    const int64_t t = blockIdx.x % tiles;
    const uint32_t blk = blockIdx.x / tiles, nblk = gridDim.x / tiles;
    const uint64_t occ = rs.cs.occupied[t];
    const int lane = lane_id();
    int32_t ln0 = 0;
    int64_t b0 = 0;
    uint64_t u = 0;
    if (occ) {
        if (threadIdx.x < TILE && ((occ >> lane) & 1ull)) {
            ln0 = rs.cs.lane_n[t * TILE + lane];
            b0 = rs.cs.lane_b[t * TILE + lane];
        }
        const uint64_t* __restrict__ h = rs.hard + (size_t)t * rs.N;
        const int part = lane >> 3;
        for (int32_t r0 = (int32_t)(blk * 4 + wave_id()) * 8; r0 < M; r0 += (int32_t)nblk * 32) {
            const int32_t row = r0 + (lane & 7);
            uint64_t p = 0;
            if (row < M) {
                const int32_t* __restrict__ cols = rs.col_idx + (size_t)row * DC;
#pragma unroll
                for (int q = 0; q < KP; ++q) {
                    const int k = part * KP + q;
                    if (k < DC) p ^= h[cols[k]];
                }
            }
            p ^= shfl_xor_u64(p, 8);
            p ^= shfl_xor_u64(p, 16);
            p ^= shfl_xor_u64(p, 32);
            u |= p;
        }
        u |= shfl_xor_u64(u, 1);
        u |= shfl_xor_u64(u, 2);
        u |= shfl_xor_u64(u, 4);
    }
    res_arrive(t, occ, u, rs, ln0, b0, nblk);
}

// k_syndrome_split for any row degrees (codes other than the regular
// degree-72 one, continuous mode): lane (part, row) XORs the ballots of edges
// part*KP .. part*KP+KP-1 of its row, KP = ceil(d / 8) of that row's degree d.
__global__ __launch_bounds__(256) void k_syndrome_split_gen(int32_t M, ResStep rs, uint32_t tiles)
{
    const int64_t t = blockIdx.x % tiles;
    const uint32_t blk = blockIdx.x / tiles, nblk = gridDim.x / tiles;
    const uint64_t occ = rs.cs.occupied[t];
    const int lane = lane_id();
    int32_t ln0 = 0;
    int64_t b0 = 0;
    uint64_t u = 0;
    if (occ) {
        if (threadIdx.x < TILE && ((occ >> lane) & 1ull)) {
            ln0 = rs.cs.lane_n[t * TILE + lane];
            b0 = rs.cs.lane_b[t * TILE + lane];
        }
        const uint64_t* __restrict__ h = rs.hard + (size_t)t * rs.N;
        const int part = lane >> 3;
        for (int32_t r0 = (int32_t)(blk * 4 + wave_id()) * 8; r0 < M; r0 += (int32_t)nblk * 32) {
            const int32_t row = r0 + (lane & 7);
            uint64_t p = 0;
            if (row < M) {
                const int32_t a = rs.row_ptr[row], b = rs.row_ptr[row + 1];
                const int32_t kp = (b - a + 7) / 8;
                const int32_t e0 = a + part * kp, e1 = e0 + kp < b ? e0 + kp : b;
                for (int32_t e = e0; e < e1; ++e) p ^= h[rs.col_idx[e]];
            }
            p ^= shfl_xor_u64(p, 8);
            p ^= shfl_xor_u64(p, 16);
            p ^= shfl_xor_u64(p, 32);
            u |= p;
        }
        u |= shfl_xor_u64(u, 1);
        u |= shfl_xor_u64(u, 2);
        u |= shfl_xor_u64(u, 4);
    }
    res_arrive(t, occ, u, rs, ln0, b0, nblk);
}

// hard ballots -> [b][N] u8 (the reference's dblk / dec_*.txt bits)
__global__ __launch_bounds__(256) void k_unpack_hard(const uint64_t* __restrict__ hard, uint8_t* __restrict__ out,
                                                     int64_t Bc, int32_t N)
{
    const int64_t nj = (N + 255) / 256;
    for (int64_t blk = blockIdx.x; blk < Bc * nj; blk += gridDim.x) {
        const int64_t b = blk / nj;
        const int32_t j = (int32_t)((blk - b * nj) * 256 + threadIdx.x);
        if (j < N) out[(size_t)b * N + j] = (uint8_t)((hard[(size_t)(b >> 6) * N + j] >> (b & 63)) & 1ull);
    }
}

// ---------------------------------------------------------------------------
// Host-API input path (capi.cpp): LR = table[code + 127], the table holding
// the host libm's exp(k * unit) -- the reference's LR = exp(LLR)
// (DNA_main.cpp:1344) for LLRs that are exact multiples k * unit, which the
// host checked value by value.  8 codes per thread (one 8-byte load).
// ---------------------------------------------------------------------------
// hard bits u8 [n][8] -> one byte per 8 (bit r = byte r), for the host API's
// D2H copy (capi.cpp unpacks them into the caller's one-byte-per-bit array)
__global__ __launch_bounds__(256) void k_pack_bits(const uint64_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = in[q];
        uint32_t b = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) b |= (uint32_t)((v >> (8 * r)) & 1ull) << r;
        out[q] = (uint8_t)b;
    }
}

__global__ __launch_bounds__(256) void k_lr_table(const int8_t* __restrict__ code, const double* __restrict__ table,
                                                  double* __restrict__ out, int64_t n)
{
    const int64_t n8 = n / 8;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n8; q += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t c = reinterpret_cast<const uint64_t*>(code)[q];
#pragma unroll
        for (int r = 0; r < 8; ++r) out[q * 8 + r] = table[(int)(int8_t)(c >> (8 * r)) + kCodeBias];
    }
    for (int64_t i = n8 * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = table[(int)code[i] + kCodeBias];
}

// ---------------------------------------------------------------------------
// synthetic BSC channel, counter-based:
//   u = splitmix64(((b << 24) | j) ^ splitmix64(seed)) >> 11, uniform in [0, 2^53)
//   flip = u * 2^-53 < p;  y = codeword[b mod n_cw][j] ^ flip
//   LLR = y ? -mag : +mag   (LR: y ? lr_neg : lr_pos, host-exp'd)
// ---------------------------------------------------------------------------
// T = int8_t: the channel as codes (+1 / -1, coded input)
template <typename T>
__global__ __launch_bounds__(256) void k_gen_bsc(T* __restrict__ out, int out_lr, int64_t b0, int64_t B,
                                                 const uint8_t* __restrict__ cws, int32_t n_cw, int32_t N,
                                                 uint64_t seedmix, double p, T pos, T negv)
{
    const int64_t total = B * (int64_t)N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t bl = i / N;
        const int32_t j = (int32_t)(i - bl * N);
        const uint64_t b = (uint64_t)(b0 + bl);
        const uint64_t u = splitmix64(((b << 24) | (uint64_t)j) ^ seedmix) >> 11;
        const bool flip = (double)u * 0x1.0p-53 < p;
        const uint8_t y = cws[(size_t)(b % (uint64_t)n_cw) * N + j] ^ (uint8_t)flip;
        (void)out_lr;
        out[i] = y ? negv : pos;
    }
}

}  // namespace dev
}  // namespace ldpc
