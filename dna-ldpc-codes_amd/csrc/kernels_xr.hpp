// kernels_xr.hpp -- XCD-resident BP decoder for array (RS / quasi-cyclic)
// codes on MI355X: one codeword per lane group is replaced by one codeword per
// SLOT, a slot's whole message state (E fp64 = 1.18 MB for the DNA code) kept
// in the 4 MB L2 of one XCD, and every access to it made from that XCD.
//
// Why: the tiled kernels (kernels.hpp) move 32 B per edge per iteration
// between launches, through the Infinity Cache / HBM (~6.4-7 TB/s for that
// access shape, tools/cachebench).  Kernel boundaries write back and
// invalidate the L2, so no launch schedule can keep messages in it.  One
// persistent launch can: a block that rewrites the same lines in one launch
// is served by its XCD's L2 at 14-16 TB/s (cachebench, <= 48 MB).
//
// Layout (per slot s, H = GA x RB blocks of Q x Q permutations, graph.hpp
// XrLayout):
//   msg [s][a][b][i]  fp64  edge of row (a, i) in column block b: d (the
//                    variable->check term 1 - 2/(1+pr)) between phases, lr
//                    after the check phase -- in place, like the resident pool
//   prior [s][b][jp] fp64  LR of column (b, jp)
//   hb [s][b][jp/64] u64   hard decisions (ballots)
// Check task (row block a, 4 waves, lane = row): the row's 72 edges are loaded
// by column block (coalesced), put into the row's own column order through
// LDS, run through the reference's sequential prefix / suffix products
// (dec.cpp:646-662, the arithmetic of check_bp_row), and stored back.  The
// same task takes the row parities of the previous decisions (check.cpp:28-45)
// from the slot's hard-bit bitmap in LDS.
// Variable task (column block b, 4 waves, lane = column): the column's 8
// edges, one per row block, ascending row = ascending a (dec.cpp:667-693, the
// arithmetic of var_m_block).
//
// Scheduling: per slot a phase word (phase << 32 | tasks claimed).  Even
// phases are check phases (GA tasks), odd phases variable phases (RB tasks).
// A workgroup claims a task of one of its own XCD's slots with one
// atomicAdd; the last task of a phase to finish runs the slot's bookkeeping
// (Run_Belief_Propagation_Decoder's loop control dec.cpp:594-599: stop when
// the syndrome is zero or n == max_iter, claim the next codeword) and opens
// the next phase.  Only memory-side atomics carry control between
// workgroups; message data moves through the XCD's L2: a task waits for its
// stores (vmcnt) before its done-count, and a task drops its CU's L1 before
// reading.  A claimed task never waits, so there is no deadlock whatever
// number of workgroups is resident.
#pragma once
#include "kernels.hpp"

namespace ldpc {
namespace dev {

__device__ __forceinline__ unsigned long long xr_get(unsigned long long* p) { return atomicAdd(p, 0ull); }
// wait for the thread's outstanding memory operations
__device__ __forceinline__ void xr_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// returning atomics whose result is consumed: performed at memory before the
// thread goes on (a no-return atomic's completion is not ordered by vmcnt alone)
__device__ __forceinline__ void xr_set(unsigned long long* p, unsigned long long v)
{
    const unsigned long long o = atomicExch(p, v);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");
}
__device__ __forceinline__ void xr_max(unsigned long long* p, unsigned long long v)
{
    const unsigned long long o = atomicMax(p, v);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");
}

// Loads of the slot state other CUs of the XCD rewrite (messages, prior,
// ballots, posterior) must not hit this CU's L1: "buffer_inv sc0" leaves the
// L1 as it is and "buffer_inv sc1" also drops the L2 (tools/l1probe).  LDM 1:
// nontemporal loads, LDM 2: agent-scope loads (sc1); both miss the L1.
template <int LDM, typename T>
__device__ __forceinline__ T xld(const T* p)
{
    if constexpr (LDM == 1) {
        return __builtin_nontemporal_load(p);
    } else if constexpr (LDM == 2) {
        if constexpr (sizeof(T) == 8) {
            const unsigned long long u =
                __hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            T v;
            __builtin_memcpy(&v, &u, 8);
            return v;
        } else {
            return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        return *p;
    }
}

__device__ __forceinline__ unsigned xr_xcc()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xfu;
}

// dec.cpp:646-662 on one row per lane, in registers: y[k] holds d_k of the
// row's k-th edge (row order) and receives lr_k.  Same operations in the same
// order as check_bp_row (prefix checkpoints every SEG edges, segments
// recomputed in the backward pass); y[k] is overwritten only once its d_k has
// had its last use.
template <int DC>
__device__ __forceinline__ void xr_check_row(double (&y)[DC])
{
    constexpr int SEG = 8;
    constexpr int NSEG = (DC + SEG - 1) / SEG;
    double cp[NSEG];
    double p = 1.0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k % SEG == 0) cp[k / SEG] = p;
        p = p * y[k];
    }
    double s = 1.0;
#pragma unroll
    for (int g = NSEG - 1; g >= 0; --g) {
        double pk[SEG];
        double q = cp[g];
        asm volatile("" : "+v"(q));
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const int k = g * SEG + i;
            if (k < DC) { pk[i] = q; q = q * y[k]; }
        }
#pragma unroll
        for (int i = SEG - 1; i >= 0; --i) {
            const int k = g * SEG + i;
            if (k < DC) {
                const double tt = pk[i] * s;
                const double lr = (1.0 + tt) / (1.0 - tt);
                s = s * y[k];
                y[k] = lr;
            }
        }
    }
}

// Check task: row block a of slot s (lane = row).  The row's edges are stored
// by column block b and processed in the row's own order k (ord4): each wave
// puts them into row order through its own [DC][64] fp64 LDS buffer (36 KB
// for the DNA code; with four waves one workgroup per CU).  Measured
// alternatives: two buffers per workgroup shared by waves in turn (two
// workgroups per CU) and a two-pass half-size permutation both ran slower.
// s_any[w]: some row of wave w is unsatisfied by the slot's current decisions.
template <int DC, int LDM>
__device__ __forceinline__ void xr_check_task(const XrArgs& x, int s, int a, double* s_perm, uint64_t* s_hb,
                                              int* s_any, unsigned long long* pc)
{
    constexpr int NR = (DC + 3) / 4, CH = 36;
    const unsigned long long t0 = threadIdx.x == 0 ? clock64() : 0;
    const int lane = lane_id(), w = wave_id();
    const int32_t Q = x.Q, QW = Q / TILE;
    const uint64_t* hb = x.hb + (size_t)s * (x.N / TILE);
    for (int t = threadIdx.x; t < DC * QW; t += blockDim.x) s_hb[t] = xld<LDM>(hb + t);
    __syncthreads();
    const bool on = w < QW;
    bool par = false;
    double* L = s_perm + (size_t)w * DC * TILE + lane;
    double* row = x.msg + (size_t)s * x.E + (size_t)a * DC * Q + (size_t)w * TILE + lane;
    const uint8_t* jpa = x.jpb + (size_t)a * DC * Q + (size_t)w * TILE + lane;
    const uint32_t* oa = x.ord4 + (size_t)a * NR * Q + (size_t)w * TILE + lane;
    double y[DC];
    // the edges go to LDS in block order and come back in row order (ord4)
    auto gather = [&]() {
#pragma unroll
        for (int c0 = 0; c0 < DC; c0 += CH) {
            double v[CH];
            uint32_t jp[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c)
                if (c0 + c < DC) {
                    v[c] = xld<LDM>(row + (size_t)(c0 + c) * Q);
                    jp[c] = jpa[(size_t)(c0 + c) * Q];
                }
#pragma unroll
            for (int c = 0; c < CH; ++c)
                if (c0 + c < DC) {
                    const int b = c0 + c;
                    L[b * TILE] = v[c];
                    par ^= ((s_hb[b * QW + (jp[c] >> 6)] >> (jp[c] & 63)) & 1ull) != 0;
                }
        }
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            const uint32_t o = oa[(size_t)q * Q];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (4 * q + r < DC) y[4 * q + r] = L[((o >> (8 * r)) & 0xffu) * TILE];
        }
    };
    auto scatter = [&]() {
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            const uint32_t o = oa[(size_t)q * Q];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (4 * q + r < DC) L[((o >> (8 * r)) & 0xffu) * TILE] = y[4 * q + r];
        }
#pragma unroll
        for (int c0 = 0; c0 < DC; c0 += CH) {
            double v[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c)
                if (c0 + c < DC) v[c] = L[(c0 + c) * TILE];
#pragma unroll
            for (int c = 0; c < CH; ++c)
                if (c0 + c < DC) row[(size_t)(c0 + c) * Q] = v[c];
        }
    };
    if (on) gather();
    unsigned long long t1 = 0;
    if (threadIdx.x == 0) {
        t1 = clock64();
        pc[8] += t1 - t0;
    }
    if (on) xr_check_row<DC>(y);
    const uint64_t anyw = __ballot(par);
    if (lane == 0) s_any[w] = anyw != 0;
    if (threadIdx.x == 0) pc[9] += clock64() - t1;
    if (on) scatter();
}

// Variable task: column blocks b0 .. b0+VB-1 of slot s (lane = column jp of
// each), mode / codewords from the bookkeeping of the check phase before it.
// A column's edge in row block a is entry (row inv8 byte a) of the segment
// [a][b][0..Q): the gathers of a wave stay inside 2 KB segments.  (Staging the
// segments through LDS with coalesced loads measured slower.)
template <int DC, int DV, int VB, int LDM>
__device__ __forceinline__ void xr_var_task(const XrArgs& x, int s, int b0, unsigned long long st,
                                            unsigned long long fin)
{
    const int lane = lane_id(), w = wave_id();
    const int32_t Q = x.Q, QW = Q / TILE, N = x.N;
    if (w >= QW) return;
    const unsigned long long mode = st >> 56;
    const int64_t cw = (int64_t)(st & XR_CW_MASK);
    const int64_t fin_cw = (int64_t)(fin & XR_CW_MASK), fin_n = (int64_t)((fin >> 40) & 0xffff);
    const int32_t jp = w * TILE + lane;
    double* msg = x.msg + (size_t)s * x.E;
    double* prior = x.prior + (size_t)s * N;
    double* post = x.post ? x.post + (size_t)s * N : nullptr;
    uint64_t* hbs = x.hb + (size_t)s * (N / TILE);
    size_t off[VB][DV];
#pragma unroll
    for (int v = 0; v < VB; ++v) {
        const uint64_t inv = x.inv8[(size_t)(b0 + v) * Q + jp];
#pragma unroll
        for (int a = 0; a < DV; ++a) off[v][a] = ((size_t)a * DC + b0 + v) * Q + ((inv >> (8 * a)) & 0xffull);
    }
    if (mode & XR_FIN) {  // the finished codeword's exit: hard bits and posterior
#pragma unroll
        for (int v = 0; v < VB; ++v) {
            const size_t pj = (size_t)(b0 + v) * Q + jp;
            const size_t ob = (size_t)fin_cw * N + x.col_orig[pj];
            x.hard_out[ob] = (uint8_t)((xld<LDM>(hbs + (size_t)(b0 + v) * QW + w) >> lane) & 1ull);
            if (x.post_out) {
                const double pv = fin_n > 0 ? xld<LDM>(post + pj) : xld<LDM>(prior + pj);
                const double P = __builtin_isnan(pv) ? 1.0 : pv;
                x.post_out[ob] = x.post_ratio ? P : log(P);
            }
        }
    }
    if (!(mode & (XR_LIVE | XR_FRESH))) return;
    double dv[VB][DV];
    bool h[VB];
    if (mode & XR_LIVE) {  // dec.cpp:667-693
        double l[VB][DV], p0[VB];
#pragma unroll
        for (int v = 0; v < VB; ++v) {
#pragma unroll
            for (int a = 0; a < DV; ++a) l[v][a] = xld<LDM>(msg + off[v][a]);
            p0[v] = xld<LDM>(prior + (size_t)(b0 + v) * Q + jp);
        }
#pragma unroll
        for (int v = 0; v < VB; ++v) {
            double pr[DV];
            double p = p0[v];
#pragma unroll
            for (int a = 0; a < DV; ++a) { pr[a] = p; p = p * l[v][a]; }
            if (__builtin_isnan(p)) p = 1.0;
            h[v] = (p <= 1.0);
            if (post) post[(size_t)(b0 + v) * Q + jp] = p;
            double acc = 1.0;
#pragma unroll
            for (int a = DV - 1; a >= 0; --a) {
                double t = pr[a] * acc;
                if (__builtin_isnan(t)) t = 1.0;
                acc = acc * l[v][a];
                dv[v][a] = 1.0 - 2.0 / (1.0 + t);
            }
        }
    } else {  // Init_Belief_Propagation dec.cpp:608-629 for the slot's new codeword
        double xi[VB];
#pragma unroll
        for (int v = 0; v < VB; ++v) xi[v] = x.in[(size_t)cw * N + x.col_orig[(size_t)(b0 + v) * Q + jp]];
#pragma unroll
        for (int v = 0; v < VB; ++v) {
            const double LR = x.in_is_llr ? exp(xi[v]) : xi[v];
            prior[(size_t)(b0 + v) * Q + jp] = LR;
            const double d0 = 1.0 - 2.0 / (1.0 + LR);
#pragma unroll
            for (int a = 0; a < DV; ++a) dv[v][a] = d0;
            h[v] = (LR < 1.0);
        }
    }
#pragma unroll
    for (int v = 0; v < VB; ++v) {
#pragma unroll
        for (int a = 0; a < DV; ++a) msg[off[v][a]] = dv[v][a];
        const uint64_t m = __ballot(h[v]);
        if (lane == 0) hbs[(size_t)(b0 + v) * QW + w] = m;
    }
}

// tasks before phase P (check phases: GA tasks, variable phases: NV tasks)
__device__ __forceinline__ unsigned long long xr_cumul(uint32_t P, unsigned GA, unsigned NV)
{
    return (unsigned long long)(P / 2) * (GA + NV) + (P & 1) * GA;
}

// End of check phase P (the slot's last task, one thread): the syndrome of
// the decisions it checked is known.  Run_Belief_Propagation_Decoder's loop
// control (dec.cpp:594-599): stop at c == 0 or n == max_iter, else iterate;
// a stopped (or empty) slot claims the next codeword.
__device__ __forceinline__ void xr_bookkeep_check(const XrArgs& x, XrCtl* c, uint32_t P)
{
    const unsigned long long u = xr_get(&c->unsat), st = xr_get(&c->state);
    const bool unsat = u == P;
    const unsigned long long cw = st & XR_CW_MASK, n = (st >> 40) & 0xffff;
    unsigned long long mode = 0, ncw = XR_NO_CW, nn = 0;
    bool claim = cw == XR_NO_CW;
    if (!claim) {
        if (!unsat || (int64_t)n == (int64_t)x.max_iter) {
            x.iters_out[cw] = (int32_t)n;
            x.valid_out[cw] = unsat ? 0 : 1;
            xr_set(&c->fin, xr_state(cw, n, 0));
            mode |= XR_FIN;
            claim = true;
        } else {
            mode |= XR_LIVE;
            ncw = cw;
            nn = n + 1;
        }
    }
    if (claim) {
        const unsigned long long nb = atomicAdd(x.next_b, 1ull);
        if (nb < (unsigned long long)x.B) {
            ncw = nb;
            mode |= XR_FRESH;
        }
    }
    xr_set(&c->state, xr_state(ncw, nn, mode));  // fin and state are performed before the phase opens
    atomicExch(&c->ctl, mode ? (unsigned long long)(P + 1) << 32 : (unsigned long long)XR_DEAD << 32);
}

template <int DC, int DV, int VB, int LDM>
__global__ __launch_bounds__(256, 1) void k_xr_bp(XrArgs x)
{
    constexpr unsigned NV = DC / VB;  // variable tasks per phase
    constexpr int LDS_D = 4 * DC * TILE;  // check tasks: one [DC][64] buffer per wave
    __shared__ double s_lds[LDS_D];
    __shared__ uint64_t s_hb[DC * 4];
    __shared__ unsigned long long s_task[5];
    __shared__ int s_any[4];
    const int K = x.K;
    const int s0 = (int)(xr_xcc() % (unsigned)x.nxcd) * K;
    int rot = (int)(blockIdx.x / (unsigned)x.nxcd);
    // LDPC_XR_PROF: thread 0's cycles in claiming / check tasks / variable
    // tasks / done-count + bookkeeping, and the counts (in LDS: no registers
    // held across the loop)
    __shared__ unsigned long long pc[16];
    if (threadIdx.x < 16) pc[threadIdx.x] = 0;
    unsigned long long tA = threadIdx.x == 0 ? clock64() : 0;
    for (;;) {
        if (threadIdx.x == 0) {
            unsigned long long got = ~0ull, P = 0, c = 0;
            for (;;) {
                int dead = 0;
                for (int q = 0; q < K && got == ~0ull; q++) {
                    const int s = s0 + (rot + q) % K;
                    const unsigned long long o = atomicAdd(&x.ctl[s].ctl, 1ull);
                    const uint32_t ph = (uint32_t)(o >> 32), cnt = (uint32_t)o;
                    if (ph == XR_DEAD) { dead++; continue; }
                    if (cnt < ((ph & 1) ? NV : (uint32_t)DV)) { got = (unsigned long long)s; P = ph; c = cnt; }
                }
                if (got != ~0ull || dead == K) break;
                __builtin_amdgcn_s_sleep(4);
            }
            rot++;
            s_task[0] = got;
            s_task[1] = P;
            s_task[2] = c;
            if (got != ~0ull && (P & 1)) {  // variable phase: what the bookkeeping decided
                s_task[3] = xr_get(&x.ctl[got].state);
                s_task[4] = xr_get(&x.ctl[got].fin);
            }
        }
        __syncthreads();
        const unsigned long long got = s_task[0];
        unsigned long long tB = 0;
        if (threadIdx.x == 0) {
            tB = clock64();
            pc[0] += tB - tA;
        }
        if (got == ~0ull) {
            if (x.prof && threadIdx.x == 0)
                for (int q = 0; q < 16; q++) x.prof[(size_t)blockIdx.x * 16 + q] = pc[q];
            return;
        }
        const int s = (int)got;
        const uint32_t P = (uint32_t)s_task[1], task = (uint32_t)s_task[2];
        const unsigned long long st = s_task[3];
        // LDM 0 (experiment): drop the CU's L1 instead, "buffer_inv sc1"
        if (LDM == 0) asm volatile("buffer_inv sc1" ::: "memory");
        if ((P & 1) == 0) {
            if (P != 0) xr_check_task<DC, LDM>(x, s, (int)task, s_lds, s_hb, s_any, pc);
        } else {
            xr_var_task<DC, DV, VB, LDM>(x, s, (int)task * VB, st, s_task[4]);
        }
        xr_wait();
        __syncthreads();
        unsigned long long tC = 0;
        if (threadIdx.x == 0) {
            tC = clock64();
            pc[(P & 1) ? 3 : 1] += tC - tB;
            pc[(P & 1) ? 4 : 2]++;
            XrCtl* cc = &x.ctl[s];
            if ((P & 1) == 0 && P != 0 && (s_any[0] | s_any[1] | s_any[2] | s_any[3])) {
                xr_max(&cc->unsat, (unsigned long long)P);
            }
            const unsigned long long prev = atomicAdd(&cc->done, 1ull);
            if (prev == xr_cumul(P + 1, DV, NV) - 1) {
                pc[6]++;
                if ((P & 1) == 0)
                    xr_bookkeep_check(x, cc, P);
                else  // variable phase: the slot goes on unless it emptied
                    atomicExch(&cc->ctl, (st & XR_CW_MASK) == XR_NO_CW ? (unsigned long long)XR_DEAD << 32
                                                                      : (unsigned long long)(P + 1) << 32);
            }
        }
        if (threadIdx.x == 0) {
            tA = clock64();
            pc[5] += tA - tC;
        }
        __syncthreads();
    }
}

// XCD id of every block (engine init: how many XCDs, and that the register reads)
__global__ void k_xr_probe(unsigned* out)
{
    if (threadIdx.x == 0) out[blockIdx.x] = xr_xcc();
}

// control words before a decode: every slot at phase 0 (an empty check
// phase whose bookkeeping claims the slot's first codeword)
__global__ void k_xr_reset(XrCtl* ctl, int S, unsigned long long* next_b)
{
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
        XrCtl& c = ctl[s];
        c.ctl = 0;
        c.done = 0;
        c.unsat = 0;  // phase 0 checks no codeword
        c.state = xr_state(XR_NO_CW, 0, 0);
        c.fin = 0;
    }
    if (threadIdx.x == 0) *next_b = 0;
}

}  // namespace dev
}  // namespace ldpc
