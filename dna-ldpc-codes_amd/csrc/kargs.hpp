// kargs.hpp -- plain argument structs shared by the kernels and the host engine.
#pragma once
#include <cstdint>

namespace ldpc {
namespace dev {

// Continuous batching (engine "cont" mode): a lane whose codeword finished is
// refilled with the next codeword by the syndrome kernel; the variable kernel
// then writes that lane's initial state (Init_Belief_Propagation dec.cpp:608-629
// / Init_MSA_INF dec.cpp:1300-1329) instead of an update.
struct Refill {
    const uint64_t* fresh;  // [tile] lanes to initialise this step (nullptr: fixed mode)
    const int64_t* lane_b;  // [tile*64] codeword index held by each lane
    const double* in;       // [B][N] input (LLR or LR)
    int in_is_llr;
    // resident pool (engine `res`, k_var_m only): outputs of the codewords
    // that finished at this step's syndrome, written before their lanes are
    // refilled (fin == nullptr: the syndrome kernel wrote them)
    const uint64_t* fin;    // [tile] finished lanes
    const int64_t* fin_b;   // [tile*64] their codeword index
    const int32_t* fin_n;   // [tile*64] their iteration count
    uint8_t* hard_out;      // [B][N]
    double* post_out;       // [B][N] or nullptr
    int post_ratio;
    int hard_vec;           // hard_out is 8-byte aligned and N % 8 == 0: packed per-lane stores
    // single fill (every lane refilled at once, none live): store only the
    // prior; the next check derives d0 = 1 - 2/(1+LR) from it (k_check_bp_first)
    int prior_only = 0;
};

struct ContState {
    uint64_t* active;      // [tile] lanes updated by check/variable this step
    uint64_t* fresh;       // [tile] lanes initialised by the variable kernel this step
    uint64_t* occupied;    // [tile] lanes holding a codeword
    int64_t* lane_b;       // [tile*64]
    int32_t* lane_n;       // [tile*64]
    unsigned long long* next_b;  // global claim counter
    unsigned long long* occ_count;  // occupied lanes after this step (host polls it)
    int64_t B;
    // the next poll's counter, zeroed by tile 0's bookkeeping of this step (its
    // previous D2H copy, kRing polls back, is stream-ordered before) instead
    // of a memset launch per poll
    unsigned long long* occ_clear = nullptr;
    // occ_count packs (tiles counted) << kOccTileShift | occupied lanes; the
    // last of ntiles tiles to count writes poll_tag << kOccTileShift |
    // occupied lanes to poll_host (pinned host memory, system scope), which
    // the host waits on instead of a D2H copy + event per poll
    unsigned long long* poll_host = nullptr;
    unsigned long long poll_tag = 0;
    int64_t ntiles = 0;
};
constexpr int kOccTileShift = 40;
constexpr unsigned long long kOccMask = (1ull << kOccTileShift) - 1ull;

struct ContOut {
    uint8_t* hard;    // [B][N]
    double* post;     // [B][N] or nullptr
    int32_t* iters;   // [B]
    uint8_t* valid;   // [B]
    const double* post_t;  // [tile][N][64] per-iteration posterior (when post)
    const double* prior;   // [tile][N][64]
    int algo_msa, post_ratio;
};

// Resident pool: the syndrome of the previous variable phase is computed by
// the check kernel (each wave its row's parity) and the last block of a tile
// to finish runs the lane bookkeeping (k_check_bp / k_check_msa with SYN).
struct ResStep {
    const uint64_t* hard;        // [tile][N] ballots
    const int32_t* col_idx;      // [E] CSR column of each edge (regular rows)
    unsigned long long* unsat;   // [tile] OR of the row parities (re-armed by the last block)
    unsigned int* done;          // [tile] blocks arrived (re-armed by the last block)
    uint64_t* fin;               // [tile] lanes finished at this step -> Refill::fin
    int64_t* fin_b;              // [tile*64]
    int32_t* fin_n;              // [tile*64]
    int32_t N, max_iter;
    ContState cs;
    ContOut co;                  // iters / valid (hard / post are written by k_var_m)
};

// XCD-resident BP decoder (kernels_xr.hpp)
constexpr uint32_t XR_DEAD = 0xFFFFFFFFu;
enum : unsigned long long { XR_LIVE = 1, XR_FIN = 2, XR_FRESH = 4 };
// packed slot state: codeword (40 bits, all ones = none) | iterations << 40 | mode << 56
constexpr unsigned long long XR_CW_MASK = (1ull << 40) - 1, XR_NO_CW = XR_CW_MASK;
__host__ __device__ constexpr unsigned long long xr_state(unsigned long long cw, unsigned long long n,
                                                          unsigned long long mode)
{
    return (cw & XR_CW_MASK) | ((n & 0xffffull) << 40) | (mode << 56);
}

// one slot's control words (128 B apart); only atomics touch them
struct XrCtl {
    unsigned long long ctl;    // (phase << 32) | tasks claimed
    unsigned long long done;   // tasks finished since the decode began (monotone)
    unsigned long long unsat;  // the last check phase that found an unsatisfied row (atomicMax)
    unsigned long long state;  // xr_state(codeword held, its iterations, variable-phase mode)
    unsigned long long fin;    // XR_FIN: xr_state(finished codeword, its iterations, 0)
    unsigned long long pad[11];
};

struct XrArgs {
    const uint8_t* jpb;       // [GA][RB][Q]
    const uint32_t* ord4;     // [GA][(RB+3)/4][Q]
    const uint64_t* inv8;     // [RB][Q]
    const int32_t* col_orig;  // [RB][Q]
    int32_t Q, N;
    int64_t E;
    double* msg;              // [S][E]
    double* prior;            // [S][N]
    double* post;             // [S][N] per-iteration posterior, or nullptr
    uint64_t* hb;             // [S][N/64]
    XrCtl* ctl;               // [S]
    int32_t K, nxcd;          // slots per XCD, XCDs
    const double* in;         // [B][N]
    int32_t in_is_llr;
    int32_t max_iter;
    int64_t B;
    unsigned long long* next_b;
    uint8_t* hard_out;        // [B][N]
    double* post_out;         // [B][N] or nullptr
    int32_t post_ratio;
    int32_t* iters_out;
    uint8_t* valid_out;
    unsigned long long* prof;  // [grid][8] or nullptr (LDPC_XR_PROF)
};

}  // namespace dev
}  // namespace ldpc
