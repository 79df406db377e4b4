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
    // continuous mode: outputs of the codewords that finished at this step's
    // syndrome, written by the variable kernel before their lanes are refilled
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
    // coded input (ldpc_engine_decode_codes): the input is int8 channel codes
    // [B][N] (in_code, `in` unused) and every lane keeps its prior as the code
    // ([tile][N][64] pcode) instead of fp64; the prior value of code k is
    // ptab[k + 128] (LR for BP, LLR for min-sum)
    const int8_t* in_code = nullptr;
    int8_t* pcode = nullptr;
    const double* ptab = nullptr;
    // first check from codes (compressed min-sum, coded input): a refilled
    // lane's first check ran in this step's check kernel straight from its
    // input codes (FirstCheck), so the variable kernel runs its first
    // iteration's update instead of Init_MSA_INF's stores
    int ff = 0;
};

// First check from codes (compressed min-sum with coded input, every refill):
// the check kernel of the step that claims a codeword computes its first
// check phase from the input codes -- Init_MSA_INF (dec.cpp:1300-1329) sets
// every v2c of column j to LLR_j, so row r's messages are the LLRs of its
// columns -- instead of spending a step on storing E copies of them.  The
// iteration-0 syndrome (the parity of !(LLR > 0) over each row, dec.cpp:1223
// on Init's decisions) is taken in the same pass: u0_rows[t][row] gets the
// ballot of the refilled lanes whose row parity is 1, and the next step's
// syndrome ORs it into the tile's iteration-0 word.
struct FirstCheck {
    const uint64_t* fresh = nullptr;  // [tile] lanes claimed at this step's syndrome
    const int64_t* lane_b = nullptr;  // [tile*64] their codeword index
    const int8_t* in_code = nullptr;  // [B][N] input codes
    const double* ptab = nullptr;     // [256] LLR of code k at k + 128
    const int32_t* col_idx = nullptr; // [E] CSR column of each edge
    uint64_t* u0_rows = nullptr;      // [tile][M] iteration-0 row parities of the refilled lanes
    int32_t N = 0;
};

// prior value of a code (coded input): table indexed by code + 128
constexpr int kCodeBias = 128;

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
    int32_t* iters;   // [B] the decode's iteration-count output
    uint8_t* valid;   // [B] its valid-flag output
};

// Continuous-mode syndrome step: the parity of every row over the previous
// variable phase's ballots, computed by the resident pool's check kernel
// (each wave its row, k_check_bp / k_check_msa with RES) or by
// k_syndrome_split (grouped schedule); the last block of a tile to finish runs
// the lane bookkeeping.
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
    ContOut co;                  // iters / valid (hard / post are written by the variable kernel)
    // first check from codes (FirstCheck): the lanes refilled at the previous
    // step are evaluated for iterations 0 and 1 at once -- iteration 0's
    // syndrome from u0_rows (OR-reduced into unsat0, re-armed by the last
    // block), iteration 1's from the ballots
    const uint64_t* u0_rows = nullptr;  // [tile][M]
    unsigned long long* unsat0 = nullptr;  // [tile]
};

}  // namespace dev
}  // namespace ldpc
