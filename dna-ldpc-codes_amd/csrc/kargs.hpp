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
};

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

}  // namespace dev
}  // namespace ldpc
