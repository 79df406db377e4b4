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

}  // namespace dev
}  // namespace ldpc
