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
    // bounds of the lane codeword indices (fin_b, lane_b): the decode's B;
    // a violation skips the access and is reported through `fault`
    int64_t nb = 0;
    unsigned long long* fault = nullptr;
};

// Device fault words (pinned host memory, device-mapped; ContState / Refill
// ::fault, one word per FaultKind): a kernel that finds a lane's codeword
// index outside [0, B) skips the store or load it would address and writes
// kFaultTag | kind << 48 | (index & kFaultIndex) to fault[kind]; the host
// turns the first nonzero word into LDPC_ERR_DEVICE.
constexpr unsigned long long kFaultTag = 1ull << 63;
constexpr unsigned long long kFaultIndex = (1ull << 48) - 1ull;
enum FaultKind : unsigned {
    kFaultIters = 1,   // iteration count / valid flag of a finished codeword (cont_lanes)
    kFaultOutput = 2,  // hard bits / posterior of a finished codeword (variable kernels; index: the lane's pool slot)
    kFaultRefill = 3,  // input row of a refilled lane (variable kernels: index = the lane's pool slot; k_fill_codes)
    kFaultSchedule = 4 // k_fill_codes on a tile with live or finished lanes (index: the tile)
};
constexpr int kFaultWords = 5;  // fault[0] unused

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
    unsigned long long* fault = nullptr;  // see kFaultTag
    // LDPC_SCHED_DEBUG_BAD_LANE (tests): the lane that claims codeword 0
    // records the index B + 4096 instead, so the guarded accesses fire
    int32_t debug_bad_lane = 0;
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
    const int32_t* row_ptr = nullptr;  // [M+1] CSR row starts (k_syndrome_split_gen: any row degrees)
};

}  // namespace dev
}  // namespace ldpc
