// engine.hpp -- internal interface between the C ABI and the HIP engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ldpc_amd.h"
#include "graph.hpp"
#include "kargs.hpp"

namespace ldpc {

// thread-local error string behind ldpc_last_error()
void set_error(const std::string& msg);
const char* last_error();

#define LDPC_HIP(call)                                                                           \
    do {                                                                                         \
        hipError_t _e = (call);                                                                  \
        if (_e != hipSuccess) {                                                                  \
            ::ldpc::set_error(std::string(#call) + ": " + hipGetErrorString(_e));                \
            return LDPC_ERR_DEVICE;                                                              \
        }                                                                                        \
    } while (0)

enum KClass { K_CHECK = 0, K_VAR = 1, K_SYN = 2, K_INIT = 3, K_FINAL = 4, K_OTHER = 5, K_NCLASS = 6 };

// A caller's ldpc_schedule with every field resolved: flags_set covers all
// bits, zero fields replaced by the defaults (include/ldpc_amd.h).  Two
// resolved schedules compare equal iff they select the same engine.  The
// input is always treated as a caller's (bits outside LDPC_SCHED_* dropped).
ldpc_schedule resolve_schedule(const ldpc_schedule* s);
inline bool sched_flag(const ldpc_schedule& s, int bit) { return (s.flags & bit) != 0; }

struct Engine {
    const HostGraph* g = nullptr;
    int device = 0;
    int algo = LDPC_ALGO_BP;
    hipStream_t stream = nullptr;
    ldpc_schedule sched{};    // resolved (resolve_schedule)
    int64_t cap = 0;          // codewords per pass / lane pool (multiple of 64)
    int64_t cap_tiles = 0;
    int64_t group_tiles = 0;  // tiles per check/variable launch; c2v holds only one group
    int64_t c2v_tiles = 0;    // tiles of c2v scratch allocated
    size_t c2v_bytes = 0;
    bool nt_d = false;        // nontemporal loads/stores of the v2c ("d") stream
    bool cont = false;        // continuous batching: refill lanes as codewords finish
    bool msa_c = false;       // min-sum with compressed c2v (records + meta words, k_check_msa_c / k_var_msa_c)
    bool res = false;         // resident pool: a few tiles iterated in place, syndrome in the check kernel
    bool first_fp = false;    // single-fill BP: the first check reads the prior (k_check_bp_first)
    bool debug_no_drain = false;  // LDPC_SCHED_DEBUG_NO_DRAIN: the host ignores a drained pool
    bool debug_bad_lane = false;  // LDPC_SCHED_DEBUG_BAD_LANE: one lane records an out-of-range codeword index
    int var_cpw = 4;          // variable phase: columns per wave (-2: by the prior's form, var_cpw_for)
    int res_poll = 8;         // res: steps between occupancy polls
    int syn_blocks = 0;       // continuous grouped mode: k_syndrome_split blocks per tile
    uint8_t* d_sgn = nullptr; // msa_c: [tile][N][64] sign bits of the v2c each column last stored
    unsigned long long* d_unsat = nullptr;  // [tile] syndrome words of the step
    unsigned int* d_done = nullptr;         // [tile] syndrome / check blocks arrived
    uint64_t* d_fin = nullptr;              // [tile] lanes finished at the step
    int64_t* d_fin_b = nullptr;             // [tile*64] their codeword index
    int32_t* d_fin_n = nullptr;             // [tile*64] their iteration count
    const dev::ResStep* rstep = nullptr;    // res: set around the check launch of a step
    static constexpr int kRing = 8, kLag = 2;
    uint64_t* d_fresh = nullptr;
    uint64_t* d_occ = nullptr;
    int64_t* d_lane_b = nullptr;
    int32_t* d_lane_n = nullptr;
    unsigned long long* d_ctr = nullptr;  // [0] claim counter, [1..kRing] occupancy ring
    // occupancy polls without copies or events: poll q's counter is
    // d_ctr[1 + q % kRing]; the device writes tag(q) << 40 | occupied lanes to
    // h_poll[q % kRing] (pinned, device-mapped at d_poll) and the host waits on it
    uint64_t poll_seq = 0;
    unsigned long long* h_poll = nullptr;
    unsigned long long* d_poll = nullptr;
    void poll_arm(dev::ContState& cs, uint64_t q) const;
    int poll_wait(uint64_t q, unsigned long long* occ);
    // device fault word (kargs.hpp kFaultTag): pinned, device-mapped at d_fault
    unsigned long long* h_fault = nullptr;
    unsigned long long* d_fault = nullptr;
    // LDPC_ERR_DEVICE (and the message) once a kernel has reported a fault;
    // the word is cleared, so each fault is reported once
    int check_fault();
    // wait for the engine's stream, then check_fault
    int sync();
    // graph on device
    int32_t* d_row_ptr = nullptr;
    int32_t* d_col_idx = nullptr;
    int32_t* d_col_idx_T = nullptr;  // [dc][M] for regular rows (syndrome gathers)
    int32_t* d_col_ptr = nullptr;
    int32_t* d_col_edge = nullptr;
    uint32_t* d_col_er = nullptr;  // [E] (row << 18) | edge id of CSC position q (MSA-C record lookups)
    int32_t* d_row_pos = nullptr;  // [E] v2c position of CSR edge e (MSA-C: v2c in column order)
    int32_t msa_pa = 8, msa_pb = 1;  // MSA-C: edge s of column j at j * msa_pa + s * msa_pb
    // decoder state
    double* v2c = nullptr;
    double* c2v = nullptr;
    double* prior = nullptr;
    uint64_t* hard = nullptr;
    uint64_t* active = nullptr;
    int32_t* iters = nullptr;
    uint8_t* valid = nullptr;
    double* post_t = nullptr;  // [tiles][N][64] per-iteration posterior (allocated on first use)
    // coded input (decode_codes): the lanes' int8 prior codes [tiles][N][64],
    // the prior table (256 fp64, code + 128), its last uploaded contents (an
    // unchanged table is not re-sent), the fp64 staging of schedules without
    // coded kernels, and the input codes of the decode in progress
    int8_t* pcode = nullptr;
    double* d_ptab = nullptr;
    double* h_ptab = nullptr;
    bool ptab_valid = false;
    double* d_expand = nullptr;  // fp64 staging of decode_codes' fixed passes (expand_rows codewords)
    int64_t expand_rows = 0;
    const int8_t* cur_codes = nullptr;
    // integer decoders (LDPC_ALGO_QMSA / GALLAGER_*): int32 views of v2c, c2v, prior
    int32_t q_precision = 6, q_beta = 0;
    double q_step = 0.5;
    uint64_t tie_seed = 0;
    int64_t tie_base = 0;  // added to the codeword index of the tie hash (host API: offset in the call)
    // profiling: HIP events on every `profile_stride`-th launch of a class
    int profile_stride = 0;
    int64_t sampled[K_NCLASS] = {0};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_live[K_NCLASS];
    std::vector<hipEvent_t> ev_pool;
    int64_t launches[K_NCLASS] = {0};
    hipEvent_t ext_stop = nullptr;  // stop event of the armed sampled launch
    double ms[K_NCLASS] = {0};

    ~Engine();
    // schedule: a caller's (resolved here), or with `resolved` one that
    // resolve_schedule already returned (the host API's slots)
    int init(const HostGraph* graph, int dev, int algorithm, int64_t chunk, const ldpc_schedule* schedule,
             bool resolved = false);
    // continuous batching; on an error the queued steps are drained and the
    // fault words cleared before returning (each fault is reported once)
    int run_cont(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                 int post_kind, int32_t* d_iters, uint8_t* d_valid);
    int run_cont_steps(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                       int post_kind, int32_t* d_iters, uint8_t* d_valid);
    // decode Bc <= cap codewords whose [Bc][N] input is at d_in (device)
    int run_chunk(const double* d_in, int in_kind, int64_t Bc, int32_t max_iter, uint8_t* d_hard, double* d_post,
                  int post_kind, int32_t* d_iters, uint8_t* d_valid);
    int decode(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
               int post_kind, int32_t* d_iters, uint8_t* d_valid);
    // coded input: d_codes [B][N] int8 on device, h_table[256] (host) the
    // channel value of code k at k + 128, of kind table_kind (LDPC_IN_LLR or,
    // BP only, LDPC_IN_LR); BP takes the host exp of an LLR table.  d_stage
    // (optional, >= min(cap, B) x N fp64): where schedules without coded
    // kernels expand a pass to fp64 (else an engine buffer)
    int decode_codes(const int8_t* d_codes, const double* h_table, int table_kind, int64_t B, int32_t max_iter,
                     uint8_t* d_hard, double* d_post, int post_kind, int32_t* d_iters, uint8_t* d_valid,
                     double* d_stage = nullptr);
    // integer decoders, Bc <= cap codewords; b_base = global index of the first (tie hash)
    int run_chunk_int(const double* d_in, int64_t Bc, int64_t b_base, int32_t max_iter, uint8_t* d_hard,
                      double* d_post, int32_t* d_iters, uint8_t* d_valid);
    int set_params(int32_t precision, double step, int32_t beta, uint64_t seed);
    int gen_bsc(double* d_out, int out_kind, int64_t b0, int64_t B, const uint8_t* d_cw, int32_t n_cw, uint64_t seed,
                double p, double llr_mag);
    // the same channel as int8 codes: +1 for a received 0, -1 for a 1
    int gen_bsc_codes(int8_t* d_out, int64_t b0, int64_t B, const uint8_t* d_cw, int32_t n_cw, uint64_t seed, double p);
    int collect_stats();
    // LDPC_SCHED_* bits in effect (ldpc_engine_info)
    int32_t flags() const;
    // out[i] = table[code[i] + 128] for i < n on stream s
    int expand_lr(const int8_t* d_code, const double* d_table, double* d_out, int64_t n, hipStream_t s);
    // out[i] bit r = in[8 i + r] for i < nbytes on the engine stream (host-API hard-bit copy)
    int pack_bits(const uint8_t* d_in, uint8_t* d_out, int64_t nbytes);

  private:
    hipEvent_t get_event();
    int mark_begin(KClass c, hipStream_t s, hipEvent_t* b);
    int mark_end(KClass c, hipStream_t s, hipEvent_t b);
    int probe(int probes);
    int launch_check(hipStream_t s, double* scratch, int64_t t0, unsigned gt);
    int launch_var(hipStream_t s, double* scratch, int64_t t0, unsigned gt, double* pt, const dev::Refill& rf);
    int var_cpw_for(const dev::Refill& rf) const;
};

// bytes of device memory per resident codeword
int64_t engine_bytes_per_codeword(const HostGraph& g);

}  // namespace ldpc
