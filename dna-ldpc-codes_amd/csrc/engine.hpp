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

struct Engine {
    const HostGraph* g = nullptr;
    int device = 0;
    int algo = LDPC_ALGO_BP;
    hipStream_t stream = nullptr;
    int64_t cap = 0;        // codewords per pass (multiple of 64)
    int64_t cap_tiles = 0;
    int64_t group_tiles = 0;  // tiles per check/variable launch; c2v holds only one group
    int64_t c2v_tiles = 0;    // tiles of c2v scratch allocated
    bool nt_d = false;        // nontemporal loads/stores of the v2c ("d") stream
    bool pipe = false;        // check(g+1) on `stream` overlaps variable(g) on `stream2`
    bool lr_csc = false;      // c2v scratch in column (CSC) order (regular kernels only)
    bool cont = false;        // continuous batching: refill lanes as codewords finish
    int full_lanes = 0;       // all lanes of an active tile store (whole cache lines)
    bool debug_no_drain = false;  // LDPC_DEBUG_NO_DRAIN: the host ignores a drained pool (tests the step bound)
    bool pingpong = false;    // res, BP: one launch = check(tile t) + variable(tile t-1), k_pingpong_bp (LDPC_PINGPONG)
    int pp_cpw = 4;           // pingpong: variable-phase columns per wave (LDPC_PP_CPW)
    int var_cpw = 1;          // variable phase: columns per wave (k_var_m when > 1)
    bool msa_c = false;       // min-sum with compressed c2v (records + codes, k_check_msa_c / k_var_msa_c)
    bool msa_meta = false;    // msa_c: per-row meta byte + variable-owned sign bytes instead of per-edge codes (LDPC_MSA_META)
    uint8_t* d_sgn = nullptr; // msa_meta: [tile][N][64] sign bits of the v2c each column last stored
    bool res = false;         // resident pool: a few tiles iterated in place (c2v overwrites v2c), syndrome in the check kernel
    int res_poll = 4;         // res: steps between occupancy polls
    int res_syn_split = 0;    // res: 0 = syndrome fused into the check kernel, >0 = k_syndrome_split blocks per tile
    int syn_split = 0;        // continuous mode: syndrome blocks per tile (k_syndrome_split; 0: k_syndrome_cont)
    bool syn_fused = false;   // grouped continuous mode: syndrome + lane bookkeeping in the check kernel (ResStep)
    unsigned long long* d_unsat = nullptr;  // res: [tile] syndrome words of the step
    unsigned int* d_done = nullptr;         // res: [tile] check blocks arrived
    uint64_t* d_fin = nullptr;              // res: [tile] lanes finished at the step
    int64_t* d_fin_b = nullptr;             // res: [tile*64] their codeword index
    int32_t* d_fin_n = nullptr;             // res: [tile*64] their iteration count
    const dev::ResStep* rstep = nullptr;    // res: set around the check launch of a step
    static constexpr int kRing = 8, kLag = 2;
    // res with tile_streams: one stream per pool tile (LDPC_RES_STREAMS)
    static constexpr int kMaxTileStreams = 4;
    int tile_streams = 0;  // 0 off, 1 on, 2 staggered start, 3 re-staggered at every poll step
    hipStream_t tstream[kMaxTileStreams] = {};
    hipEvent_t ev_tjoin[kMaxTileStreams] = {};
    hipEvent_t ev_tring[kRing][kMaxTileStreams] = {};
    unsigned long long* d_occ_t = nullptr;  // [kRing][kMaxTileStreams] per-tile occupancy counters
    unsigned long long* h_occ_t = nullptr;
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
    int32_t* d_csc_pos = nullptr;  // [E] CSC position of CSR edge e
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_chk[2] = {nullptr, nullptr}, ev_var[2] = {nullptr, nullptr}, ev_join = nullptr;
    // graph on device
    int32_t* d_row_ptr = nullptr;
    int32_t* d_col_idx = nullptr;
    int32_t* d_col_idx_T = nullptr;  // [dc][M] for regular rows (syndrome gathers)
    int32_t* d_col_ptr = nullptr;
    int32_t* d_col_edge = nullptr;
    int32_t* d_col_row = nullptr;  // [E] row of edge col_edge[q] (MSA-C record lookups)
    // decoder state
    double* v2c = nullptr;
    double* c2v = nullptr;
    double* prior = nullptr;
    uint64_t* hard = nullptr;
    uint64_t* active = nullptr;
    int32_t* iters = nullptr;
    uint8_t* valid = nullptr;
    double* post_t = nullptr;  // [tiles][N][64] per-iteration posterior (allocated on first use)
    // integer decoders (LDPC_ALGO_QMSA / GALLAGER_*): int32 views of v2c, c2v, prior
    int32_t q_precision = 6, q_beta = 0;
    double q_step = 0.5;
    uint64_t tie_seed = 0;
    int64_t tie_base = 0;  // added to the codeword index of the tie hash (host API: offset in the call)
    // profiling: HIP events around every `profile_stride`-th launch of a class
    int profile_stride = 0;
    int64_t sampled[K_NCLASS] = {0};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_live[K_NCLASS];
    std::vector<hipEvent_t> ev_pool;
    int64_t launches[K_NCLASS] = {0};
    hipEvent_t ext_stop = nullptr;  // stop event of the armed sampled launch
    double ms[K_NCLASS] = {0};
    // whole continuous decodes with concurrent tile streams (HIP events on
    // `stream` around each run while profiling): their kernels overlap, so
    // the roofline of the concurrent set is bytes / this wall time
    std::vector<std::pair<hipEvent_t, hipEvent_t>> wall_live;
    double wall_ms = 0;
    int64_t wall_runs = 0;
    // XCD-resident BP decoder (kernels_xr.hpp, LDPC_XR): array codes only
    bool xr = false;
    int xr_k = 3;           // slots (codewords in flight) per XCD
    int xr_vb = 2;          // column blocks per variable task
    int xr_nxcd = 0;        // XCDs (probed from HW_REG_XCC_ID)
    int xr_grid = 0;        // persistent workgroups
    const XrLayout* xr_layout = nullptr;
    uint8_t* d_xr_jpb = nullptr;
    uint32_t* d_xr_ord4 = nullptr;
    uint64_t* d_xr_inv8 = nullptr;
    int32_t* d_xr_col = nullptr;
    double* xr_msg = nullptr;
    double* xr_prior = nullptr;
    double* xr_post = nullptr;
    uint64_t* xr_hb = nullptr;
    dev::XrCtl* xr_ctl = nullptr;
    unsigned long long* xr_next = nullptr;

    ~Engine();
    int init(const HostGraph* graph, int dev, int algorithm, int64_t chunk, int64_t group = -1, int nt = -1,
             int pipelined = -1, int csc = -1, int cont_mode = -1, int res_mode = -1);
    int run_cont(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                 int post_kind, int32_t* d_iters, uint8_t* d_valid);
    // decode Bc <= cap codewords whose [Bc][N] input is at d_in (device)
    int run_chunk(const double* d_in, int in_kind, int64_t Bc, int32_t max_iter, uint8_t* d_hard, double* d_post,
                  int post_kind, int32_t* d_iters, uint8_t* d_valid);
    int decode(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
               int post_kind, int32_t* d_iters, uint8_t* d_valid);
    // integer decoders, Bc <= cap codewords; b_base = global index of the first (tie hash)
    int run_chunk_int(const double* d_in, int64_t Bc, int64_t b_base, int32_t max_iter, uint8_t* d_hard,
                      double* d_post, int32_t* d_iters, uint8_t* d_valid);
    int set_params(int32_t precision, double step, int32_t beta, uint64_t seed);
    int gen_bsc(double* d_out, int out_kind, int64_t b0, int64_t B, const uint8_t* d_cw, int32_t n_cw, uint64_t seed,
                double p, double llr_mag);
    int collect_stats();
    // out[i] = table[code[i] + 127] for i < n on stream s (host-API input path)
    int expand_lr(const int8_t* d_code, const double* d_table, double* d_out, int64_t n, hipStream_t s);
    // out[i] bit r = in[8 i + r] for i < nbytes on the engine stream (host-API hard-bit copy)
    int pack_bits(const uint8_t* d_in, uint8_t* d_out, int64_t nbytes);

  private:
    hipEvent_t get_event();
    int mark_begin(KClass c, hipStream_t s, hipEvent_t* b);
    int mark_end(KClass c, hipStream_t s, hipEvent_t b);
    int probe_c2v(int probes);
    int probe_res(int probes);
    int launch_check(hipStream_t s, double* scratch, int64_t t0, unsigned gt);
    int launch_var(hipStream_t s, double* scratch, int64_t t0, unsigned gt, double* pt, const dev::Refill& rf);
    int launch_pingpong(hipStream_t s, int64_t tc, int64_t tv, double* pt, const dev::ResStep& rs,
                        const dev::Refill& rf);
    int init_xr();
    int run_xr(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
               int post_kind, int32_t* d_iters, uint8_t* d_valid);
};

// bytes of device memory per resident codeword
int64_t engine_bytes_per_codeword(const HostGraph& g);

}  // namespace ldpc
