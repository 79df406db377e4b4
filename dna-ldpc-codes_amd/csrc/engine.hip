// engine.hip -- device engine: memory, launch sequence, profiling.
//
// One Engine = one device, one HIP stream, message buffers for `cap`
// resident codewords.  A decode is the reference's per-frame loop
// (Run_Belief_Propagation_Decoder dec.cpp:583-605 / Run_MSA_Decoder_INF
// dec.cpp:1216-1250) executed for many codewords at once:
//
//   init                                  (Init_*: dec.cpp:608 / 1300)
//   for n = 0..max_iter:
//       syndrome(n)  -> codewords with c == 0 or n == max_iter stop
//       if n == max_iter: break
//       check phase  (dec.cpp:646-662 / 1398-1433)
//       variable phase + hard decision (dec.cpp:667-693 / 1597-1678)
//   finalize (posterior, hard bits, iteration counts)
//
// Three schedules (include/ldpc_amd.h ldpc_schedule), all
// bit-exact; they differ only in which codewords share a launch:
//   * fixed passes (run_chunk): passes of <= cap codewords, stopped codewords
//     masked out of every later kernel (the integer decoders, irregular
//     graphs, or LDPC_SCHED_CONTINUOUS off);
//   * continuous grouped (run_cont): a lane pool refilled as codewords
//     finish, check/variable launches per tile group so the group's c2v
//     stays in the Infinity Cache, a multi-block syndrome per step;
//   * resident pool (run_cont, `res`): a few tiles iterated in place, sized to
//     the 256 MB Infinity Cache, the syndrome fused into the check kernel.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "engine.hpp"
#include "kernels.hpp"
#include "kernels_int.hpp"

namespace ldpc {

// Defaults, each chosen by a same-process A/B on MI355X (profiles/r*/README.md).
constexpr int32_t kDefaultGroupTiles = 3;     // grouped schedule (tools/sweep.py)
constexpr int32_t kDefaultMsaGroupTiles = 8;  // compressed min-sum, 1024-lane pool: one tile per XCD (+2.7 %)
constexpr int32_t kDefaultVarCpw = 4;         // fp64 priors: +2.6-2.9 % over 1 column per wave
constexpr int32_t kDefaultVarCpwCoded = 2;    // coded priors, resident pool / compressed min-sum: +0.5 % / +1.9 %
                                              // over 4 (the grouped BP schedule stays at 4: 2 is 10 % slower)
constexpr int32_t kDefaultPoolTiles = 3;      // resident pool: 3 x 85 MB ~ the 256 MB Infinity Cache
constexpr int32_t kDefaultResPoll = 8;
constexpr int32_t kDefaultSynBlocks = 32;     // continuous-mode syndrome blocks per tile (config 5 +5-6 %)
constexpr int64_t kMsaPool = 1024;            // compressed min-sum lanes (scattered v2c stores: small pool)
constexpr int64_t kResAutoMaxTiles = 4;       // explicit pools above this: grouped unless RESIDENT is set
constexpr int kProbes = 4;                    // placement probe: candidate scratch allocations timed at init

constexpr int32_t kDefaultFlags = LDPC_SCHED_NONTEMPORAL | LDPC_SCHED_CONTINUOUS | LDPC_SCHED_MSA_COMPRESSED |
                                  LDPC_SCHED_RESIDENT | LDPC_SCHED_FIRST_FROM_PRIOR | LDPC_SCHED_LR_TABLE;
constexpr int32_t kAllFlags = kDefaultFlags | LDPC_SCHED_DEBUG_NO_DRAIN | LDPC_SCHED_DEBUG_BAD_LANE;

// flags_set bits of a resolved schedule, outside kAllFlags: resolved, and
// whether the caller chose the resident pool (the auto-disable rule for
// large explicit pools applies only when it did not).  A caller's bits
// outside kAllFlags are dropped, so no caller can mark a schedule resolved.
constexpr int32_t kResolved = 1 << 30, kResChosen = 1 << 29;

ldpc_schedule resolve_schedule(const ldpc_schedule* s)
{
    ldpc_schedule r{};
    if (s) r = *s;
    r.flags_set &= kAllFlags;
    r.flags = (kDefaultFlags & ~r.flags_set) | (r.flags & r.flags_set);
    r.flags &= kAllFlags;
    r.flags_set = kAllFlags | kResolved | ((r.flags_set & LDPC_SCHED_RESIDENT) ? kResChosen : 0);
    if (r.group_tiles == 0) r.group_tiles = -2;  // per-algorithm default, resolved at init
    // (3: compressed min-sum only; the fp64 variable kernels take 1, 2, 4 or
    // 8); -2: the default, chosen per decode by the prior's form (var_cpw_for)
    if (r.var_cpw < 1 || r.var_cpw > 8 || (r.var_cpw > 4 && r.var_cpw != 8)) r.var_cpw = -2;
    if (r.pool_tiles <= 0) r.pool_tiles = 0;  // the default, resolved at init (kDefaultPoolTiles / gen_pool_tiles)
    if (r.poll_every <= 0) r.poll_every = kDefaultResPoll;
    if (r.syn_blocks <= 0) r.syn_blocks = kDefaultSynBlocks;
    r.syn_blocks = std::min(r.syn_blocks, 256);
    r.reserved = 0;
    return r;
}

static thread_local std::string g_err;

// Sampled launches (Engine::profile): the start / stop events ride on the
// kernel's own dispatch packet (hipExtLaunchKernelGGL), so they time the
// kernel as the profiler does -- separate marker packets around it added the
// dispatch latency (~4 us per 71 us launch against the rocprofv3 trace).
// mark_begin arms g_ext; the next klaunch on this thread consumes it, and
// mark_end disarms it on every path.
struct ExtEvents {
    hipEvent_t b = nullptr, e = nullptr;
};
static thread_local ExtEvents g_ext;

template <typename F, typename... Args>
static void klaunch(F kernel, dim3 grid, dim3 block, uint32_t shm, hipStream_t s, Args... args)
{
    if (g_ext.b) {
        hipExtLaunchKernelGGL(kernel, grid, block, shm, s, g_ext.b, g_ext.e, 0, args...);
        g_ext = {};
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
    }
}
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }

int64_t engine_bytes_per_codeword(const HostGraph& g)
{
    // v2c + c2v (E fp64 each) + prior (N fp64) + hard (N bits) + state
    return 2 * g.E * 8 + (int64_t)g.N * 8 + (g.N + 7) / 8 + 8;
}

Engine::~Engine()
{
    if (device >= 0) hipSetDevice(device);
    if (stream) hipStreamSynchronize(stream);
    for (int c = 0; c < K_NCLASS; c++)
        for (auto& p : ev_live[c]) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    for (auto e : ev_pool) hipEventDestroy(e);
    hipFree(d_fresh); hipFree(d_occ); hipFree(d_lane_b); hipFree(d_lane_n); hipFree(d_ctr);
    if (h_poll) hipHostFree(h_poll);
    if (h_fault) hipHostFree(h_fault);
    hipFree(d_row_ptr); hipFree(d_col_idx); hipFree(d_col_idx_T); hipFree(d_col_ptr); hipFree(d_col_edge); hipFree(d_col_er); hipFree(d_row_pos);
    hipFree(d_unsat); hipFree(d_done); hipFree(d_fin); hipFree(d_fin_b); hipFree(d_fin_n);
    hipFree(d_sgn);
    hipFree(v2c); if (c2v != v2c) hipFree(c2v); hipFree(prior); hipFree(hard); hipFree(active); hipFree(iters); hipFree(valid);
    hipFree(post_t);
    hipFree(pcode); hipFree(d_ptab); hipFree(d_expand);
    if (h_ptab) hipHostFree(h_ptab);
    if (stream) hipStreamDestroy(stream);
}

template <typename T>
static int upload(T** dst, const std::vector<T>& v)
{
    const size_t n = std::max<size_t>(v.size(), 1);
    LDPC_HIP(hipMalloc((void**)dst, n * sizeof(T)));
    if (!v.empty()) LDPC_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return LDPC_OK;
}

// MSA-C scratch of `tiles` group tiles: record planes [tiles][M][4][64] fp64
// (m1, m2, n0, n1), then the meta words [tiles][M][64] u16
static size_t msa_scratch_bytes(int64_t tiles, int32_t M)
{
    return (size_t)tiles * M * dev::TILE * (dev::MSA_REC_PLANES * sizeof(double) + sizeof(uint16_t));
}
static double* msa_rec(double* scratch) { return scratch; }
static uint16_t* msa_meta(double* scratch, int64_t tiles, int32_t M)
{
    return reinterpret_cast<uint16_t*>(scratch + (size_t)tiles * M * dev::MSA_REC_PLANES * dev::TILE);
}

// Degree buckets of the register-staged generic kernels (kernels.hpp *_gr):
// the smallest bucket >= the graph's maximum degree, 0 when none holds it
// (the memory-staged *_gen kernels then run; no continuous mode without a
// variable bucket).
static constexpr int kGenCheckBuckets[] = {8, 16, 32, 48, 64, 96, 0};
static constexpr int kGenVarBuckets[] = {4, 8, 12, 16, 24, 32, 0};
static int gen_bucket(int32_t dmax, const int* buckets)
{
    for (const int* b = buckets; *b; ++b)
        if (dmax <= *b) return *b;
    return 0;
}

// Default resident pool of a code other than the (8, 72)-regular one: as many
// tiles as keep the pool's messages + fp64 priors within the DNA pool's
// footprint (kDefaultPoolTiles x 85 MB ~ the 256 MB Infinity Cache).
constexpr double kGenPoolBytes = 226e6;
static int32_t gen_pool_tiles(const HostGraph& g)
{
    const double per_tile = 64.0 * 8.0 * ((double)g.E + (double)g.N);
    return (int32_t)std::max(1.0, std::min(256.0, std::floor(kGenPoolBytes / std::max(per_tile, 1.0))));
}

int Engine::init(const HostGraph* graph, int dev, int algorithm, int64_t chunk, const ldpc_schedule* schedule,
                 bool resolved)
{
    g = graph;
    device = dev;
    algo = algorithm;
    if (resolved && schedule && (schedule->flags_set & kResolved)) {
        sched = *schedule;  // the host API's slot: resolved once per call (capi.cpp)
        sched.pool_tiles = std::max(sched.pool_tiles, 0);
        sched.poll_every = std::max(sched.poll_every, 1);
        sched.syn_blocks = std::min(std::max(sched.syn_blocks, 1), 256);
    } else {
        sched = resolve_schedule(schedule);
    }
    if (algo < LDPC_ALGO_BP || algo > LDPC_ALGO_GALLAGER_B2) { set_error("unknown algorithm"); return LDPC_ERR_ARG; }
    const bool int_algo = algo >= LDPC_ALGO_QMSA;
    int ndev = 0;
    LDPC_HIP(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) { set_error("device ordinal out of range"); return LDPC_ERR_DEVICE; }
    LDPC_HIP(hipSetDevice(dev));
    LDPC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));

    const bool reg_72_8 = g->regular_dc && g->dc_max == 72 && g->regular_dv && g->dv_max == 8;
    // compressed min-sum: the packed column table carries edge ids (E < 2^18)
    msa_c = algo == LDPC_ALGO_MSA && reg_72_8 && g->N % 16 == 0 && g->E < ((int64_t)1 << dev::MSA_ER_SHIFT) &&
            sched_flag(sched, LDPC_SCHED_MSA_COMPRESSED);
    // continuous mode: the specialised kernels, or any code whose column
    // degrees fit a register bucket of the generic continuous variable kernel
    // (k_var_gr_cont; its syndrome k_syndrome_split_gen)
    cont = sched_flag(sched, LDPC_SCHED_CONTINUOUS) && !int_algo &&
           (reg_72_8 || (g->regular_dv && g->dv_max == 8) || gen_bucket(g->dv_max, kGenVarBuckets) != 0);
    // resident pool: a few tiles whose whole state fits the
    // Infinity Cache, check->variable messages written over the variable->check
    // messages they are computed from (each row's / column's edges are read
    // into registers before its outputs are stored), no c2v scratch
    // (other codes: row and column degrees in register buckets, k_check_gr_res + k_var_gr_cont in place)
    const bool gen_res = !reg_72_8 && gen_bucket(g->dc_max, kGenCheckBuckets) != 0 &&
                         gen_bucket(g->dv_max, kGenVarBuckets) != 0;
    res = sched_flag(sched, LDPC_SCHED_RESIDENT) && cont && !msa_c && ((reg_72_8 && g->N % 32 == 0) || gen_res);
    // by default the resident pool is the Infinity-Cache-sized one: a caller's
    // explicit larger pool (the host API's chunks, the DNA batch) runs the
    // grouped schedule (A/B, 272-codeword DNA batch at cap 320: 193k -> 250k cw/s)
    const bool res_chosen = (sched.flags_set & kResChosen) != 0;
    if (res && !res_chosen && chunk > kResAutoMaxTiles * 64) res = false;
    // an (8, 72)-regular code larger than the DNA code: its default 3-tile pool
    // would overflow the Infinity Cache (RS(9,72,8), N = 36 864: 509 MB, 12 %
    // slower than the grouped schedule, profiles/r6/generic_codes.txt)
    if (res && !res_chosen && reg_72_8 && sched.pool_tiles <= 0 &&
        64.0 * 8.0 * kDefaultPoolTiles * ((double)g->E + (double)g->N) > 1.15 * kGenPoolBytes)
        res = false;
    nt_d = sched_flag(sched, LDPC_SCHED_NONTEMPORAL) && !res;  // the pool is meant to stay cached
    debug_no_drain = sched_flag(sched, LDPC_SCHED_DEBUG_NO_DRAIN);
    debug_bad_lane = sched_flag(sched, LDPC_SCHED_DEBUG_BAD_LANE);
    var_cpw = sched.var_cpw;
    res_poll = sched.poll_every;
    if (chunk <= 0) {
        size_t fr = 0, tot = 0;
        LDPC_HIP(hipMemGetInfo(&fr, &tot));
        // half of the free memory for the resident state, at most 16384 codewords;
        // compressed min-sum in continuous mode: a small lane pool (its scattered
        // v2c stores run ~45 % longer over a 19 GB pool than over 1.2 GB, A/B)
        const int64_t ptiles = sched.pool_tiles > 0 ? sched.pool_tiles : reg_72_8 ? kDefaultPoolTiles : gen_pool_tiles(*g);
        const int64_t want = res ? 64 * ptiles : (msa_c && cont) ? kMsaPool : 16384;
        chunk = std::min<int64_t>(want, (int64_t)(fr / 2) / engine_bytes_per_codeword(*g));
    }
    cap = std::max<int64_t>(64, (chunk + 63) / 64 * 64);
    cap_tiles = cap / 64;
    if (cap_tiles > 65535) { set_error("chunk too large (max 4194240 codewords)"); return LDPC_ERR_ARG; }
    // group: tiles whose check->variable messages are live at once.  Small
    // groups keep c2v resident in the 256 MB Infinity Cache between the check
    // and the variable phase; the resident pool launches
    // each phase over the whole pool.
    int64_t group = sched.group_tiles;
    if (group == -2) group = msa_c ? kDefaultMsaGroupTiles : kDefaultGroupTiles;
    group_tiles = (res || group <= 0 || group > cap_tiles) ? cap_tiles : group;

    int rc;
    if ((rc = upload(&d_row_ptr, g->row_ptr)) || (rc = upload(&d_col_idx, g->col_idx)) ||
        (rc = upload(&d_col_ptr, g->col_ptr)) || (rc = upload(&d_col_edge, g->col_edge)))
        return rc;
    if (msa_c) {  // (row << 18) | edge id per CSC position (k_var_msa_c); E < 2^18 (above), M < 2^14
        if (g->M >= (1 << (32 - dev::MSA_ER_SHIFT))) { set_error("MSA-C: too many rows"); return LDPC_ERR_UNSUPPORTED; }
        std::vector<uint32_t> er(g->col_edge.size());
        for (size_t q = 0; q < er.size(); q++)
            er[q] = ((uint32_t)g->edge_row[(size_t)g->col_edge[q]] << dev::MSA_ER_SHIFT) | (uint32_t)g->col_edge[q];
        if ((rc = upload(&d_col_er, er))) return rc;
        // CSR edge -> its v2c position: the compressed min-sum keeps v2c in
        // column order (contiguous variable-phase stores, gathered check
        // reads), edge s of column j at j * DV + s -- or, row-block-major,
        // at s * N + j when edge s of every column lies in row block s
        // (array codes such as the DNA code's RS-LDPC H: M = DV blocks of
        // M / DV rows), so a row's gathers stay inside one N-segment region
        const int dv = g->dv_max;
        bool rb = g->M % dv == 0;  // (round 4 A/B: +1.1 %, profiles/r4/rb/)
        for (int32_t j = 0; rb && j < g->N; j++)
            for (int s2 = 0; rb && s2 < dv; s2++)
                rb = g->edge_row[(size_t)g->col_edge[(size_t)j * dv + s2]] / (g->M / dv) == s2;
        msa_pa = rb ? 1 : dv;
        msa_pb = rb ? g->N : 1;
        std::vector<int32_t> pos(g->col_edge.size());
        for (size_t q = 0; q < pos.size(); q++)
            pos[(size_t)g->col_edge[q]] = (int32_t)(q / dv) * msa_pa + (int32_t)(q % dv) * msa_pb;
        if ((rc = upload(&d_row_pos, pos))) return rc;
    }
    if (g->regular_dc && g->dc_max > 0) {
        std::vector<int32_t> T((size_t)g->dc_max * g->M);
        for (int32_t i = 0; i < g->M; i++)
            for (int k = 0; k < g->dc_max; k++) T[(size_t)k * g->M + i] = g->col_idx[(size_t)i * g->dc_max + k];
        if ((rc = upload(&d_col_idx_T, T))) return rc;
    }
    if (cont) {
        LDPC_HIP(hipMalloc((void**)&d_fresh, (size_t)cap_tiles * sizeof(uint64_t)));
        LDPC_HIP(hipMalloc((void**)&d_occ, (size_t)cap_tiles * sizeof(uint64_t)));
        LDPC_HIP(hipMalloc((void**)&d_lane_b, (size_t)cap * sizeof(int64_t)));
        LDPC_HIP(hipMalloc((void**)&d_lane_n, (size_t)cap * sizeof(int32_t)));
        LDPC_HIP(hipMalloc((void**)&d_ctr, (size_t)(1 + kRing) * sizeof(unsigned long long)));
        LDPC_HIP(hipHostMalloc((void**)&h_poll, (size_t)kRing * sizeof(unsigned long long),
                               hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(h_poll, 0, (size_t)kRing * sizeof(unsigned long long));
        LDPC_HIP(hipHostGetDevicePointer((void**)&d_poll, h_poll, 0));
        LDPC_HIP(hipHostMalloc((void**)&h_fault, dev::kFaultWords * sizeof(unsigned long long),
                               hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(h_fault, 0, dev::kFaultWords * sizeof(unsigned long long));
        LDPC_HIP(hipHostGetDevicePointer((void**)&d_fault, h_fault, 0));
        LDPC_HIP(hipMalloc((void**)&d_unsat, (size_t)cap_tiles * sizeof(unsigned long long)));
        LDPC_HIP(hipMalloc((void**)&d_done, (size_t)cap_tiles * sizeof(unsigned int)));
        LDPC_HIP(hipMalloc((void**)&d_fin, (size_t)cap_tiles * sizeof(uint64_t)));
        LDPC_HIP(hipMalloc((void**)&d_fin_b, (size_t)cap * sizeof(int64_t)));
        LDPC_HIP(hipMalloc((void**)&d_fin_n, (size_t)cap * sizeof(int32_t)));
        // grouped continuous schedule: a separate syndrome launch spread over
        // several blocks per tile (the resident pool fuses it into the check)
        syn_blocks = res ? 0 : sched.syn_blocks;
        // single fill (the DNA batch): step 0's refill stores only the prior and
        // step 1's check derives the first messages from it (k_check_bp_first)
        first_fp = !res && reg_72_8 && algo == LDPC_ALGO_BP && sched_flag(sched, LDPC_SCHED_FIRST_FROM_PRIOR);
    }
    const size_t E = (size_t)std::max<int64_t>(g->E, 1);
    LDPC_HIP(hipMalloc((void**)&v2c, (size_t)cap * E * sizeof(double)));
    if (res) {
        c2v_tiles = cap_tiles;
        c2v = v2c;  // in place
    } else {
        // continuous mode's drain tail (< 1/32 occupancy) launches wider groups
        c2v_tiles = std::max<int64_t>(group_tiles, cont ? (cap_tiles + 3) / 4 : 0);
        c2v_bytes = msa_c ? msa_scratch_bytes(c2v_tiles, g->M) : (size_t)c2v_tiles * 64 * E * sizeof(double);
        LDPC_HIP(hipMalloc((void**)&c2v, c2v_bytes));
    }
    LDPC_HIP(hipMalloc((void**)&prior, (size_t)cap * g->N * sizeof(double)));
    if (msa_c) LDPC_HIP(hipMalloc((void**)&d_sgn, (size_t)cap * g->N));
    LDPC_HIP(hipMalloc((void**)&hard, (size_t)cap_tiles * g->N * sizeof(uint64_t)));
    LDPC_HIP(hipMalloc((void**)&active, (size_t)cap_tiles * sizeof(uint64_t)));
    LDPC_HIP(hipMalloc((void**)&iters, (size_t)cap * sizeof(int32_t)));
    LDPC_HIP(hipMalloc((void**)&valid, (size_t)cap * sizeof(uint8_t)));
    if (!int_algo && (res || group_tiles < cap_tiles)) return probe(kProbes);
    return LDPC_OK;
}

int32_t Engine::flags() const
{
    return (nt_d ? LDPC_SCHED_NONTEMPORAL : 0) | (cont ? LDPC_SCHED_CONTINUOUS : 0) |
           (msa_c ? LDPC_SCHED_MSA_COMPRESSED : 0) | (res ? LDPC_SCHED_RESIDENT : 0) |
           (syn_blocks > 0 ? LDPC_SCHED_SPLIT_SYNDROME : 0) | (first_fp ? LDPC_SCHED_FIRST_FROM_PRIOR : 0) |
           (sched.flags & (LDPC_SCHED_LR_TABLE | LDPC_SCHED_DEBUG_NO_DRAIN | LDPC_SCHED_DEBUG_BAD_LANE));
}

// Placement probe.  The resident pool (~226 MB at 3 tiles) and the grouped
// schedule's check->variable scratch (~226 MB at G = 3) are meant to stay in
// the 256 MB Infinity Cache, a memory-side cache whose slices belong to HBM
// channels: how well a given allocation fits depends on where its physical
// pages land, and identical engines were measured 3-4 % apart.  Allocate
// `probes` candidate buffers, time a few real check + variable steps on each
// (state zeroed, results discarded -- every decode re-initialises), keep the
// fastest.  The resident pool's candidates are timed with the plain check
// kernel on the same buffer (no syndrome bookkeeping; timing only).
int Engine::probe(int probes)
{
    const size_t E = (size_t)std::max<int64_t>(g->E, 1);
    const size_t bytes = res ? (size_t)cap * E * sizeof(double) : c2v_bytes;
    const unsigned gt = (unsigned)(res ? cap_tiles : std::min<int64_t>(group_tiles, cap_tiles));
    LDPC_HIP(hipMemsetAsync(v2c, 0, (size_t)gt * 64 * E * sizeof(double), stream));
    LDPC_HIP(hipMemsetAsync(prior, 0, (size_t)gt * 64 * g->N * sizeof(double), stream));
    LDPC_HIP(hipMemsetAsync(active, 0xff, (size_t)gt * sizeof(uint64_t), stream));
    if (d_sgn) LDPC_HIP(hipMemsetAsync(d_sgn, 0, (size_t)gt * 64 * g->N, stream));
    std::vector<double*> cand{res ? v2c : c2v};
    for (int i = 1; i < probes; i++) {
        double* p = nullptr;
        if (hipMalloc((void**)&p, bytes) != hipSuccess) { (void)hipGetLastError(); break; }
        cand.push_back(p);
    }
    for (double* p : cand) LDPC_HIP(hipMemsetAsync(p, 0, bytes, stream));
    hipEvent_t e0, e1;
    LDPC_HIP(hipEventCreate(&e0));
    LDPC_HIP(hipEventCreate(&e1));
    const int saved_stride = profile_stride;
    profile_stride = 0;
    const bool saved_res = res;
    res = false;  // plain check kernel (launch_check), in place when scratch == v2c
    size_t best = 0;
    float best_ms = 1e30f;
    int rc = LDPC_OK;
    for (size_t c = 0; c < cand.size() && rc == LDPC_OK; c++) {
        double* scratch = cand[c];
        if (saved_res) v2c = c2v = cand[c];
        for (int rep = 0; rep < 5 && rc == LDPC_OK; rep++) {  // rep 0 warms up
            if (rep == 1 && hipEventRecord(e0, stream) != hipSuccess) rc = LDPC_ERR_DEVICE;
            if (!rc) rc = launch_check(stream, scratch, 0, gt);
            if (!rc) rc = launch_var(stream, scratch, 0, gt, nullptr, dev::Refill{});
        }
        if (rc) break;
        LDPC_HIP(hipEventRecord(e1, stream));
        LDPC_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LDPC_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_ms) { best_ms = ms; best = c; }
    }
    res = saved_res;
    profile_stride = saved_stride;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    for (size_t c = 0; c < cand.size(); c++)
        if (c != best) (void)hipFree(cand[c]);
    if (res) v2c = c2v = cand[best];
    else c2v = cand[best];
    for (int k = 0; k < K_NCLASS; k++) launches[k] = 0;
    return rc;
}

hipEvent_t Engine::get_event()
{
    if (!ev_pool.empty()) { hipEvent_t e = ev_pool.back(); ev_pool.pop_back(); return e; }
    // no system-scope fence: a default event record writes back and
    // invalidates the caches, which inflated the sampled launch by ~7 %
    // against the rocprofv3 kernel trace
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

int Engine::mark_begin(KClass c, hipStream_t s, hipEvent_t* b)
{
    const int64_t idx = launches[c]++;
    *b = nullptr;
    (void)s;
    if (profile_stride <= 0 || idx % profile_stride != 0) return LDPC_OK;
    *b = get_event();
    hipEvent_t e = get_event();
    if (!*b || !e) {
        if (*b) ev_pool.push_back(*b);
        if (e) ev_pool.push_back(e);
        *b = nullptr;
        set_error("hipEventCreate failed");
        return LDPC_ERR_DEVICE;
    }
    sampled[c]++;
    g_ext = {*b, e};  // the launch inside LAUNCH_ON records them (klaunch)
    ext_stop = e;
    return LDPC_OK;
}

// Disarms g_ext on every path: a sample whose launch did not happen (nothing
// launched, or the launch failed) returns its events to the pool.
int Engine::mark_end(KClass c, hipStream_t s, hipEvent_t b)
{
    (void)s;
    const hipError_t le = hipGetLastError();
    if (b) {
        if (g_ext.b || le != hipSuccess) {
            ev_pool.push_back(b);
            ev_pool.push_back(ext_stop);
            g_ext = {};
            sampled[c]--;
        } else {
            ev_live[c].push_back({b, ext_stop});
        }
    }
    if (le != hipSuccess) {
        set_error(std::string("kernel launch: ") + hipGetErrorString(le));
        return LDPC_ERR_DEVICE;
    }
    return LDPC_OK;
}

int Engine::collect_stats()
{
    LDPC_HIP(hipSetDevice(device));
    LDPC_HIP(hipStreamSynchronize(stream));
    for (int c = 0; c < K_NCLASS; c++) {
        for (auto& p : ev_live[c]) {
            float t = 0.f;
            LDPC_HIP(hipEventElapsedTime(&t, p.first, p.second));
            ms[c] += t;
            ev_pool.push_back(p.first);
            ev_pool.push_back(p.second);
        }
        ev_live[c].clear();
    }
    return LDPC_OK;
}

#define LAUNCH_ON(strm, cls, ...)                         \
    do {                                                  \
        hipEvent_t _b;                                    \
        int _rc = mark_begin(cls, strm, &_b);             \
        if (_rc) return _rc;                              \
        __VA_ARGS__;                                      \
        _rc = mark_end(cls, strm, _b);                    \
        if (_rc) return _rc;                              \
    } while (0)
#define LAUNCH(cls, ...) LAUNCH_ON(stream, cls, __VA_ARGS__)

// check phase of tiles t0 .. t0+gt-1 into `scratch` (that group's c2v); with
// `res` the resident pool's in-place check + fused syndrome step (rstep)
int Engine::launch_check(hipStream_t s, double* scratch, int64_t t0, unsigned gt)
{
    using namespace dev;
    const int32_t M = g->M;
    const int64_t E = g->E;
    const bool reg72 = g->regular_dc && g->dc_max == 72;
    const dim3 grid((M + 3) / 4, gt), blk(256);
    const int msa = algo == LDPC_ALGO_MSA;
    if (res && !reg72) {
        if (!rstep || scratch != v2c || t0 != 0) { set_error("resident check: bad state"); return LDPC_ERR_ARG; }
#define CHECK_RES(D)                                                                                            \
    (msa ? klaunch((k_check_gr_res<true, D>), grid, blk, 0, s, v2c, d_row_ptr, M, E, *rstep)                   \
         : klaunch((k_check_gr_res<false, D>), grid, blk, 0, s, v2c, d_row_ptr, M, E, *rstep))
        const int cb = gen_bucket(g->dc_max, kGenCheckBuckets);
        LAUNCH_ON(s, K_CHECK, {
            if (cb == 8) CHECK_RES(8);
            else if (cb == 16) CHECK_RES(16);
            else if (cb == 32) CHECK_RES(32);
            else if (cb == 48) CHECK_RES(48);
            else if (cb == 64) CHECK_RES(64);
            else CHECK_RES(96);
        });
#undef CHECK_RES
        return LDPC_OK;
    }
    if (res) {
        if (!rstep || msa_c || scratch != v2c) { set_error("resident check: bad state"); return LDPC_ERR_ARG; }
        if (msa)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa<72, false, true>), grid, blk, 0, s, v2c, v2c, active, M, E, t0, *rstep));
        else
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_bp<72, false, true>), grid, blk, 0, s, v2c, v2c, active, M, E, t0, *rstep));
        return LDPC_OK;
    }
    if (msa_c) {  // 1-D XCD-affine grid (k_check_msa_c)
        const dim3 g1((unsigned)((M + 3) / 4) * gt);
        if (nt_d)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, true>), g1, blk, 0, s, v2c, msa_rec(scratch),
                                          msa_meta(scratch, c2v_tiles, M), active, d_row_pos, M, E, t0, gt));
        else
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, false>), g1, blk, 0, s, v2c, msa_rec(scratch),
                                          msa_meta(scratch, c2v_tiles, M), active, d_row_pos, M, E, t0, gt));
        return LDPC_OK;
    }
    if (reg72) {
        // scratch == v2c only in the resident pool's placement probe (timing)
        LAUNCH_ON(s, K_CHECK, {
            if (msa && nt_d) klaunch((k_check_msa<72, true, false>), grid, blk, 0, s, v2c, scratch, active, M, E, t0, ResStep{});
            else if (msa) klaunch((k_check_msa<72, false, false>), grid, blk, 0, s, v2c, scratch, active, M, E, t0, ResStep{});
            else if (nt_d) klaunch((k_check_bp<72, true, false>), grid, blk, 0, s, v2c, scratch, active, M, E, t0, ResStep{});
            else klaunch((k_check_bp<72, false, false>), grid, blk, 0, s, v2c, scratch, active, M, E, t0, ResStep{});
        });
    } else {
        // generic row degrees: registers up to the bucket of dc_max, else memory
        const bool bp = algo == LDPC_ALGO_BP;
#define CHECK_GR(D)                                                                                                 \
    (bp ? klaunch(k_check_bp_gr<D>, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0)                    \
        : klaunch(k_check_msa_gr<D>, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0))
        LAUNCH_ON(s, K_CHECK, {
            switch (gen_bucket(g->dc_max, kGenCheckBuckets)) {
                case 8: CHECK_GR(8); break;
                case 16: CHECK_GR(16); break;
                case 32: CHECK_GR(32); break;
                case 48: CHECK_GR(48); break;
                case 64: CHECK_GR(64); break;
                case 96: CHECK_GR(96); break;
                default:
                    if (bp) klaunch(k_check_bp_gen, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0);
                    else klaunch(k_check_msa_gen, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0);
            }
        });
#undef CHECK_GR
    }
    return LDPC_OK;
}

template <bool MSA, bool NT, bool CONT, bool INPLACE, bool PC = false>
static void var_m_cpw(int cpw, hipStream_t s, dim3 grid, const double* c2v, double* v2c, double* prior, uint64_t* hard,
                      const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N, int64_t E, int64_t t0,
                      const dev::Refill& rf)
{
    using namespace dev;
    if (cpw == 8)
        klaunch((k_var_m<MSA, 8, NT, CONT, 8, INPLACE, PC>), grid, dim3(256), 0, s, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (cpw == 4)
        klaunch((k_var_m<MSA, 8, NT, CONT, 4, INPLACE, PC>), grid, dim3(256), 0, s, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (cpw == 2)
        klaunch((k_var_m<MSA, 8, NT, CONT, 2, INPLACE, PC>), grid, dim3(256), 0, s, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else
        klaunch((k_var_m<MSA, 8, NT, CONT, 1, INPLACE, PC>), grid, dim3(256), 0, s, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
}

// PC: coded priors (continuous refills only: rf.in_code set)
template <bool MSA>
static void var_m(bool nt, bool cont, bool inplace, int cpw, hipStream_t s, dim3 grid, const double* c2v, double* v2c,
                  double* prior, uint64_t* hard, const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N,
                  int64_t E, int64_t t0, const dev::Refill& rf)
{
    const bool pc = cont && rf.in_code != nullptr;
    // in place (the resident pool, or its placement probe) is never nontemporal
    if (inplace && pc) var_m_cpw<MSA, false, true, true, true>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (inplace && cont) var_m_cpw<MSA, false, true, true>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (inplace) var_m_cpw<MSA, false, false, true>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (nt && pc) var_m_cpw<MSA, true, true, false, true>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (nt && cont) var_m_cpw<MSA, true, true, false>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (nt) var_m_cpw<MSA, true, false, false>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (pc) var_m_cpw<MSA, false, true, false, true>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else if (cont) var_m_cpw<MSA, false, true, false>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else var_m_cpw<MSA, false, false, false>(cpw, s, grid, c2v, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
}

// columns per variable-phase wave: the schedule's, or by default 2 for coded
// priors in the resident pool and the compressed min-sum, else 4 (same-box
// A/Bs, profiles/r3/coded/cpw_probe.txt)
int Engine::var_cpw_for(const dev::Refill& rf) const
{
    if (var_cpw > 0) return var_cpw;
    return (rf.fresh && rf.in_code && (res || msa_c)) ? kDefaultVarCpwCoded : kDefaultVarCpw;
}

// variable phase (+ hard decisions, optional posterior, continuous mode's
// refills and finished lanes' outputs) of tiles t0 .. t0+gt-1
int Engine::launch_var(hipStream_t s, double* scratch, int64_t t0, unsigned gt, double* pt, const dev::Refill& rf)
{
    using namespace dev;
    const int32_t N = g->N, M = g->M;
    const int64_t E = g->E;
    const bool reg8 = g->regular_dv && g->dv_max == 8;
    const bool cnt = rf.fresh != nullptr;
    if (msa_c) {  // N % 16 == 0 (init)
        int cpw = std::min(var_cpw_for(rf), 4);
        if (N % (4 * cpw) != 0) cpw = 1;  // (N % 16 == 0: every CPW but 3 divides)
        const unsigned nb = gt * (unsigned)(N / (4 * cpw));
        const double* rec = msa_rec(scratch);
        const uint16_t* meta = msa_meta(scratch, c2v_tiles, M);
#define VAR_MSA_C3(CONT, CPW, NT, PC)                                                                                \
    klaunch((k_var_msa_c<72, 8, CONT, CPW, NT, PC>), dim3(nb), dim3(256), 0, s, rec, meta, v2c, prior, hard, d_sgn, \
            active, d_col_er, pt, N, M, E, t0, (uint32_t)gt, msa_pa, msa_pb, rf)
#define VAR_MSA_C2(CONT, CPW, NT)                                   \
    do {                                                            \
        if (CONT && rf.in_code) VAR_MSA_C3(CONT, CPW, NT, CONT);    \
        else VAR_MSA_C3(CONT, CPW, NT, false);                      \
    } while (0)
#define VAR_MSA_C(CONT, CPW)              \
    do {                                  \
        if (nt_d) VAR_MSA_C2(CONT, CPW, true); \
        else VAR_MSA_C2(CONT, CPW, false);     \
    } while (0)
        LAUNCH_ON(s, K_VAR, {
            if (cnt && cpw == 4) VAR_MSA_C(true, 4);
            else if (cnt && cpw == 3) VAR_MSA_C(true, 3);
            else if (cnt && cpw == 2) VAR_MSA_C(true, 2);
            else if (cnt) VAR_MSA_C(true, 1);
            else if (cpw == 4) VAR_MSA_C(false, 4);
            else if (cpw == 3) VAR_MSA_C(false, 3);
            else if (cpw == 2) VAR_MSA_C(false, 2);
            else VAR_MSA_C(false, 1);
        });
#undef VAR_MSA_C
#undef VAR_MSA_C2
#undef VAR_MSA_C3
        return LDPC_OK;
    }
    if (reg8) {
        const bool inplace = scratch == v2c;
        const int want = var_cpw_for(rf);
        const int cpw = (want != 3 && N % (4 * want) == 0) ? want : 1;
        const dim3 grid((unsigned)((N + 4 * cpw - 1) / (4 * cpw)), gt);
        LAUNCH_ON(s, K_VAR, {
            if (algo == LDPC_ALGO_MSA) var_m<true>(nt_d, cnt, inplace, cpw, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
            else var_m<false>(nt_d, cnt, inplace, cpw, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
        });
        return LDPC_OK;
    }
    const dim3 grid((N + 3) / 4, gt), blk(256);
    // generic column degrees: registers up to the bucket of dv_max, else memory
    const int vb = gen_bucket(g->dv_max, kGenVarBuckets);
    if (cnt) {
        if (!vb) { set_error("continuous mode needs column degrees <= 32"); return LDPC_ERR_ARG; }
        const bool pc = rf.in_code != nullptr;
        const bool inplace = scratch == v2c;  // the resident pool
#define VAR_GRC3(MSA, D, PC)                                                                                         \
    (inplace ? klaunch((k_var_gr_cont<MSA, D, PC, true>), grid, blk, 0, s, scratch, v2c, prior, hard, active,       \
                       d_col_ptr, d_col_edge, pt, N, E, t0, rf)                                                      \
             : klaunch((k_var_gr_cont<MSA, D, PC, false>), grid, blk, 0, s, scratch, v2c, prior, hard, active,      \
                       d_col_ptr, d_col_edge, pt, N, E, t0, rf))
#define VAR_GRC2(MSA, D) (pc ? VAR_GRC3(MSA, D, true) : VAR_GRC3(MSA, D, false))
#define VAR_GRC(D)                          \
    do {                                    \
        if (algo == LDPC_ALGO_MSA) VAR_GRC2(true, D); \
        else VAR_GRC2(false, D);            \
    } while (0)
        LAUNCH_ON(s, K_VAR, {
            if (vb == 4) VAR_GRC(4);
            else if (vb == 8) VAR_GRC(8);
            else if (vb == 12) VAR_GRC(12);
            else if (vb == 16) VAR_GRC(16);
            else if (vb == 24) VAR_GRC(24);
            else VAR_GRC(32);
        });
#undef VAR_GRC
#undef VAR_GRC2
#undef VAR_GRC3
        return LDPC_OK;
    }
    if (vb) {
        const bool bp = algo == LDPC_ALGO_BP;
#define VAR_GR(D)                                                                                                   \
    (bp ? klaunch(k_var_bp_gr<D>, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt, N, \
                  E, t0)                                                                                            \
        : klaunch(k_var_msa_gr<D>, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt,   \
                  N, E, t0))
        LAUNCH_ON(s, K_VAR, {
            if (vb == 4) VAR_GR(4);
            else if (vb == 8) VAR_GR(8);
            else if (vb == 12) VAR_GR(12);
            else if (vb == 16) VAR_GR(16);
            else if (vb == 24) VAR_GR(24);
            else VAR_GR(32);
        });
#undef VAR_GR
        return LDPC_OK;
    }
    if (algo == LDPC_ALGO_BP)
        LAUNCH_ON(s, K_VAR, klaunch(k_var_bp_gen, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt, N, E, t0));
    else
        LAUNCH_ON(s, K_VAR, klaunch(k_var_msa_gen, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt, N, E, t0));
    return LDPC_OK;
}

// Fixed passes: every codeword of the pass is initialised at once and masked
// out of later kernels when it stops.
int Engine::run_chunk(const double* d_in, int in_kind, int64_t Bc, int32_t max_iter, uint8_t* d_hard,
                      double* d_post, int post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    using namespace dev;
    const int32_t M = g->M, N = g->N;
    const int64_t E = g->E;
    const int64_t tiles = (Bc + 63) / 64;
    const int msa = algo == LDPC_ALGO_MSA;
    if (msa && in_kind == LDPC_IN_LR) { set_error("min-sum takes LLR input"); return LDPC_ERR_ARG; }
    if (msa && post_kind == LDPC_POST_RATIO) { set_error("LDPC_POST_RATIO is BP-only"); return LDPC_ERR_ARG; }
    const bool reg_rowT = g->regular_dc && d_col_idx_T != nullptr;
    if (d_post && !post_t) LDPC_HIP(hipMalloc((void**)&post_t, (size_t)cap * N * sizeof(double)));
    double* pt = d_post ? post_t : nullptr;

    const dim3 blk(256);
    const dim3 g_init((N + 63) / 64, (unsigned)tiles);
    const dim3 g_cols_all((N + 3) / 4, (unsigned)tiles);

    LAUNCH(K_INIT, klaunch(k_init, g_init, blk, 0, stream, d_in, in_kind == LDPC_IN_LLR ? 1 : 0, msa, Bc, N,
                           E, d_col_ptr, d_col_edge, prior, v2c, hard, active, iters, valid, d_sgn, msa_pa, msa_pb));
    for (int32_t n = 0;; n++) {
        if (reg_rowT && g->dc_max == 72)
            LAUNCH(K_SYN, klaunch(k_syndrome<72>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                  iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        else
            LAUNCH(K_SYN, klaunch(k_syndrome<0>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                  iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        if (n >= max_iter) break;
        // groups of G tiles: check(group) then variable(group), the group's
        // c2v in the scratch
        for (int64_t t0 = 0; t0 < tiles; t0 += group_tiles) {
            const unsigned gt = (unsigned)std::min<int64_t>(group_tiles, tiles - t0);
            int rc;
            if ((rc = launch_check(stream, c2v, t0, gt))) return rc;
            if ((rc = launch_var(stream, c2v, t0, gt, pt, dev::Refill{}))) return rc;
        }
    }
    if (d_post)
        LAUNCH(K_FINAL, klaunch(k_finalize, g_cols_all, blk, 0, stream, post_t, prior, iters, d_post, msa,
                                post_kind == LDPC_POST_RATIO ? 1 : 0, Bc, N));
    if (d_hard) {
        const int64_t nblk = Bc * ((N + 255) / 256);
        const unsigned grid = (unsigned)std::min<int64_t>(nblk, 1 << 20);
        LAUNCH(K_FINAL, klaunch(k_unpack_hard, dim3(grid), blk, 0, stream, hard, d_hard, Bc, N));
    }
    if (d_iters) LDPC_HIP(hipMemcpyAsync(d_iters, iters, (size_t)Bc * sizeof(int32_t), hipMemcpyDeviceToDevice, stream));
    if (d_valid) LDPC_HIP(hipMemcpyAsync(d_valid, valid, (size_t)Bc, hipMemcpyDeviceToDevice, stream));
    return LDPC_OK;
}

int Engine::set_params(int32_t precision, double step, int32_t beta, uint64_t seed)
{
    if (precision < 2 || precision > 16 || !(step > 0) || beta < 0) {
        set_error("quantized min-sum needs 2 <= precision <= 16, step > 0, offset >= 0");
        return LDPC_ERR_ARG;
    }
    q_precision = precision;
    q_step = step;
    q_beta = beta;
    tie_seed = seed;
    return LDPC_OK;
}

// Integer-message decoders (kernels_int.hpp): fixed schedule, the same
// syndrome / group loop as run_chunk on int32 views of the fp64 buffers.
int Engine::run_chunk_int(const double* d_in, int64_t Bc, int64_t b_base, int32_t max_iter, uint8_t* d_hard,
                          double* d_post, int32_t* d_iters, uint8_t* d_valid)
{
    using namespace dev;
    const int32_t M = g->M, N = g->N;
    const int64_t E = g->E;
    const int64_t tiles = (Bc + 63) / 64;
    IntParams ip{};
    ip.algo = algo;
    ip.max_value = (1 << (q_precision - 1)) - 1;  // Set_MSA dec.cpp:1688-1689
    ip.min_value = -ip.max_value;
    ip.beta = q_beta;
    ip.step = q_step;
    ip.seed = tie_seed;
    b_base += tie_base;
    const int dv = g->dv_max;  // D_v (CheckRegular)
    if (algo == LDPC_ALGO_GALLAGER_A) { ip.b_var = dv - 1; ip.b_dec = dv; }
    else if (algo == LDPC_ALGO_GALLAGER_B1) { ip.b_var = dv - 2; ip.b_dec = dv - 1; }
    else { ip.b_var = dv / 2 + dv % 2; ip.b_dec = dv / 2 + 1; }
    const bool reg_rowT = g->regular_dc && d_col_idx_T != nullptr;
    if (d_post && !post_t) LDPC_HIP(hipMalloc((void**)&post_t, (size_t)cap * N * sizeof(double)));
    double* pt = d_post ? post_t : nullptr;
    int32_t* iv2c = reinterpret_cast<int32_t*>(v2c);
    int32_t* ic2v = reinterpret_cast<int32_t*>(c2v);
    int32_t* iprior = reinterpret_cast<int32_t*>(prior);
    const dim3 blk(256);
    const dim3 g_cols_all((N + 3) / 4, (unsigned)tiles);
    LAUNCH(K_INIT, klaunch(k_init_int, dim3((N + 63) / 64, (unsigned)tiles), blk, 0, stream, d_in, Bc,
                           b_base, N, E, d_col_ptr, d_col_edge, ip, iprior, iv2c, hard, active, iters, valid));
    for (int32_t n = 0;; n++) {
        if (reg_rowT && g->dc_max == 72)
            LAUNCH(K_SYN, klaunch(k_syndrome<72>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                  iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        else
            LAUNCH(K_SYN, klaunch(k_syndrome<0>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                  iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        if (n >= max_iter) break;
        for (int64_t t0 = 0; t0 < tiles; t0 += group_tiles) {
            const unsigned gt = (unsigned)std::min<int64_t>(group_tiles, tiles - t0);
            LAUNCH(K_CHECK, klaunch(k_check_int, dim3((M + 3) / 4, gt), blk, 0, stream, iv2c, ic2v, active,
                                    d_row_ptr, M, E, t0, ip));
            LAUNCH(K_VAR, klaunch(k_var_int, dim3((N + 3) / 4, gt), blk, 0, stream, ic2v, iv2c, iprior,
                                  hard, active, d_col_ptr, d_col_edge, pt, N, E, t0, b_base, n, ip));
        }
    }
    if (d_post)
        LAUNCH(K_FINAL, klaunch(k_finalize_int, g_cols_all, blk, 0, stream, post_t, iprior, iters, d_post, Bc, N));
    if (d_hard) {
        const int64_t nblk = Bc * ((N + 255) / 256);
        const unsigned grid = (unsigned)std::min<int64_t>(nblk, 1 << 20);
        LAUNCH(K_FINAL, klaunch(k_unpack_hard, dim3(grid), blk, 0, stream, hard, d_hard, Bc, N));
    }
    if (d_iters) LDPC_HIP(hipMemcpyAsync(d_iters, iters, (size_t)Bc * sizeof(int32_t), hipMemcpyDeviceToDevice, stream));
    if (d_valid) LDPC_HIP(hipMemcpyAsync(d_valid, valid, (size_t)Bc, hipMemcpyDeviceToDevice, stream));
    return LDPC_OK;
}

// Coded input.  The continuous schedules keep every lane's prior as its code
// (1 byte per column and lane instead of 8; the kernels look the value up in
// the 256-entry table); the others decode fp64 input expanded from the codes
// one pass of <= cap codewords at a time.  Either way each codeword sees
// exactly the prior values the table gives its codes.
int Engine::decode_codes(const int8_t* d_codes, const double* h_table, int table_kind, int64_t B, int32_t max_iter,
                         uint8_t* d_hard, double* d_post, int post_kind, int32_t* d_iters, uint8_t* d_valid,
                         double* d_stage)
{
    if (B < 0 || max_iter < 0) { set_error("B and max_iter must be >= 0"); return LDPC_ERR_ARG; }
    if (!h_table || (B > 0 && !d_codes)) { set_error("decode_codes: null codes or table"); return LDPC_ERR_ARG; }
    if (table_kind != LDPC_IN_LLR && table_kind != LDPC_IN_LR) { set_error("table kind: LDPC_IN_LLR or LDPC_IN_LR"); return LDPC_ERR_ARG; }
    const bool bp = algo == LDPC_ALGO_BP;
    if (!bp && table_kind != LDPC_IN_LLR) { set_error("min-sum and the integer decoders take an LLR table"); return LDPC_ERR_ARG; }
    if (B == 0) return LDPC_OK;
    LDPC_HIP(hipSetDevice(device));
    constexpr int T = 256;
    // the prior of code k: BP's LR (the host libm exp of an LLR table, as
    // DNA_main.cpp:1344 computes LR), the LLR otherwise
    double tab[T];
    for (int i = 0; i < T; i++) tab[i] = (bp && table_kind == LDPC_IN_LLR) ? std::exp(h_table[i]) : h_table[i];
    if (!d_ptab) {
        LDPC_HIP(hipMalloc((void**)&d_ptab, T * sizeof(double)));
        LDPC_HIP(hipHostMalloc((void**)&h_ptab, T * sizeof(double), hipHostMallocDefault));
    }
    if (!ptab_valid || std::memcmp(tab, h_ptab, sizeof tab) != 0) {
        // the previous upload (and every kernel that reads the table) done first
        LDPC_HIP(hipStreamSynchronize(stream));
        std::memcpy(h_ptab, tab, sizeof tab);
        LDPC_HIP(hipMemcpyAsync(d_ptab, h_ptab, sizeof tab, hipMemcpyHostToDevice, stream));
        ptab_valid = true;
    }
    const int in_kind = bp ? LDPC_IN_LR : LDPC_IN_LLR;
    if (cont && algo < LDPC_ALGO_QMSA) {
        if (!pcode) LDPC_HIP(hipMalloc((void**)&pcode, (size_t)cap * g->N));
        cur_codes = d_codes;
        const int rc = run_cont(nullptr, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
        cur_codes = nullptr;
        return rc;
    }
    // fp64 staging of one pass: the caller's (the host API's d_in) or the
    // engine's own, sized to the largest pass seen
    const size_t N = (size_t)g->N;
    const int64_t pass = std::min<int64_t>(cap, B);
    double* stage = d_stage;
    if (!stage) {
        if (expand_rows < pass) {
            LDPC_HIP(hipStreamSynchronize(stream));  // a previous decode may still read it
            LDPC_HIP(hipFree(d_expand));
            d_expand = nullptr;
            expand_rows = 0;
            LDPC_HIP(hipMalloc((void**)&d_expand, (size_t)pass * N * sizeof(double)));
            expand_rows = pass;
        }
        stage = d_expand;
    }
    const int64_t tb = tie_base;
    for (int64_t b0 = 0; b0 < B; b0 += cap) {
        const int64_t Bc = std::min<int64_t>(cap, B - b0);
        if (int rc = expand_lr(d_codes + (size_t)b0 * N, d_ptab, stage, Bc * (int64_t)N, stream)) return rc;
        tie_base = tb + b0;  // the integer decoders' tie hash keys on the index in the whole call
        const int rc = decode(stage, in_kind, Bc, max_iter, d_hard ? d_hard + (size_t)b0 * N : nullptr,
                              d_post ? d_post + (size_t)b0 * N : nullptr, post_kind, d_iters ? d_iters + b0 : nullptr,
                              d_valid ? d_valid + b0 : nullptr);
        tie_base = tb;
        if (rc) return rc;
    }
    return LDPC_OK;
}

int Engine::decode(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                   int post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    if (B < 0 || max_iter < 0) { set_error("B and max_iter must be >= 0"); return LDPC_ERR_ARG; }
    if (B == 0) return LDPC_OK;
    LDPC_HIP(hipSetDevice(device));
    if (algo >= LDPC_ALGO_QMSA) {
        if (in_kind != LDPC_IN_LLR) { set_error("integer decoders take LLR input"); return LDPC_ERR_ARG; }
        if (post_kind == LDPC_POST_RATIO && d_post) { set_error("LDPC_POST_RATIO is BP-only"); return LDPC_ERR_ARG; }
        const size_t N = (size_t)g->N;
        for (int64_t b0 = 0; b0 < B; b0 += cap) {
            const int64_t Bc = std::min<int64_t>(cap, B - b0);
            int rc = run_chunk_int(d_in + (size_t)b0 * N, Bc, b0, max_iter, d_hard ? d_hard + (size_t)b0 * N : nullptr,
                                   d_post ? d_post + (size_t)b0 * N : nullptr, d_iters ? d_iters + b0 : nullptr,
                                   d_valid ? d_valid + b0 : nullptr);
            if (rc) return rc;
        }
        return LDPC_OK;
    }
    if (cont) return run_cont(d_in, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
    // balanced passes of <= cap codewords (multiples of 64 except the tail)
    const int64_t npass = (B + cap - 1) / cap;
    const int64_t per = std::min<int64_t>(cap, ((B + npass - 1) / npass + 63) / 64 * 64);
    const size_t N = (size_t)g->N;
    for (int64_t b0 = 0; b0 < B; b0 += per) {
        const int64_t Bc = std::min<int64_t>(per, B - b0);
        int rc = run_chunk(d_in + (size_t)b0 * N, in_kind, Bc, max_iter, d_hard ? d_hard + (size_t)b0 * N : nullptr,
                           d_post ? d_post + (size_t)b0 * N : nullptr, post_kind, d_iters ? d_iters + b0 : nullptr,
                           d_valid ? d_valid + b0 : nullptr);
        if (rc) return rc;
    }
    return LDPC_OK;
}

void Engine::poll_arm(dev::ContState& cs, uint64_t q) const
{
    cs.occ_count = d_ctr + 1 + (q % kRing);
    cs.occ_clear = d_ctr + 1 + ((q + 1) % kRing);
    cs.poll_host = d_poll + (q % kRing);
    cs.poll_tag = (q + 1) & ((1ull << (64 - dev::kOccTileShift)) - 1ull);  // never the initial 0
}

// Wait for poll q's device-written word.  The engine-wide sequence keeps tags
// unique across decodes (a previous decode's trailing steps may still write
// their slots).  The stream is queried while waiting: a device error, or a
// stream that finished without the word, is an error instead of a hang.
int Engine::poll_wait(uint64_t q, unsigned long long* occ)
{
    const unsigned long long want = (q + 1) & ((1ull << (64 - dev::kOccTileShift)) - 1ull);
    volatile unsigned long long* w = h_poll + (q % kRing);
    for (uint64_t spin = 1;; spin++) {
        const unsigned long long v = *w;
        if ((v >> dev::kOccTileShift) == want) {
            *occ = v & dev::kOccMask;
            return check_fault();
        }
        if (spin % 64 == 0) {
            if (int rc = check_fault()) return rc;
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipSuccess) {
                const unsigned long long v2 = *w;
                if ((v2 >> dev::kOccTileShift) == want) {
                    *occ = v2 & dev::kOccMask;
                    return LDPC_OK;
                }
                set_error("occupancy poll " + std::to_string(q) + ": the step finished without its device write");
                return LDPC_ERR_DEVICE;
            }
            if (e != hipErrorNotReady) {
                set_error(std::string("occupancy poll: ") + hipGetErrorString(e));
                return LDPC_ERR_DEVICE;
            }
            std::this_thread::yield();
        }
    }
}

int Engine::check_fault()
{
    if (!h_fault) return LDPC_OK;
    volatile unsigned long long* w = h_fault;
    std::string msg;
    for (int k = 1; k < dev::kFaultWords; k++) {  // every word is read and cleared; the first set one is reported
        const unsigned long long v = w[k];
        if (!(v & dev::kFaultTag)) continue;
        w[k] = 0ull;
        if (!msg.empty()) continue;
        int64_t idx = (int64_t)(v & dev::kFaultIndex);
        if (idx & (int64_t)(1ull << 47)) idx -= (int64_t)(1ull << 48);  // sign of the 48-bit field
        if (k == dev::kFaultSchedule)
            msg = "device schedule fault: the code fill of tile " + std::to_string(-1 - idx) +
                  " found live or finished lanes";
        else if (k == dev::kFaultIters)
            msg = "device lane bookkeeping fault: codeword index " + std::to_string(idx) +
                  " out of range for the iteration count / valid flag access";
        else  // the variable kernels report the lane's pool slot (k_fill_codes the codeword index)
            msg = "device lane bookkeeping fault: pool slot or codeword index " + std::to_string(idx) +
                  " out of range for " + (k == dev::kFaultOutput ? "a finished codeword's hard bits / posterior" : "a refill's input row");
    }
    if (msg.empty()) return LDPC_OK;
    set_error(msg + " (skipped; the decode's outputs are incomplete)");
    return LDPC_ERR_DEVICE;
}

int Engine::sync()
{
    LDPC_HIP(hipSetDevice(device));
    LDPC_HIP(hipStreamSynchronize(stream));
    return check_fault();
}

// Continuous batching over the whole batch: lanes are refilled as codewords
// finish (the last syndrome / check block of a tile runs the lane
// bookkeeping, res_arrive), so a 64-codeword tile never idles on its slowest
// member.  The host enqueues steps and stops kLag (1 for a single fill) polls
// after the device reports an empty pool (occupied lanes == 0 once the claim
// counter has passed B); the few surplus steps find no occupied lane.
// A decode that stops on an error (a device fault at a poll, a step overrun)
// leaves the steps it already enqueued running, and they can set the fault
// words again.  Wait for them and clear the words, so that the error belongs
// to this decode alone: the next sync or decode on the engine starts clean.
int Engine::run_cont(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                     int post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    const int rc = run_cont_steps(d_in, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
    if (rc != LDPC_OK && h_fault && hipStreamSynchronize(stream) == hipSuccess) {
        volatile unsigned long long* w = h_fault;
        for (int k = 1; k < dev::kFaultWords; k++) w[k] = 0ull;
    }
    return rc;
}

int Engine::run_cont_steps(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard,
                           double* d_post, int post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    using namespace dev;
    const int msa = algo == LDPC_ALGO_MSA;
    if (msa && in_kind == LDPC_IN_LR) { set_error("min-sum takes LLR input"); return LDPC_ERR_ARG; }
    if (msa && post_kind == LDPC_POST_RATIO) { set_error("LDPC_POST_RATIO is BP-only"); return LDPC_ERR_ARG; }
    if (!d_hard || !d_iters || !d_valid) { set_error("continuous mode needs hard, iters and valid outputs"); return LDPC_ERR_ARG; }
    const int32_t M = g->M, N = g->N;
    const int64_t tiles = std::min<int64_t>(cap_tiles, (B + 63) / 64);
    if (d_post && !post_t) LDPC_HIP(hipMalloc((void**)&post_t, (size_t)cap * N * sizeof(double)));
    double* pt = d_post ? post_t : nullptr;
    // lane masks, claim counter + occupancy ring and the syndrome words in one launch
    static_assert(1 + kRing <= 256, "occupancy ring");
    LAUNCH(K_OTHER, klaunch(k_cont_reset, dim3((unsigned)std::min<int64_t>((tiles + 255) / 256, 1024)), dim3(256), 0,
                            stream, active, d_fresh, d_occ, d_ctr, 1 + kRing, d_unsat, d_done, tiles));
    ContState cs{active, d_fresh, d_occ, d_lane_b, d_lane_n, d_ctr, nullptr, B};
    cs.ntiles = tiles;
    cs.fault = d_fault;
    cs.debug_bad_lane = debug_bad_lane ? 1 : 0;
    const uint64_t q0 = poll_seq;  // this decode's first poll
    ResStep rs{hard, d_col_idx, d_unsat, d_done, d_fin, d_fin_b, d_fin_n, N, max_iter, cs, ContOut{d_iters, d_valid},
               d_row_ptr};
    const bool syn72 = g->regular_dc && g->dc_max == 72;
    const int hard_vec = ((uintptr_t)d_hard % 8 == 0 && N % 8 == 0) ? 1 : 0;
    Refill rf{d_fresh, d_lane_b, d_in, in_kind == LDPC_IN_LLR ? 1 : 0, d_fin, d_fin_b, d_fin_n,
              d_hard, d_post, post_kind == LDPC_POST_RATIO ? 1 : 0, hard_vec};
    rf.nb = B;
    rf.fault = d_fault;
    if (cur_codes) {  // coded input (decode_codes): int8 priors
        rf.in = nullptr;
        rf.in_code = cur_codes;
        rf.pcode = pcode;
        rf.ptab = d_ptab;
    }
    // A batch that fits the lane pool in one fill (the DNA batch) polls one
    // step behind instead of kLag in the resident pool, and in the grouped
    // schedule waits for the step's own poll (below): its steps take >= 30
    // us, time enough to enqueue the next, and the decode ends sooner.
    const bool single_fill = B <= tiles * 64;
    const int lag = single_fill ? 1 : kLag;
    // Host step bound.  A lane finishes its codeword at most max_iter + 2
    // steps after claiming it (refill step, max_iter iterations, the final
    // syndrome), so within every window of max_iter + 2 steps each lane either
    // finishes a codeword or has found the input drained; after
    // ceil(B / lanes) + 1 windows every lane is empty.  The host reads the
    // occupancy up to kLag polls late.  A decode still running past the bound
    // means broken device bookkeeping: stop enqueueing and report it instead
    // of spinning.  LDPC_SCHED_DEBUG_NO_DRAIN ignores the drained reading (tests).
    const int64_t lanes = tiles * 64;
    const int64_t windows = (B + lanes - 1) / lanes + 1;
    auto step_limit = [&](int64_t every) {
        return windows * ((int64_t)max_iter + 2) + (int64_t)(lag + 2) * every + 8;
    };
    auto drained = [&](unsigned long long occ) { return occ == 0 && !debug_no_drain; };
    auto overrun = [&](int64_t steps) {
        set_error("continuous decode of " + std::to_string(B) + " codewords did not drain within " +
                  std::to_string(steps) + " steps (device lane bookkeeping)");
        return LDPC_ERR_DEVICE;
    };
    if (res) {
        // resident pool: every step is check (+ the syndrome of the previous
        // step and the lane bookkeeping, ResStep) then variable (+ the
        // finished codewords' outputs) over the whole pool, messages in place;
        // the occupancy is read every res_poll steps, kLag polls behind.
        // Batches of a few pool fills (the DNA batch) poll every step: the
        // host stops at most kLag steps after the pool empties.
        const int every = B <= 8 * cap ? 1 : res_poll;
        const int64_t limit = step_limit(every);
        int rc = LDPC_OK;
        for (int64_t s = 0; rc == LDPC_OK; s++) {
            if (s >= limit) { rc = overrun(s); break; }
            const bool poll = (s % every) == every - 1;
            const uint64_t q = poll ? poll_seq++ : 0;
            if (poll) poll_arm(rs.cs, q);
            else rs.cs.occ_count = rs.cs.occ_clear = rs.cs.poll_host = nullptr;
            rstep = &rs;
            rc = launch_check(stream, c2v, 0, (unsigned)tiles);
            rstep = nullptr;
            if (rc) break;
            if ((rc = launch_var(stream, c2v, 0, (unsigned)tiles, pt, rf))) break;
            if (poll && q >= q0 + (uint64_t)lag) {
                unsigned long long occ = 0;
                if ((rc = poll_wait(q - lag, &occ))) break;
                if (drained(occ)) break;
            }
        }
        return rc;
    }
    // Grouped steps: the multi-block syndrome (+ lane bookkeeping) of every
    // tile, then check(group) + variable(group) per tile group so the group's
    // c2v stays in the Infinity Cache.  Once the input is drained and few lanes
    // remain, one check + one variable launch over all tiles per step (the
    // tail is launch-bound, and the c2v traffic is small); `low` lags the
    // device by kLag.
    bool low = false;
    // single fill: step 0's refill stores only the prior, step 1's check reads it
    const bool ffp = first_fp && single_fill && c2v != v2c;
    // single fill: wait for the step's own poll -- its syndrome (and with it
    // the poll word) comes first, so the answer arrives while the step's
    // check / variable launches still run, and no empty step follows the
    // drain; step 0 (claims and refills only) is not awaited
    const int glag = single_fill ? 0 : lag;
    Refill rf0 = rf;
    rf0.prior_only = ffp ? 1 : 0;
    const int64_t limit = step_limit(1);
    for (int64_t s = 0;; s++) {
        if (s >= limit) return overrun(s);
        const uint64_t q = poll_seq++;
        poll_arm(rs.cs, q);
        if (syn72)
            LAUNCH(K_SYN, klaunch(k_syndrome_split<72>, dim3((unsigned)(syn_blocks * tiles)), dim3(256), 0, stream,
                                  M, rs, (uint32_t)tiles));
        else
            LAUNCH(K_SYN, klaunch(k_syndrome_split_gen, dim3((unsigned)(syn_blocks * tiles)), dim3(256), 0, stream,
                                  M, rs, (uint32_t)tiles));
        const int64_t gstep = low ? std::max(group_tiles, c2v_tiles) : group_tiles;
        if (ffp && cur_codes && s == 0 && N % 64 == 0) {
            // single fill on codes: step 0 is the transpose of the claimed
            // rows into the lane codes (+ Init's decision ballots).  It stands
            // in for that step's variable kernel because k_cont_reset left
            // every lane empty, so step 0 has no live lane (active) and no
            // finished one (fin) -- k_fill_codes checks both per tile and
            // reports a violation as a device fault.
            LAUNCH(K_INIT, klaunch(k_fill_codes, dim3((unsigned)(N / 64), (unsigned)tiles), dim3(256), 0, stream,
                                   cur_codes, d_lane_b, d_fresh, pcode, d_ptab, hard, N, B, d_fault, active, d_fin));
            continue;  // (the poll of step 0 is never awaited)
        }
        for (int64_t t0 = 0; t0 < tiles; t0 += gstep) {
            const unsigned gt = (unsigned)std::min<int64_t>(gstep, tiles - t0);
            int rc;
            if (ffp && s == 1) {
                if (cur_codes)
                    LAUNCH(K_CHECK, klaunch((k_check_bp_first<72, true>), dim3((M + 3) / 4, gt), dim3(256), 0, stream,
                                            prior, pcode, d_ptab, d_col_idx, c2v, active, M, N, (int64_t)g->E, t0));
                else
                    LAUNCH(K_CHECK, klaunch((k_check_bp_first<72>), dim3((M + 3) / 4, gt), dim3(256), 0, stream,
                                            prior, pcode, d_ptab, d_col_idx, c2v, active, M, N, (int64_t)g->E, t0));
            } else if (s == 0) {
                // step 0: the reset left every lane empty and the syndrome
                // launch above only claims codewords, so no lane is active
            } else if ((rc = launch_check(stream, c2v, t0, gt))) {
                return rc;
            }
            if ((rc = launch_var(stream, c2v, t0, gt, pt, s == 0 ? rf0 : rf))) return rc;
        }
        if (q >= q0 + (uint64_t)glag && s > 0) {
            unsigned long long occ = 0;
            if (int r = poll_wait(q - glag, &occ)) return r;
            if (drained(occ)) break;
            low = occ * 32 < (unsigned long long)(tiles * 64);
        }
    }
    return LDPC_OK;
}

int Engine::gen_bsc(double* d_out, int out_kind, int64_t b0, int64_t B, const uint8_t* d_cw, int32_t n_cw,
                    uint64_t seed, double p, double llr_mag)
{
    if (B <= 0) return LDPC_OK;
    if (n_cw <= 0 || !d_cw || !d_out) { set_error("gen_bsc: bad arguments"); return LDPC_ERR_ARG; }
    LDPC_HIP(hipSetDevice(device));
    double pos = llr_mag, neg = -llr_mag;
    if (out_kind == LDPC_IN_LR) {  // the reference's host exp (DNA_main.cpp:1344)
        pos = std::exp(llr_mag);
        neg = std::exp(-llr_mag);
    }
    const uint64_t seedmix = dev::splitmix64(seed);
    LAUNCH(K_OTHER, klaunch(dev::k_gen_bsc<double>, dim3(8192), dim3(256), 0, stream, d_out,
                            out_kind == LDPC_IN_LR ? 1 : 0, b0, B, d_cw, n_cw, g->N, seedmix, p, pos, neg));
    return LDPC_OK;
}

int Engine::gen_bsc_codes(int8_t* d_out, int64_t b0, int64_t B, const uint8_t* d_cw, int32_t n_cw, uint64_t seed,
                          double p)
{
    if (B <= 0) return LDPC_OK;
    if (n_cw <= 0 || !d_cw || !d_out) { set_error("gen_bsc_codes: bad arguments"); return LDPC_ERR_ARG; }
    LDPC_HIP(hipSetDevice(device));
    const uint64_t seedmix = dev::splitmix64(seed);
    LAUNCH(K_OTHER, klaunch(dev::k_gen_bsc<int8_t>, dim3(8192), dim3(256), 0, stream, d_out, 0, b0, B, d_cw, n_cw,
                            g->N, seedmix, p, (int8_t)1, (int8_t)-1));
    return LDPC_OK;
}

int Engine::expand_lr(const int8_t* d_code, const double* d_table, double* d_out, int64_t n, hipStream_t s)
{
    if (n <= 0) return LDPC_OK;
    LDPC_HIP(hipSetDevice(device));
    const int64_t blocks = std::min<int64_t>(4096, (n / 8 + 255) / 256 + 1);
    klaunch(dev::k_lr_table, dim3((unsigned)blocks), dim3(256), 0, s, d_code, d_table, d_out, n);
    LDPC_HIP(hipGetLastError());
    return LDPC_OK;
}

int Engine::pack_bits(const uint8_t* d_in, uint8_t* d_out, int64_t nbytes)
{
    if (nbytes <= 0) return LDPC_OK;
    LDPC_HIP(hipSetDevice(device));
    const int64_t blocks = std::min<int64_t>(4096, (nbytes + 255) / 256);
    klaunch(dev::k_pack_bits, dim3((unsigned)blocks), dim3(256), 0, stream, (const uint64_t*)d_in, d_out, nbytes);
    LDPC_HIP(hipGetLastError());
    return LDPC_OK;
}

}  // namespace ldpc
