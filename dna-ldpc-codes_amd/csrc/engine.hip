// engine.hip -- device engine: memory, launch sequence, profiling.
//
// One Engine = one device, one HIP stream, message buffers for `cap`
// resident codewords.  A decode of B codewords runs in passes of <= cap
// codewords; each pass is the reference's per-frame loop
// (Run_Belief_Propagation_Decoder dec.cpp:583-605 / Run_MSA_Decoder_INF
// dec.cpp:1216-1250) executed for all resident codewords at once:
//
//   init                                  (Init_*: dec.cpp:608 / 1300)
//   for n = 0..max_iter:
//       syndrome(n)  -> codewords with c == 0 or n == max_iter stop
//       if n == max_iter: break
//       check phase  (dec.cpp:646-662 / 1398-1433)
//       variable phase + hard decision (dec.cpp:667-693 / 1597-1678)
//   finalize (posterior, hard bits, iteration counts)
//
// Stopped codewords are masked out of every later kernel (their state stays
// frozen, exactly as the reference stops touching it), and a tile whose 64
// codewords have all stopped costs one scalar load per wave.
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
#include "kernels_xr.hpp"

namespace ldpc {

constexpr int64_t kDefaultGroupTiles = 3;  // tools/sweep.py on MI355X
constexpr int64_t kDefaultNT = 1;
constexpr int64_t kDefaultPipe = 0;
constexpr int64_t kDefaultCsc = 0;
constexpr int64_t kDefaultCont = 1;
constexpr int64_t kDefaultC2vProbe = 4;  // LDPC_C2V_PROBE: candidate c2v scratch buffers timed at init
constexpr int64_t kDefaultFullLanes = 1;  // LDPC_FULL_LANES: whole-wave stores in partially converged tiles (A/B: MSA p=.002 +5.6%, BP p=.002 +7.5%, config 3 neutral)
constexpr int64_t kDefaultMsaGroupTiles = 4;  // LDPC_GROUP_TILES default for compressed min-sum (A/B, 1024-lane pool)
constexpr int64_t kDefaultMsaPool = 1024;  // LDPC_MSA_POOL: resident lanes, compressed min-sum + continuous mode (A/B)
constexpr int64_t kDefaultMsaC = 1;  // LDPC_MSA_C: compressed min-sum c2v (tools/icbench: 52.6 -> 33.5 us per tile-iteration)
constexpr int64_t kDefaultVarCpw = 4;  // LDPC_VAR_CPW (A/B over two boxes: +2.6-2.9% over 1 column per wave)
constexpr int64_t kDefaultRes = 1;       // LDPC_RES: resident in-place pool for BP / fp64 min-sum in continuous mode
constexpr int64_t kDefaultResTiles = 3;  // LDPC_RES_TILES: pool tiles (3 x 85 MB ~ the 256 MB Infinity Cache; A/B)
constexpr int64_t kDefaultResPoll = 8;
constexpr int64_t kResAutoMaxTiles = 4;      // explicit pools above this many tiles: grouped schedule unless LDPC_RES is set
constexpr int64_t kDefaultResStreams = 0;    // LDPC_RES_STREAMS: resident pool, one HIP stream per pool tile (bimodal 25.1-28.4k vs 25.7-26.2k single-stream; neutral in bench.py, so off)
constexpr int64_t kDefaultResSyn = 0;        // LDPC_RES_SYN: resident pool syndrome, 0 = fused into the check kernel, >0 = k_syndrome_split blocks per tile
constexpr int64_t kDefaultSynSplit = 32;     // LDPC_SYN_SPLIT: syndrome blocks per tile in continuous mode (0: one block, k_syndrome_cont; A/B min-sum config 5 +5-6 %)
constexpr int64_t kDefaultSynFused = 0;      // LDPC_SYN_FUSED: grouped continuous mode, syndrome fused into the check kernel
constexpr int64_t kDefaultMsaMeta = 1;  // LDPC_MSA_META: MSA-C without per-edge code bytes (32-bit meta word per row, sign bytes per column; config 5 A/B +2-3 %)
constexpr int64_t kDefaultResMsaC = 0;       // LDPC_RES_MSA_C: resident pool for compressed min-sum
constexpr int64_t kDefaultResTilesMsaC = 2;  // LDPC_RES_TILES_MSA_C: its pool tiles   // LDPC_RES_POLL: steps between occupancy polls
constexpr int64_t kDefaultPingpong = 0;      // LDPC_PINGPONG: resident BP pool, check(t) + variable(t-1) per launch
constexpr int64_t kDefaultPpCpw = 4;         // LDPC_PP_CPW: its variable-phase columns per wave
constexpr int64_t kDefaultXr = 0;            // LDPC_XR: XCD-resident BP decoder for array codes (kernels_xr.hpp)
constexpr int64_t kDefaultXrK = 3;           // LDPC_XR_K: its slots (codewords in flight) per XCD
constexpr int64_t kDefaultXrVb = 4;          // LDPC_XR_VB: column blocks per variable task (1, 2, 4)
constexpr int64_t kDefaultXrLdm = 1;         // LDPC_XR_LDM: L1-bypassing loads, 1 nontemporal, 2 agent scope

static thread_local std::string g_err;

// Sampled launches (Engine::profile): the start / stop events ride on the
// kernel's own dispatch packet (hipExtLaunchKernelGGL), so they time the
// kernel as the profiler does -- separate marker packets around it added the
// dispatch latency (~4 us per 71 us launch against the rocprofv3 trace).
// mark_begin arms g_ext; the next klaunch on this thread consumes it.
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
    if (stream2) hipStreamSynchronize(stream2);
    for (int i = 0; i < 2; i++) {
        if (ev_chk[i]) hipEventDestroy(ev_chk[i]);
        if (ev_var[i]) hipEventDestroy(ev_var[i]);
    }
    if (ev_join) hipEventDestroy(ev_join);
    for (int c = 0; c < K_NCLASS; c++)
        for (auto& p : ev_live[c]) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    for (auto e : ev_pool) hipEventDestroy(e);
    hipFree(d_csc_pos);
    hipFree(d_fresh); hipFree(d_occ); hipFree(d_lane_b); hipFree(d_lane_n); hipFree(d_ctr);
    if (h_poll) hipHostFree(h_poll);
    for (int t = 0; t < kMaxTileStreams; t++) {
        if (tstream[t]) { hipStreamSynchronize(tstream[t]); hipStreamDestroy(tstream[t]); }
        if (ev_tjoin[t]) hipEventDestroy(ev_tjoin[t]);
        for (int i = 0; i < kRing; i++)
            if (ev_tring[i][t]) hipEventDestroy(ev_tring[i][t]);
    }
    if (h_occ_t) hipHostFree(h_occ_t);
    hipFree(d_occ_t);
    hipFree(d_row_ptr); hipFree(d_col_idx); hipFree(d_col_idx_T); hipFree(d_col_ptr); hipFree(d_col_edge); hipFree(d_col_row);
    hipFree(d_unsat); hipFree(d_done); hipFree(d_fin); hipFree(d_fin_b); hipFree(d_fin_n);
    hipFree(d_sgn);
    hipFree(v2c); if (c2v != v2c) hipFree(c2v); hipFree(prior); hipFree(hard); hipFree(active); hipFree(iters); hipFree(valid);
    hipFree(post_t);
    hipFree(d_xr_jpb); hipFree(d_xr_ord4); hipFree(d_xr_inv8); hipFree(d_xr_col); hipFree(xr_msg); hipFree(xr_prior); hipFree(xr_post);
    hipFree(xr_hb); hipFree(xr_ctl); hipFree(xr_next);
    if (stream) hipStreamDestroy(stream);
    if (stream2) hipStreamDestroy(stream2);
}

template <typename T>
static int upload(T** dst, const std::vector<T>& v)
{
    const size_t n = std::max<size_t>(v.size(), 1);
    LDPC_HIP(hipMalloc((void**)dst, n * sizeof(T)));
    if (!v.empty()) LDPC_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return LDPC_OK;
}

static int64_t env_int(const char* name, int64_t dflt)
{
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoll(v) : dflt;
}

int Engine::init(const HostGraph* graph, int dev, int algorithm, int64_t chunk, int64_t group, int nt, int pipelined,
                 int csc, int cont_mode, int res_mode)
{
    g = graph;
    device = dev;
    algo = algorithm;
    if (algo < LDPC_ALGO_BP || algo > LDPC_ALGO_GALLAGER_B2) { set_error("unknown algorithm"); return LDPC_ERR_ARG; }
    const bool int_algo = algo >= LDPC_ALGO_QMSA;
    int ndev = 0;
    LDPC_HIP(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) { set_error("device ordinal out of range"); return LDPC_ERR_DEVICE; }
    LDPC_HIP(hipSetDevice(dev));
    LDPC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));

    if (nt < 0) nt = (int)env_int("LDPC_NT_D", kDefaultNT);
    const bool reg_72_8 = g->regular_dc && g->dc_max == 72 && g->regular_dv && g->dv_max == 8;
    msa_c = algo == LDPC_ALGO_MSA && reg_72_8 && nt != 0 && g->N % 16 == 0 && env_int("LDPC_MSA_C", kDefaultMsaC) != 0;
    // XCD-resident decoder: array codes (block structure found) with the
    // instantiated degrees; everything below is then only a small fallback state
    if (algo == LDPC_ALGO_BP && reg_72_8 && env_int("LDPC_XR", kDefaultXr) != 0 && (xr_layout = xr_layout_of(*g))) {
        const int rc = init_xr();
        if (rc) return rc;
        if (xr) {
            res_mode = 0;
            chunk = 64;
        }
    }
    if (cont_mode < 0) cont_mode = (int)env_int("LDPC_CONT", kDefaultCont);
    cont = cont_mode != 0 && !int_algo && reg_72_8;
    // resident pool: a few tiles whose whole state fits the
    // Infinity Cache, check->variable messages written over the variable->check
    // messages they are computed from (each row's / column's edges are read
    // into registers before its outputs are stored), no c2v scratch
    // (compressed min-sum: its own switch, LDPC_RES_MSA_C; k_var_msa_c needs N % 16)
    bool res_auto = false;  // neither the caller nor the environment chose
    if (res_mode < 0) {
        const char* ev = std::getenv(msa_c ? "LDPC_RES_MSA_C" : "LDPC_RES");
        res_auto = !(ev && *ev);
        res_mode = (int)(msa_c ? env_int("LDPC_RES_MSA_C", kDefaultResMsaC) : env_int("LDPC_RES", kDefaultRes));
    }
    res = res_mode != 0 && cont && (msa_c ? g->N % 16 == 0 : g->N % 32 == 0);  // k_var_m at any columns-per-wave
    // by default the resident pool is the Infinity-Cache-sized one: a caller's
    // explicit larger pool (the host API's chunks, the DNA batch) runs the
    // grouped schedule (A/B, 272-codeword DNA batch at cap 320: 193k -> 250k cw/s)
    if (res && res_auto && chunk > kResAutoMaxTiles * 64) res = false;
    if (res) {
        nt = 0;  // the pool is meant to stay cached
        tile_streams = (int)env_int("LDPC_RES_STREAMS", kDefaultResStreams);  // 2: staggered start, 3: re-staggered at polls
        pipelined = 0;
        csc = 0;
        res_poll = (int)std::max<int64_t>(1, env_int("LDPC_RES_POLL", kDefaultResPoll));
        res_syn_split = (int)std::max<int64_t>(0, std::min<int64_t>(env_int("LDPC_RES_SYN", kDefaultResSyn), 256));
        pp_cpw = (int)env_int("LDPC_PP_CPW", kDefaultPpCpw);
        pingpong = !msa_c && algo == LDPC_ALGO_BP && res_syn_split == 0 && !tile_streams &&
                   env_int("LDPC_PINGPONG", kDefaultPingpong) != 0 && (pp_cpw == 2 || pp_cpw == 4 || pp_cpw == 8) &&
                   g->N % (4 * pp_cpw) == 0;
    }
    if (chunk <= 0) {
        size_t fr = 0, tot = 0;
        LDPC_HIP(hipMemGetInfo(&fr, &tot));
        // half of the free memory for the resident state, at most 16384 codewords;
        // compressed min-sum in continuous mode: a small lane pool (its scattered
        // v2c stores run ~45 % longer over a 19 GB pool than over 1.2 GB, A/B)
        const int64_t want = res ? 64 * (msa_c ? env_int("LDPC_RES_TILES_MSA_C", kDefaultResTilesMsaC)
                                             : env_int("LDPC_RES_TILES", kDefaultResTiles))
                             : (msa_c && cont) ? env_int("LDPC_MSA_POOL", kDefaultMsaPool) : 16384;
        chunk = std::min<int64_t>(want, (int64_t)(fr / 2) / engine_bytes_per_codeword(*g));
    }
    cap = std::max<int64_t>(64, (chunk + 63) / 64 * 64);
    cap_tiles = cap / 64;
    if (cap_tiles > 65535) { set_error("chunk too large (max 4194240 codewords)"); return LDPC_ERR_ARG; }
    // group: tiles whose check->variable messages are live at once.  Small
    // groups keep c2v resident in the 256 MB Infinity Cache between the check
    // and the variable phase; 0 = the whole pass.
    if (res) group = 0;  // one launch per phase over the whole pool
    else if (group < 0) group = env_int("LDPC_GROUP_TILES", msa_c ? kDefaultMsaGroupTiles : kDefaultGroupTiles);
    group_tiles = (group <= 0 || group > cap_tiles) ? cap_tiles : group;
    nt_d = nt != 0;
    if (pipelined < 0) pipelined = (int)env_int("LDPC_PIPE", kDefaultPipe);
    pipe = pipelined != 0 && group_tiles < cap_tiles;
    if (pipe) {
        LDPC_HIP(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        for (int i = 0; i < 2; i++) {
            LDPC_HIP(hipEventCreateWithFlags(&ev_chk[i], hipEventDisableTiming));
            LDPC_HIP(hipEventCreateWithFlags(&ev_var[i], hipEventDisableTiming));
        }
        LDPC_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }

    int rc;
    if ((rc = upload(&d_row_ptr, g->row_ptr)) || (rc = upload(&d_col_idx, g->col_idx)) ||
        (rc = upload(&d_col_ptr, g->col_ptr)) || (rc = upload(&d_col_edge, g->col_edge)))
        return rc;
    if (msa_c) {
        std::vector<int32_t> cr(g->col_edge.size());
        for (size_t q = 0; q < cr.size(); q++) cr[q] = g->edge_row[(size_t)g->col_edge[q]];
        if ((rc = upload(&d_col_row, cr))) return rc;
    }
    if (g->regular_dc && g->dc_max > 0) {
        std::vector<int32_t> T((size_t)g->dc_max * g->M);
        for (int32_t i = 0; i < g->M; i++)
            for (int k = 0; k < g->dc_max; k++) T[(size_t)k * g->M + i] = g->col_idx[(size_t)i * g->dc_max + k];
        if ((rc = upload(&d_col_idx_T, T))) return rc;
    }
    {
        std::vector<int32_t> pos((size_t)std::max<int64_t>(g->E, 1), 0);
        for (size_t q = 0; q < g->col_edge.size(); q++) pos[(size_t)g->col_edge[q]] = (int32_t)q;
        if ((rc = upload(&d_csc_pos, pos))) return rc;
    }
    debug_no_drain = env_int("LDPC_DEBUG_NO_DRAIN", 0) != 0;
    var_cpw = (int)env_int("LDPC_VAR_CPW", kDefaultVarCpw);
    full_lanes = (int)env_int("LDPC_FULL_LANES", kDefaultFullLanes);
    if (var_cpw != 1 && var_cpw != 2 && var_cpw != 4 && var_cpw != 8) var_cpw = 1;
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
        if (tile_streams) {
            for (int t = 0; t < kMaxTileStreams; t++) {
                LDPC_HIP(hipStreamCreateWithFlags(&tstream[t], hipStreamNonBlocking));
                LDPC_HIP(hipEventCreateWithFlags(&ev_tjoin[t], hipEventDisableTiming));
                for (int i = 0; i < kRing; i++) LDPC_HIP(hipEventCreateWithFlags(&ev_tring[i][t], hipEventDisableTiming));
            }
            LDPC_HIP(hipMalloc((void**)&d_occ_t, (size_t)kRing * kMaxTileStreams * sizeof(unsigned long long)));
            LDPC_HIP(hipHostMalloc((void**)&h_occ_t, (size_t)kRing * kMaxTileStreams * sizeof(unsigned long long),
                                   hipHostMallocDefault));
        }
    }
    if (csc < 0) csc = (int)env_int("LDPC_LR_CSC", kDefaultCsc);
    lr_csc = csc != 0 && g->regular_dc && g->dc_max == 72 && g->regular_dv && g->dv_max == 8;
    // grouped continuous mode with the resident pool's fused syndrome step:
    // check(group) runs the syndrome + lane bookkeeping of its tiles (ResStep),
    // variable(group) writes the finished lanes' outputs (k_var_m / k_var_msa_c)
    syn_fused = cont && !res && !pipe && !lr_csc && g->N % 32 == 0 && env_int("LDPC_SYN_FUSED", kDefaultSynFused) != 0;
    // or a separate syndrome launch spread over several blocks per tile, same hand-off
    syn_split = (cont && !res && !syn_fused && !pipe && !lr_csc && g->N % 32 == 0)
                    ? (int)std::max<int64_t>(0, std::min<int64_t>(env_int("LDPC_SYN_SPLIT", kDefaultSynSplit), 256))
                    : 0;
    const size_t E = (size_t)std::max<int64_t>(g->E, 1);
    LDPC_HIP(hipMalloc((void**)&v2c, (size_t)cap * E * sizeof(double)));
    // continuous mode's drain tail (< 1/32 occupancy) launches wider groups
    if (res || syn_fused || syn_split) {
        LDPC_HIP(hipMalloc((void**)&d_unsat, (size_t)cap_tiles * sizeof(unsigned long long)));
        LDPC_HIP(hipMalloc((void**)&d_done, (size_t)cap_tiles * sizeof(unsigned int)));
        LDPC_HIP(hipMalloc((void**)&d_fin, (size_t)cap_tiles * sizeof(uint64_t)));
        LDPC_HIP(hipMalloc((void**)&d_fin_b, (size_t)cap * sizeof(int64_t)));
        LDPC_HIP(hipMalloc((void**)&d_fin_n, (size_t)cap * sizeof(int32_t)));
    }
    if (res) {
        c2v_tiles = cap_tiles;
        if (msa_c)  // codes + records of the whole pool (13.6 MB per tile for the DNA code)
            LDPC_HIP(hipMalloc((void**)&c2v, (size_t)cap_tiles * 64 * (E + (size_t)g->M * (dev::MSA_REC_PLANES * 8 + 4))));
        else
            c2v = v2c;  // in place
    } else {
        c2v_tiles = std::max<int64_t>((pipe ? 2 : 1) * group_tiles, cont ? (cap_tiles + 3) / 4 : 0);
        LDPC_HIP(hipMalloc((void**)&c2v, (size_t)c2v_tiles * 64 * E * sizeof(double)));
    }
    LDPC_HIP(hipMalloc((void**)&prior, (size_t)cap * g->N * sizeof(double)));
    msa_meta = msa_c && E < (size_t)dev::MSA_META_NONE && env_int("LDPC_MSA_META", kDefaultMsaMeta) != 0;
    if (msa_meta) LDPC_HIP(hipMalloc((void**)&d_sgn, (size_t)cap * g->N));
    LDPC_HIP(hipMalloc((void**)&hard, (size_t)cap_tiles * g->N * sizeof(uint64_t)));
    LDPC_HIP(hipMalloc((void**)&active, (size_t)cap_tiles * sizeof(uint64_t)));
    LDPC_HIP(hipMalloc((void**)&iters, (size_t)cap * sizeof(int32_t)));
    LDPC_HIP(hipMalloc((void**)&valid, (size_t)cap * sizeof(uint8_t)));
    const int probes = (int)env_int("LDPC_C2V_PROBE", kDefaultC2vProbe);
    if (probes > 1 && res) return probe_res(probes);
    if (probes > 1 && !int_algo && group_tiles < cap_tiles) return probe_c2v(probes);
    return LDPC_OK;
}

// Resident pool: the same placement probe for the in-place message pool
// (v2c, ~226 MB at 3 tiles, sized to the 256 MB Infinity Cache): time one
// in-place check + variable step of the whole pool on each candidate
// allocation (state zeroed, results discarded), keep the fastest.
int Engine::probe_res(int probes)
{
    const size_t E = (size_t)std::max<int64_t>(g->E, 1);
    const size_t bytes = (size_t)cap * E * sizeof(double);
    const unsigned gt = (unsigned)cap_tiles;
    LDPC_HIP(hipMemsetAsync(prior, 0, (size_t)cap * g->N * sizeof(double), stream));
    LDPC_HIP(hipMemsetAsync(active, 0xff, (size_t)cap_tiles * sizeof(uint64_t), stream));
    std::vector<double*> cand{v2c};
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
    size_t best = 0;
    float best_ms = 1e30f;
    int rc = LDPC_OK;
    // with one stream per tile the placement is judged on that schedule:
    // staggered per-tile chains of 5 steps, joined back into `stream`
    const bool ts = tile_streams && !msa_c && cap_tiles <= kMaxTileStreams;
    const size_t tsz = E * 64;
    for (size_t c = 0; ts && c < cand.size() && rc == LDPC_OK; c++) {
        v2c = c2v = cand[c];
        LDPC_HIP(hipEventRecord(e0, stream));
        for (int64_t t = 0; t < cap_tiles; t++) LDPC_HIP(hipStreamWaitEvent(tstream[t], e0, 0));
        for (int rep = 0; rep < 5 && rc == LDPC_OK; rep++)
            for (int64_t t = 0; t < cap_tiles && rc == LDPC_OK; t++) {
                if (rep == 0 && t > 0) LDPC_HIP(hipStreamWaitEvent(tstream[t], ev_tjoin[t - 1], 0));
                rc = launch_check(tstream[t], c2v + t * tsz, t, 1u);
                if (rep == 0) LDPC_HIP(hipEventRecord(ev_tjoin[t], tstream[t]));
                if (!rc) rc = launch_var(tstream[t], c2v + t * tsz, t, 1u, nullptr, dev::Refill{});
            }
        if (rc) break;
        for (int64_t t = 0; t < cap_tiles; t++) {
            LDPC_HIP(hipEventRecord(ev_tjoin[t], tstream[t]));
            LDPC_HIP(hipStreamWaitEvent(stream, ev_tjoin[t], 0));
        }
        LDPC_HIP(hipEventRecord(e1, stream));
        LDPC_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LDPC_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_ms) { best_ms = ms; best = c; }
    }
    for (size_t c = 0; !ts && c < cand.size() && rc == LDPC_OK; c++) {
        v2c = cand[c];
        if (!msa_c) c2v = v2c;
        for (int rep = 0; rep < 5 && rc == LDPC_OK; rep++) {  // rep 0 warms up
            if (rep == 1 && hipEventRecord(e0, stream) != hipSuccess) rc = LDPC_ERR_DEVICE;
            if (!rc) rc = launch_check(stream, c2v, 0, gt);  // rstep == nullptr: plain (in-place) check
            if (!rc) rc = launch_var(stream, c2v, 0, gt, nullptr, dev::Refill{});
        }
        if (rc) break;
        LDPC_HIP(hipEventRecord(e1, stream));
        LDPC_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LDPC_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_ms) { best_ms = ms; best = c; }
    }
    profile_stride = saved_stride;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    for (size_t c = 0; c < cand.size(); c++)
        if (c != best) (void)hipFree(cand[c]);
    v2c = cand[best];
    if (!msa_c) c2v = v2c;
    for (int k = 0; k < K_NCLASS; k++) launches[k] = 0;
    return rc;
}

// The check->variable scratch of one tile group (~226 MB at G = 3) is meant
// to stay in the 256 MB Infinity Cache, a memory-side cache whose slices
// belong to HBM channels: how well a given allocation fits depends on where
// its physical pages land, and identical engines were measured 3-4 % apart.
// Allocate `probes` candidate scratch buffers, time one real check+variable
// step of a tile group on each (state zeroed, results discarded -- every
// decode re-initialises), keep the fastest.
int Engine::probe_c2v(int probes)
{
    const size_t E = (size_t)std::max<int64_t>(g->E, 1);
    const size_t bytes = (size_t)c2v_tiles * 64 * E * sizeof(double);
    const unsigned gt = (unsigned)std::min<int64_t>(group_tiles, cap_tiles);
    LDPC_HIP(hipMemsetAsync(v2c, 0, (size_t)gt * 64 * E * sizeof(double), stream));
    LDPC_HIP(hipMemsetAsync(prior, 0, (size_t)gt * 64 * g->N * sizeof(double), stream));
    LDPC_HIP(hipMemsetAsync(active, 0xff, (size_t)gt * sizeof(uint64_t), stream));
    std::vector<double*> cand{c2v};
    for (int i = 1; i < probes; i++) {
        double* p = nullptr;
        if (hipMalloc((void**)&p, bytes) != hipSuccess) { (void)hipGetLastError(); break; }
        cand.push_back(p);
    }
    hipEvent_t e0, e1;
    LDPC_HIP(hipEventCreate(&e0));
    LDPC_HIP(hipEventCreate(&e1));
    const int saved_stride = profile_stride;
    profile_stride = 0;
    size_t best = 0;
    float best_ms = 1e30f;
    int rc = LDPC_OK;
    for (size_t c = 0; c < cand.size() && rc == LDPC_OK; c++) {
        for (int rep = 0; rep < 4 && rc == LDPC_OK; rep++) {  // rep 0 warms up
            if (rep == 1 && hipEventRecord(e0, stream) != hipSuccess) rc = LDPC_ERR_DEVICE;
            if (!rc) rc = launch_check(stream, cand[c], 0, gt);
            if (!rc) rc = launch_var(stream, cand[c], 0, gt, nullptr, dev::Refill{});
        }
        if (rc) break;
        LDPC_HIP(hipEventRecord(e1, stream));
        LDPC_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LDPC_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_ms) { best_ms = ms; best = c; }
    }
    profile_stride = saved_stride;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    for (size_t c = 0; c < cand.size(); c++)
        if (c != best) (void)hipFree(cand[c]);
    c2v = cand[best];
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
    if (profile_stride <= 0 || idx % profile_stride != 0) return LDPC_OK;
    sampled[c]++;
    *b = get_event();
    hipEvent_t e = get_event();
    if (!*b || !e) { set_error("hipEventCreate failed"); return LDPC_ERR_DEVICE; }
    g_ext = {*b, e};  // the launch inside LAUNCH_ON records them (klaunch)
    ext_stop = e;
    (void)s;
    return LDPC_OK;
}

int Engine::mark_end(KClass c, hipStream_t s, hipEvent_t b)
{
    LDPC_HIP(hipGetLastError());
    if (!b) return LDPC_OK;
    if (g_ext.b) {  // nothing was launched: no sample
        ev_pool.push_back(g_ext.b);
        ev_pool.push_back(g_ext.e);
        g_ext = {};
        sampled[c]--;
        return LDPC_OK;
    }
    ev_live[c].push_back({b, ext_stop});
    (void)s;
    return LDPC_OK;
}

int Engine::collect_stats()
{
    LDPC_HIP(hipSetDevice(device));
    LDPC_HIP(hipStreamSynchronize(stream));
    if (stream2) LDPC_HIP(hipStreamSynchronize(stream2));
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
    for (auto& p : wall_live) {
        float t = 0.f;
        LDPC_HIP(hipEventElapsedTime(&t, p.first, p.second));
        wall_ms += t;
        wall_runs++;
        ev_pool.push_back(p.first);
        ev_pool.push_back(p.second);
    }
    wall_live.clear();
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

// check phase of tiles t0 .. t0+gt-1 into `scratch` (that group's c2v;
// INPLACE: scratch == v2c, the resident pool)
template <bool NT, bool CSCL, bool INPLACE>
static void check_regular(int algo, hipStream_t s, dim3 grid, const double* v2c, double* scratch, const uint64_t* active,
                          const int32_t* pos, int32_t M, int64_t E, int64_t t0, int full)
{
    using namespace dev;
    if (algo == LDPC_ALGO_BP)
        klaunch((k_check_bp<72, NT, CSCL, false, INPLACE>), grid, dim3(256), 0, s, v2c, scratch, active, pos,
                           M, E, t0, full, ResStep{});
    else
        klaunch((k_check_msa<72, NT, CSCL, false, INPLACE>), grid, dim3(256), 0, s, v2c, scratch, active,
                           pos, M, E, t0, full, ResStep{});
}

template <bool NT, bool CSCL, bool CONT>
static void var_regular3(int algo, hipStream_t s, dim3 grid, const double* scratch, double* v2c, double* prior,
                         uint64_t* hard, const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N,
                         int64_t E, int64_t t0, const dev::Refill& rf)
{
    using namespace dev;
    if (algo == LDPC_ALGO_BP)
        klaunch((k_var_bp<8, NT, CSCL, CONT>), grid, dim3(256), 0, s, scratch, v2c, prior, hard, active,
                           col_edge, pt, N, E, t0, rf);
    else
        klaunch((k_var_msa<8, NT, CSCL, CONT>), grid, dim3(256), 0, s, scratch, v2c, prior, hard, active,
                           col_edge, pt, N, E, t0, rf);
}

template <bool MSA, bool NT, int CPW, bool INPLACE>
static void var_multi2(hipStream_t s, dim3 grid, const double* scratch, double* v2c, double* prior, uint64_t* hard,
                       const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N, int64_t E, int64_t t0,
                       const dev::Refill& rf, int full)
{
    using namespace dev;
    if (rf.fresh)
        klaunch((k_var_m<MSA, 8, NT, true, CPW, INPLACE>), grid, dim3(256), 0, s, scratch, v2c, prior, hard,
                           active, col_edge, pt, N, E, t0, rf, full);
    else
        klaunch((k_var_m<MSA, 8, NT, false, CPW, INPLACE>), grid, dim3(256), 0, s, scratch, v2c, prior, hard,
                           active, col_edge, pt, N, E, t0, rf, full);
}

template <bool MSA, bool NT, bool INPLACE>
static void var_multi1(int cpw, hipStream_t s, dim3 grid, const double* scratch, double* v2c, double* prior,
                       uint64_t* hard, const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N, int64_t E,
                       int64_t t0, const dev::Refill& rf, int full)
{
    if (cpw == 1) var_multi2<MSA, NT, 1, INPLACE>(s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
    else if (cpw == 2) var_multi2<MSA, NT, 2, INPLACE>(s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
    else if (cpw == 4) var_multi2<MSA, NT, 4, INPLACE>(s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
    else var_multi2<MSA, NT, 8, INPLACE>(s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
}

// inplace: scratch == v2c (the resident pool, never nontemporal)
static void var_multi(int algo, bool nt, bool inplace, int cpw, hipStream_t s, dim3 grid, const double* scratch,
                      double* v2c, double* prior, uint64_t* hard, const uint64_t* active, const int32_t* col_edge,
                      double* pt, int32_t N, int64_t E, int64_t t0, const dev::Refill& rf, int full)
{
    if (algo == LDPC_ALGO_MSA) {
        if (inplace) var_multi1<true, false, true>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
        else if (nt) var_multi1<true, true, false>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
        else var_multi1<true, false, false>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
    } else {
        if (inplace) var_multi1<false, false, true>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
        else if (nt) var_multi1<false, true, false>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
        else var_multi1<false, false, false>(cpw, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf, full);
    }
}

template <bool NT, bool CSCL>
static void var_regular(int algo, hipStream_t s, dim3 grid, const double* scratch, double* v2c, double* prior,
                        uint64_t* hard, const uint64_t* active, const int32_t* col_edge, double* pt, int32_t N,
                        int64_t E, int64_t t0, const dev::Refill& rf)
{
    if (rf.fresh) var_regular3<NT, CSCL, true>(algo, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
    else var_regular3<NT, CSCL, false>(algo, s, grid, scratch, v2c, prior, hard, active, col_edge, pt, N, E, t0, rf);
}

// MSA-C scratch: codes [c2v_tiles][E][64] u8, then records [c2v_tiles][M][4][64]
// fp64, inside the c2v allocation (13.6 MB of its 75.5 MB per tile for the
// DNA code; also with the two-slot `pipe` layout).
static uint8_t* msa_codes(double* scratch) { return reinterpret_cast<uint8_t*>(scratch); }
static double* msa_rec(double* scratch, int64_t tiles, int64_t E)
{
    return reinterpret_cast<double*>(reinterpret_cast<uint8_t*>(scratch) + (size_t)tiles * E * 64);
}

// then (msa_meta) the meta words [c2v_tiles][M][64] u32
static uint32_t* msa_meta_p(double* scratch, int64_t tiles, int64_t E, int32_t M)
{
    return reinterpret_cast<uint32_t*>(msa_rec(scratch, tiles, E) + (size_t)tiles * M * dev::MSA_REC_PLANES * 64);
}

template <bool NT, int CPW>
static void var_msa_c(hipStream_t s, unsigned nb, const uint8_t* codes, const double* rec, double* v2c, double* prior,
                      uint64_t* hard, const uint64_t* active, const int32_t* col_edge, const int32_t* col_row,
                      double* pt, int32_t N, int32_t M, int64_t E, int64_t t0, unsigned gt, const dev::Refill& rf,
                      int full, const uint32_t* meta, uint8_t* sgn)
{
    using namespace dev;
    if (rf.fresh && meta)
        klaunch((k_var_msa_c<8, NT, true, CPW, false, true>), dim3(nb), dim3(256), 0, s, codes, rec, v2c, prior, hard,
                           active, col_edge, col_row, pt, N, M, E, t0, (uint32_t)gt, rf, full, meta, sgn);
    else if (meta)
        klaunch((k_var_msa_c<8, NT, false, CPW, false, true>), dim3(nb), dim3(256), 0, s, codes, rec, v2c, prior, hard,
                           active, col_edge, col_row, pt, N, M, E, t0, (uint32_t)gt, rf, full, meta, sgn);
    else if (rf.fresh)
        klaunch((k_var_msa_c<8, NT, true, CPW>), dim3(nb), dim3(256), 0, s, codes, rec, v2c, prior, hard,
                           active, col_edge, col_row, pt, N, M, E, t0, (uint32_t)gt, rf, full, meta, sgn);
    else
        klaunch((k_var_msa_c<8, NT, false, CPW>), dim3(nb), dim3(256), 0, s, codes, rec, v2c, prior, hard,
                           active, col_edge, col_row, pt, N, M, E, t0, (uint32_t)gt, rf, full, meta, sgn);
}

int Engine::launch_check(hipStream_t s, double* scratch, int64_t t0, unsigned gt)
{
    using namespace dev;
    const int32_t M = g->M;
    const int64_t E = g->E;
    const bool reg72 = g->regular_dc && g->dc_max == 72;
    const dim3 grid((M + 3) / 4, gt), blk(256);
    // the resident pool writes the check messages over the variable messages
    const bool inplace = scratch == v2c;
    uint32_t* mmeta = msa_meta ? msa_meta_p(scratch, c2v_tiles, E, M) : nullptr;
    if (inplace && (msa_c || !reg72)) { set_error("in-place check phase needs the regular fp64 kernels"); return LDPC_ERR_ARG; }
    if ((res || syn_fused) && rstep) {  // syndrome + lane bookkeeping fused (ResStep)
        if (msa_c && nt_d)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, true, true>), grid, blk, 0, s, v2c,
                                                     msa_codes(scratch), msa_rec(scratch, c2v_tiles, E), mmeta, active, M, E,
                                                     t0, full_lanes, *rstep));
        else if (msa_c)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, false, true>), grid, blk, 0, s, v2c,
                                                     msa_codes(scratch), msa_rec(scratch, c2v_tiles, E), mmeta, active, M, E,
                                                     t0, full_lanes, *rstep));
        else if (algo == LDPC_ALGO_BP && inplace)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_bp<72, false, false, true, true>), grid, blk, 0, s, v2c,
                                                     scratch, active, d_csc_pos, M, E, t0, full_lanes, *rstep));
        else if (algo == LDPC_ALGO_BP)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_bp<72, false, false, true, false>), grid, blk, 0, s, v2c,
                                                     scratch, active, d_csc_pos, M, E, t0, full_lanes, *rstep));
        else if (inplace)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa<72, false, false, true, true>), grid, blk, 0, s, v2c,
                                                     scratch, active, d_csc_pos, M, E, t0, full_lanes, *rstep));
        else
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa<72, false, false, true, false>), grid, blk, 0, s, v2c,
                                                     scratch, active, d_csc_pos, M, E, t0, full_lanes, *rstep));
        return LDPC_OK;
    }
    if (msa_c) {
        if (nt_d)
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, true, false>), grid, blk, 0, s, v2c,
                                                     msa_codes(scratch), msa_rec(scratch, c2v_tiles, E), mmeta, active, M, E,
                                                     t0, full_lanes, ResStep{}));
        else
            LAUNCH_ON(s, K_CHECK, klaunch((k_check_msa_c<72, false, false>), grid, blk, 0, s, v2c,
                                                     msa_codes(scratch), msa_rec(scratch, c2v_tiles, E), mmeta, active, M, E,
                                                     t0, full_lanes, ResStep{}));
        return LDPC_OK;
    }
    if (reg72) {
        LAUNCH_ON(s, K_CHECK, {
            if (inplace) check_regular<false, false, true>(algo, s, grid, v2c, scratch, active, d_csc_pos, M, E, t0, full_lanes);
            else if (nt_d && lr_csc) check_regular<true, true, false>(algo, s, grid, v2c, scratch, active, d_csc_pos, M, E, t0, full_lanes);
            else if (nt_d) check_regular<true, false, false>(algo, s, grid, v2c, scratch, active, d_csc_pos, M, E, t0, full_lanes);
            else if (lr_csc) check_regular<false, true, false>(algo, s, grid, v2c, scratch, active, d_csc_pos, M, E, t0, full_lanes);
            else check_regular<false, false, false>(algo, s, grid, v2c, scratch, active, d_csc_pos, M, E, t0, full_lanes);
        });
    } else if (algo == LDPC_ALGO_BP) {
        LAUNCH_ON(s, K_CHECK, klaunch(k_check_bp_gen, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0));
    } else {
        LAUNCH_ON(s, K_CHECK, klaunch(k_check_msa_gen, grid, blk, 0, s, v2c, scratch, active, d_row_ptr, M, E, t0));
    }
    return LDPC_OK;
}

// resident BP pool, ping-pong schedule: check(tc) + variable(tv) in one launch
// (kernels.hpp k_pingpong_bp); tv < 0: check only
int Engine::launch_pingpong(hipStream_t s, int64_t tc, int64_t tv, double* pt, const dev::ResStep& rs,
                            const dev::Refill& rf)
{
    using namespace dev;
    const int32_t M = g->M, N = g->N;
    const int64_t E = g->E;
    const uint32_t nchk = (uint32_t)((M + 3) / 4);
    const uint32_t nvar = tv < 0 ? 0u : (uint32_t)(N / (4 * pp_cpw));
    const dim3 grid(nchk + nvar), blk(256);
    LAUNCH_ON(s, K_CHECK, {
        if (pp_cpw == 2)
            klaunch((k_pingpong_bp<72, 8, 2>), grid, blk, 0, s, v2c, prior, hard, active, d_col_edge, pt, M,
                               N, E, tc, tv, nchk, nvar, full_lanes, rs, rf);
        else if (pp_cpw == 8)
            klaunch((k_pingpong_bp<72, 8, 8>), grid, blk, 0, s, v2c, prior, hard, active, d_col_edge, pt, M,
                               N, E, tc, tv, nchk, nvar, full_lanes, rs, rf);
        else
            klaunch((k_pingpong_bp<72, 8, 4>), grid, blk, 0, s, v2c, prior, hard, active, d_col_edge, pt, M,
                               N, E, tc, tv, nchk, nvar, full_lanes, rs, rf);
    });
    return LDPC_OK;
}

// variable phase (+ hard decisions, optional posterior) of tiles t0 .. t0+gt-1
int Engine::launch_var(hipStream_t s, double* scratch, int64_t t0, unsigned gt, double* pt, const dev::Refill& rf)
{
    using namespace dev;
    const int32_t N = g->N;
    const int64_t E = g->E;
    const bool reg8 = g->regular_dv && g->dv_max == 8;
    const dim3 grid((N + 3) / 4, gt), blk(256);
    if (msa_c) {  // N % 16 == 0 (init)
        const int cpw = var_cpw >= 4 ? 4 : var_cpw;
        const unsigned nb = gt * (unsigned)(N / (4 * cpw));
        const uint8_t* codes = msa_codes(scratch);
        const double* rec = msa_rec(scratch, c2v_tiles, E);
        const uint32_t* mmeta = msa_meta ? msa_meta_p(scratch, c2v_tiles, E, g->M) : nullptr;
        LAUNCH_ON(s, K_VAR, {
            if (nt_d) {
                if (cpw == 1) var_msa_c<true, 1>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
                else if (cpw == 2) var_msa_c<true, 2>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
                else var_msa_c<true, 4>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
            } else {  // resident pool: keep v2c cached
                if (cpw == 1) var_msa_c<false, 1>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
                else if (cpw == 2) var_msa_c<false, 2>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
                else var_msa_c<false, 4>(s, nb, codes, rec, v2c, prior, hard, active, d_col_edge, d_col_row, pt, N, g->M, E, t0, gt, rf, full_lanes, mmeta, d_sgn);
            }
        });
        return LDPC_OK;
    }
    // (the resident pool always takes k_var_m: it writes the finished lanes'
    // outputs, and it is the only variable kernel with an in-place form)
    const bool inplace = scratch == v2c;
    const bool multi = reg8 && (res || syn_fused || syn_split || (var_cpw > 1 && nt_d)) && !lr_csc && N % (4 * var_cpw) == 0;
    if (inplace && !multi) { set_error("in-place variable phase needs k_var_m"); return LDPC_ERR_ARG; }
    if (multi) {
        const dim3 gm((unsigned)(N / (4 * var_cpw)), gt);
        LAUNCH_ON(s, K_VAR, var_multi(algo, nt_d, inplace, var_cpw, s, gm, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf, full_lanes));
        return LDPC_OK;
    }
    if (reg8) {
        // lr_csc implies both phases use the regular kernels
        LAUNCH_ON(s, K_VAR, {
            if (nt_d && lr_csc) var_regular<true, true>(algo, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
            else if (nt_d) var_regular<true, false>(algo, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
            else if (lr_csc) var_regular<false, true>(algo, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
            else var_regular<false, false>(algo, s, grid, scratch, v2c, prior, hard, active, d_col_edge, pt, N, E, t0, rf);
        });
    } else if (algo == LDPC_ALGO_BP) {
        LAUNCH_ON(s, K_VAR, klaunch(k_var_bp_gen, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt, N, E, t0));
    } else {
        LAUNCH_ON(s, K_VAR, klaunch(k_var_msa_gen, grid, blk, 0, s, scratch, v2c, prior, hard, active, d_col_ptr, d_col_edge, pt, N, E, t0));
    }
    return LDPC_OK;
}

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
                                      E, d_col_ptr, d_col_edge, prior, v2c, hard, active, iters, valid, d_sgn));
    for (int32_t n = 0;; n++) {
        if (reg_rowT && g->dc_max == 72)
            LAUNCH(K_SYN, klaunch(k_syndrome<72>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                             iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        else
            LAUNCH(K_SYN, klaunch(k_syndrome<0>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard, active,
                                             iters, valid, d_row_ptr, d_col_idx, d_col_idx_T, M, N, n, max_iter));
        if (n >= max_iter) break;
        // groups of G tiles: check(group) then variable(group); with `pipe`,
        // check(g+1) on `stream` overlaps variable(g) on `stream2` and the
        // c2v scratch is double-buffered (slot g & 1).
        const size_t slot_elems = (size_t)group_tiles * 64 * (size_t)E;
        int64_t gi = 0;
        for (int64_t t0 = 0; t0 < tiles; t0 += group_tiles, gi++) {
            const unsigned gt = (unsigned)std::min<int64_t>(group_tiles, tiles - t0);
            const int slot = pipe ? (int)(gi & 1) : 0;
            double* scratch = c2v + (size_t)slot * slot_elems;
            int rc;
            if (!pipe) {
                if ((rc = launch_check(stream, scratch, t0, gt))) return rc;
                if ((rc = launch_var(stream, scratch, t0, gt, pt, dev::Refill{}))) return rc;
                continue;
            }
            if (gi >= 2) LDPC_HIP(hipStreamWaitEvent(stream, ev_var[slot], 0));  // slot free again
            if ((rc = launch_check(stream, scratch, t0, gt))) return rc;
            LDPC_HIP(hipEventRecord(ev_chk[slot], stream));
            LDPC_HIP(hipStreamWaitEvent(stream2, ev_chk[slot], 0));
            if ((rc = launch_var(stream2, scratch, t0, gt, pt, dev::Refill{}))) return rc;
            LDPC_HIP(hipEventRecord(ev_var[slot], stream2));
        }
        if (pipe) {  // the next syndrome needs every variable phase of this iteration
            LDPC_HIP(hipEventRecord(ev_join, stream2));
            LDPC_HIP(hipStreamWaitEvent(stream, ev_join, 0));
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
                                      b_base, N, E, d_col_ptr, d_col_edge, ip, iprior, iv2c, hard, active, iters,
                                      valid));
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
        LAUNCH(K_FINAL, klaunch(k_finalize_int, g_cols_all, blk, 0, stream, post_t, iprior, iters, d_post,
                                           Bc, N));
    if (d_hard) {
        const int64_t nblk = Bc * ((N + 255) / 256);
        const unsigned grid = (unsigned)std::min<int64_t>(nblk, 1 << 20);
        LAUNCH(K_FINAL, klaunch(k_unpack_hard, dim3(grid), blk, 0, stream, hard, d_hard, Bc, N));
    }
    if (d_iters) LDPC_HIP(hipMemcpyAsync(d_iters, iters, (size_t)Bc * sizeof(int32_t), hipMemcpyDeviceToDevice, stream));
    if (d_valid) LDPC_HIP(hipMemcpyAsync(d_valid, valid, (size_t)Bc, hipMemcpyDeviceToDevice, stream));
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
    // (the XCD-resident slots pack iteration counts in 16 bits; longer decodes
    // take the engine's small tiled state)
    if (xr && max_iter <= 0xffff) return run_xr(d_in, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
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

// XCD-resident decoder (kernels_xr.hpp): probe the XCDs, then the slots'
// state (K per XCD, ~1.33 MB each for the DNA code) and the block tables.
int Engine::init_xr()
{
    int cus = 0;
    LDPC_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const int nb = 8 * std::max(cus, 1);
    unsigned* d_x = nullptr;
    LDPC_HIP(hipMalloc((void**)&d_x, (size_t)nb * sizeof(unsigned)));
    klaunch(dev::k_xr_probe, dim3(nb), dim3(64), 0, stream, d_x);
    std::vector<unsigned> hx((size_t)nb);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(hx.data(), d_x, (size_t)nb * sizeof(unsigned), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    hipFree(d_x);
    if (e != hipSuccess) { set_error(std::string("XCD probe: ") + hipGetErrorString(e)); return LDPC_ERR_DEVICE; }
    unsigned mx = 0;
    for (unsigned v : hx) mx = std::max(mx, v);
    std::vector<int> seen(mx + 1, 0);
    for (unsigned v : hx) seen[v]++;
    for (int v : seen)
        if (v == 0) return LDPC_OK;  // ids not dense: keep the tiled decoders (xr stays off)
    xr_nxcd = (int)mx + 1;
    xr_k = (int)std::max<int64_t>(1, std::min<int64_t>(env_int("LDPC_XR_K", kDefaultXrK), 64));
    xr_vb = (int)env_int("LDPC_XR_VB", kDefaultXrVb);
    if (xr_vb != 1 && xr_vb != 2) xr_vb = 4;
    xr_grid = (int)env_int("LDPC_XR_GRID", cus);
    if (xr_grid <= 0) xr_grid = cus;
    const XrLayout& L = *xr_layout;
    const size_t S = (size_t)xr_nxcd * xr_k, E = (size_t)g->E, N = (size_t)g->N;
    int rc;
    if ((rc = upload(&d_xr_jpb, L.jpb)) || (rc = upload(&d_xr_ord4, L.ord4)) || (rc = upload(&d_xr_inv8, L.inv8)) || (rc = upload(&d_xr_col, L.col_orig)))
        return rc;
    LDPC_HIP(hipMalloc((void**)&xr_msg, S * E * sizeof(double)));
    LDPC_HIP(hipMalloc((void**)&xr_prior, S * N * sizeof(double)));
    LDPC_HIP(hipMalloc((void**)&xr_hb, S * (N / 64) * sizeof(uint64_t)));
    LDPC_HIP(hipMalloc((void**)&xr_ctl, S * sizeof(dev::XrCtl)));
    LDPC_HIP(hipMalloc((void**)&xr_next, sizeof(unsigned long long)));
    xr = true;
    return LDPC_OK;
}

// One persistent launch decodes the whole batch: each XCD's workgroups run the
// check / variable tasks of that XCD's slots, each slot claiming codewords
// from the batch as it finishes one (kernels_xr.hpp).
int Engine::run_xr(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                   int post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    using namespace dev;
    if (!d_hard || !d_iters || !d_valid) { set_error("the XCD-resident decoder needs hard, iters and valid outputs"); return LDPC_ERR_ARG; }
    const int S = xr_nxcd * xr_k;
    const size_t N = (size_t)g->N;
    if (d_post && !xr_post) LDPC_HIP(hipMalloc((void**)&xr_post, (size_t)S * N * sizeof(double)));
    klaunch(k_xr_reset, dim3(1), dim3(256), 0, stream, xr_ctl, S, xr_next);
    LDPC_HIP(hipGetLastError());
    XrArgs a{};
    a.jpb = d_xr_jpb;
    a.ord4 = d_xr_ord4;
    a.inv8 = d_xr_inv8;
    a.col_orig = d_xr_col;
    a.Q = xr_layout->Q;
    a.N = g->N;
    a.E = g->E;
    a.msg = xr_msg;
    a.prior = xr_prior;
    a.post = d_post ? xr_post : nullptr;
    a.hb = xr_hb;
    a.ctl = xr_ctl;
    a.K = xr_k;
    a.nxcd = xr_nxcd;
    a.in = d_in;
    a.in_is_llr = in_kind == LDPC_IN_LLR ? 1 : 0;
    a.max_iter = max_iter;
    a.B = B;
    a.next_b = xr_next;
    a.hard_out = d_hard;
    a.post_out = d_post;
    a.post_ratio = post_kind == LDPC_POST_RATIO ? 1 : 0;
    a.iters_out = d_iters;
    a.valid_out = d_valid;
    unsigned long long* prof = nullptr;
    if (env_int("LDPC_XR_PROF", 0)) {
        LDPC_HIP(hipMalloc((void**)&prof, (size_t)xr_grid * 16 * sizeof(unsigned long long)));
        LDPC_HIP(hipMemsetAsync(prof, 0, (size_t)xr_grid * 16 * sizeof(unsigned long long), stream));
    }
    a.prof = prof;
#define XR_LAUNCH(VB, LDM) \
    LAUNCH_ON(stream, K_CHECK, klaunch((k_xr_bp<72, 8, VB, LDM>), dim3(xr_grid), dim3(256), 0, stream, a))
    const int ldm = (int)env_int("LDPC_XR_LDM", kDefaultXrLdm);
    if (xr_vb == 4 && ldm == 1) XR_LAUNCH(4, 1);
    else if (xr_vb == 4) XR_LAUNCH(4, 2);
    else if (xr_vb == 1 && ldm == 1) XR_LAUNCH(1, 1);
    else if (xr_vb == 1) XR_LAUNCH(1, 2);
    else if (ldm == 0) XR_LAUNCH(2, 0);
    else if (ldm == 1) XR_LAUNCH(2, 1);
    else XR_LAUNCH(2, 2);
#undef XR_LAUNCH
    if (prof) {  // debug: per-workgroup cycle split, summed, to stderr
        std::vector<unsigned long long> h((size_t)xr_grid * 16);
        LDPC_HIP(hipMemcpyAsync(h.data(), prof, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
        LDPC_HIP(hipStreamSynchronize(stream));
        hipFree(prof);
        unsigned long long t[16] = {0};
        for (int b = 0; b < xr_grid; b++)
            for (int q = 0; q < 16; q++) t[q] += h[(size_t)b * 16 + q];
        const double tot = (double)(t[0] + t[1] + t[3] + t[5]);
        std::fprintf(stderr,
                     "xr prof B=%lld K=%d grid=%d: claim %.3f check %.3f (%llu, %.0f cyc) var %.3f (%llu, %.0f cyc) "
                     "done+book %.3f (%llu bookkeepings); check split load %.0f compute %.0f rest %.0f cyc\n",
                     (long long)B, xr_k, xr_grid, t[0] / tot, t[1] / tot, t[2], t[2] ? (double)t[1] / t[2] : 0.0,
                     t[3] / tot, t[4], t[4] ? (double)t[3] / t[4] : 0.0, t[5] / tot, t[6],
                     t[2] ? (double)t[8] / t[2] : 0.0, t[2] ? (double)t[9] / t[2] : 0.0,
                     t[2] ? (double)(t[1] - t[8] - t[9]) / t[2] : 0.0);
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
            return LDPC_OK;
        }
        if (spin % 64 == 0) {
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

// Continuous batching over the whole batch: lanes are refilled as codewords
// finish (kernels.hpp k_syndrome_cont), so a 64-codeword tile never idles on
// its slowest member.  The host enqueues steps and stops kLag (1 for a
// single fill) steps after the device reports an empty pool (occupied lanes
// == 0 once the claim counter has passed B); the few surplus steps find no
// occupied lane.
int Engine::run_cont(const double* d_in, int in_kind, int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post,
                     int post_kind, int32_t* d_iters, uint8_t* d_valid)
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
    // lane masks, claim counter + occupancy ring, and (when allocated) the
    // syndrome words, in one launch
    static_assert(1 + kRing <= 256, "occupancy ring");
    LAUNCH(K_OTHER, klaunch(k_cont_reset, dim3((unsigned)std::min<int64_t>((tiles + 255) / 256, 1024)), dim3(256), 0,
                            stream, active, d_fresh, d_occ, d_ctr, 1 + kRing, d_unsat, d_done, tiles));
    ContState cs{active, d_fresh, d_occ, d_lane_b, d_lane_n, d_ctr, nullptr, B};
    cs.ntiles = tiles;
    const uint64_t q0 = poll_seq;  // this decode's first poll
    ContOut co{d_hard, d_post, d_iters, d_valid, post_t, prior, msa, post_kind == LDPC_POST_RATIO ? 1 : 0};
    const Refill rf{d_fresh, d_lane_b, d_in, in_kind == LDPC_IN_LLR ? 1 : 0};
    const bool reg_rowT = d_col_idx_T != nullptr;
    const int hard_vec = ((uintptr_t)d_hard % 8 == 0 && N % 8 == 0) ? 1 : 0;
    // A batch that fits the lane pool in one fill (the DNA batch) polls one
    // step behind instead of kLag: its steps take >= 30 us, time enough to
    // enqueue the next, and the decode ends one empty step sooner.
    const int lag = B <= tiles * 64 ? 1 : kLag;
    // Host step bound.  A lane finishes its codeword at most max_iter + 2
    // steps after claiming it (refill step, max_iter iterations, the final
    // syndrome), so within every window of max_iter + 2 steps each lane either
    // finishes a codeword or has found the input drained; after
    // ceil(B / lanes) + 1 windows every lane is empty.  The host reads the
    // occupancy up to kLag polls late.  A decode still running past the bound
    // means broken device bookkeeping: stop enqueueing and report it instead
    // of spinning.  LDPC_DEBUG_NO_DRAIN=1 ignores the drained reading (tests).
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
        // the occupancy is read every res_poll steps, kLag polls behind
        ResStep rs{hard, d_col_idx, d_unsat, d_done, d_fin, d_fin_b, d_fin_n, N, max_iter, cs, co};
        const Refill rfr{d_fresh, d_lane_b, d_in, in_kind == LDPC_IN_LLR ? 1 : 0, d_fin, d_fin_b, d_fin_n,
                         d_hard, d_post, post_kind == LDPC_POST_RATIO ? 1 : 0, hard_vec};
        // batches of a few pool fills (the DNA batch) poll every step: the
        // host stops at most kLag steps after the pool empties
        const int every = B <= 8 * cap ? 1 : res_poll;
        int rc = LDPC_OK;
        if (pingpong && tiles >= 2) {
            // ping-pong: step s = launches (s, t) for t = 0..tiles-1, each the
            // check of tile t and the variable phase of tile t-1 (mod tiles),
            // checked by the launch before.  The poll counter spans one whole
            // step (every tile's bookkeeping).  The decode stops kLag polls
            // after the pool drained, so the last tile's variable phase left
            // pending by the final step has no finished lane to write.
            const int64_t limit = step_limit(every);
            for (int64_t s = 0; rc == LDPC_OK; s++) {
                if (s >= limit) { rc = overrun(s); break; }
                const bool poll = (s % every) == every - 1;
                const uint64_t q = poll ? poll_seq++ : 0;
                if (poll) poll_arm(rs.cs, q);
                else rs.cs.occ_count = rs.cs.occ_clear = rs.cs.poll_host = nullptr;
                for (int64_t t = 0; t < tiles && rc == LDPC_OK; t++)
                    rc = launch_pingpong(stream, t, (s == 0 && t == 0) ? -1 : (t + tiles - 1) % tiles, pt, rs, rfr);
                if (rc) break;
                if (poll && q >= q0 + (uint64_t)lag) {
                    unsigned long long occ = 0;
                    if ((rc = poll_wait(q - lag, &occ))) break;
                    if (drained(occ)) break;
                }
            }
            return rc;
        }
        if (tile_streams && !msa_c && res_syn_split == 0 && tiles <= kMaxTileStreams) {
            // one stream per pool tile: the tiles' check/variable chains are
            // independent (lane bookkeeping, refill claims and occupancy are
            // per tile), so one tile's phase boundary overlaps the others' work
            const size_t tsz = (size_t)g->E * 64;
            hipEvent_t wb = nullptr;  // profiling: the whole concurrent decode on `stream`
            if (profile_stride > 0) {
                if (!(wb = get_event())) { set_error("hipEventCreate failed"); return LDPC_ERR_DEVICE; }
                LDPC_HIP(hipEventRecord(wb, stream));
            }
            LDPC_HIP(hipEventRecord(ev_tjoin[0], stream));  // the memsets above
            for (int64_t t = 0; t < tiles; t++) LDPC_HIP(hipStreamWaitEvent(tstream[t], ev_tjoin[0], 0));
            const int64_t limit = step_limit(every);
            for (int64_t s = 0; rc == LDPC_OK; s++) {
                if (s >= limit) { rc = overrun(s); break; }
                const bool poll = (s % every) == every - 1;
                const int64_t pi = s / every;
                const int slot = (int)(pi % kRing);
                for (int64_t t = 0; t < tiles && rc == LDPC_OK; t++) {
                    hipStream_t st = tstream[t];
                    ResStep rst = rs;
                    unsigned long long* oc = d_occ_t + (size_t)slot * kMaxTileStreams + t;
                    rst.cs.occ_count = poll ? oc : nullptr;
                    if (poll) LDPC_HIP(hipMemsetAsync(oc, 0, sizeof(unsigned long long), st));
                    // first step: tile t starts once tile t-1's first check is
                    // done, so the chains run out of phase (checks overlap
                    // variable phases instead of all tiles' checks at once)
                    // (mode 3: again at every poll step, in case the chains drifted into step)
                    const bool stag = tile_streams > 1 && (s == 0 || (tile_streams > 2 && poll));
                    if (stag && t > 0) LDPC_HIP(hipStreamWaitEvent(st, ev_tjoin[t - 1], 0));
                    rstep = &rst;
                    rc = launch_check(st, c2v + t * tsz, t, 1u);
                    rstep = nullptr;
                    if (rc) break;
                    if (stag) LDPC_HIP(hipEventRecord(ev_tjoin[t], st));
                    if (poll) {
                        LDPC_HIP(hipMemcpyAsync(h_occ_t + (size_t)slot * kMaxTileStreams + t, oc,
                                                sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
                        LDPC_HIP(hipEventRecord(ev_tring[slot][t], st));
                    }
                    rc = launch_var(st, c2v + t * tsz, t, 1u, pt, rfr);
                }
                if (rc) break;
                if (poll && pi >= lag) {
                    const int old = (int)((pi - lag) % kRing);
                    unsigned long long occ = 0;
                    for (int64_t t = 0; t < tiles; t++) {
                        LDPC_HIP(hipEventSynchronize(ev_tring[old][t]));
                        occ += h_occ_t[(size_t)old * kMaxTileStreams + t] & dev::kOccMask;
                    }
                    if (drained(occ)) break;
                }
            }
            for (int64_t t = 0; t < tiles; t++) {  // join: later work on `stream` sees every tile's last step
                LDPC_HIP(hipEventRecord(ev_tjoin[t], tstream[t]));
                LDPC_HIP(hipStreamWaitEvent(stream, ev_tjoin[t], 0));
            }
            if (wb) {
                hipEvent_t we = get_event();
                if (!we) { set_error("hipEventCreate failed"); return LDPC_ERR_DEVICE; }
                LDPC_HIP(hipEventRecord(we, stream));
                wall_live.push_back({wb, we});
            }
            return rc;
        }
        const int64_t limit = step_limit(every);
        for (int64_t s = 0; rc == LDPC_OK; s++) {
            if (s >= limit) { rc = overrun(s); break; }
            const bool poll = (s % every) == every - 1;
            const uint64_t q = poll ? poll_seq++ : 0;
            if (poll) poll_arm(rs.cs, q);
            else rs.cs.occ_count = rs.cs.occ_clear = rs.cs.poll_host = nullptr;
            if (res_syn_split > 0) {  // separate multi-block syndrome, then a plain in-place check
                LAUNCH(K_SYN, klaunch(k_syndrome_split<72>, dim3((unsigned)res_syn_split, (unsigned)tiles),
                                                 dim3(256), 0, stream, M, rs));
                rc = launch_check(stream, c2v, 0, (unsigned)tiles);
            } else {
                rstep = &rs;
                rc = launch_check(stream, c2v, 0, (unsigned)tiles);  // c2v == v2c unless MSA-C
                rstep = nullptr;
            }
            if (rc) break;
            if ((rc = launch_var(stream, c2v, 0, (unsigned)tiles, pt, rfr))) break;
            if (poll && q >= q0 + (uint64_t)lag) {
                unsigned long long occ = 0;
                if ((rc = poll_wait(q - lag, &occ))) break;
                if (drained(occ)) break;
            }
        }
        return rc;
    }
    if (syn_fused) {
        // grouped steps with the syndrome fused into each group's check
        // launch (as the resident pool); polled every step, kLag behind
        ResStep rs{hard, d_col_idx, d_unsat, d_done, d_fin, d_fin_b, d_fin_n, N, max_iter, cs, co};
        const Refill rfr{d_fresh, d_lane_b, d_in, in_kind == LDPC_IN_LLR ? 1 : 0, d_fin, d_fin_b, d_fin_n,
                         d_hard, d_post, post_kind == LDPC_POST_RATIO ? 1 : 0, hard_vec};
        bool low = false;
        const int64_t limit = step_limit(1);
        for (int64_t s = 0;; s++) {
            if (s >= limit) return overrun(s);
            const uint64_t q = poll_seq++;
            poll_arm(rs.cs, q);
            const int64_t gstep = low ? std::max(group_tiles, c2v_tiles) : group_tiles;
            for (int64_t t0 = 0; t0 < tiles; t0 += gstep) {
                const unsigned gt = (unsigned)std::min<int64_t>(gstep, tiles - t0);
                rstep = &rs;
                int rc = launch_check(stream, c2v, t0, gt);
                rstep = nullptr;
                if (rc) return rc;
                if ((rc = launch_var(stream, c2v, t0, gt, pt, rfr))) return rc;
            }
            if (q >= q0 + (uint64_t)lag) {
                unsigned long long occ = 0;
                if (int r = poll_wait(q - lag, &occ)) return r;
                if (drained(occ)) break;
                low = occ * 32 < (unsigned long long)(tiles * 64);
            }
        }
        return LDPC_OK;
    }
    // While the pool is mostly occupied, launch per tile group (c2v stays in the
    // Infinity Cache); once the input is drained and few lanes remain, one
    // check + one variable launch over all tiles per step (the tail is launch-
    // bound, and the c2v traffic is small).  `low` lags the device by kLag.
    bool low = false;
    ResStep rss{hard, d_col_idx, d_unsat, d_done, d_fin, d_fin_b, d_fin_n, N, max_iter, cs, co};
    const Refill rfs{d_fresh, d_lane_b, d_in, in_kind == LDPC_IN_LLR ? 1 : 0, d_fin, d_fin_b, d_fin_n,
                     d_hard, d_post, post_kind == LDPC_POST_RATIO ? 1 : 0, hard_vec};
    const bool split = syn_split > 0 && reg_rowT && g->dc_max == 72;
    // single fill (the DNA batch): step 0's refill stores only the prior and
    // step 1's check derives the first messages from it (k_check_bp_first),
    // instead of writing and re-reading E copies per codeword
    const bool first_fp = split && B <= tiles * 64 && algo == LDPC_ALGO_BP && !pipe && c2v != v2c &&
                          env_int("LDPC_FIRST_FROM_PRIOR", 1) != 0;
    Refill rfs0 = rfs;
    rfs0.prior_only = first_fp ? 1 : 0;
    const int64_t limit = step_limit(1);
    for (int64_t s = 0;; s++) {
        if (s >= limit) return overrun(s);
        const uint64_t q = poll_seq++;
        poll_arm(cs, q);
        poll_arm(rss.cs, q);
        if (split)
            LAUNCH(K_SYN, klaunch(k_syndrome_split<72>, dim3((unsigned)syn_split, (unsigned)tiles), dim3(256),
                                             0, stream, M, rss));
        else if (reg_rowT)
            LAUNCH(K_SYN, klaunch(k_syndrome_cont<72>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard,
                                             d_row_ptr, d_col_idx, d_col_idx_T, M, N, max_iter, cs, co));
        else
            LAUNCH(K_SYN, klaunch(k_syndrome_cont<0>, dim3((unsigned)tiles), dim3(1024), 0, stream, hard,
                                             d_row_ptr, d_col_idx, d_col_idx_T, M, N, max_iter, cs, co));

        const int64_t gstep = low ? std::max(group_tiles, c2v_tiles) : group_tiles;
        for (int64_t t0 = 0; t0 < tiles; t0 += gstep) {
            const unsigned gt = (unsigned)std::min<int64_t>(gstep, tiles - t0);
            int rc;
            if (first_fp && s == 1) {
                const dim3 grid((M + 3) / 4, gt);
                if (lr_csc)
                    LAUNCH(K_CHECK, klaunch((k_check_bp_first<72, true>), grid, dim3(256), 0, stream, prior,
                                            d_col_idx, c2v, active, d_csc_pos, M, N, (int64_t)g->E, t0, full_lanes));
                else
                    LAUNCH(K_CHECK, klaunch((k_check_bp_first<72, false>), grid, dim3(256), 0, stream, prior,
                                            d_col_idx, c2v, active, d_csc_pos, M, N, (int64_t)g->E, t0, full_lanes));
            } else if (s == 0) {
                // step 0: the reset left every lane empty and the syndrome
                // launch above only claims codewords, so no lane is active
            } else if ((rc = launch_check(stream, c2v, t0, gt))) {
                return rc;
            }
            if ((rc = launch_var(stream, c2v, t0, gt, pt, split ? (s == 0 ? rfs0 : rfs) : rf))) return rc;
        }
        if (q >= q0 + (uint64_t)lag) {
            unsigned long long occ = 0;
            if (int r = poll_wait(q - lag, &occ)) return r;
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
    LAUNCH(K_OTHER, klaunch(dev::k_gen_bsc, dim3(8192), dim3(256), 0, stream, d_out,
                                       out_kind == LDPC_IN_LR ? 1 : 0, b0, B, d_cw, n_cw, g->N, seedmix, p, pos, neg));
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
    klaunch(dev::k_pack_bits, dim3((unsigned)blocks), dim3(256), 0, stream, (const uint64_t*)d_in, d_out,
                       nbytes);
    LDPC_HIP(hipGetLastError());
    return LDPC_OK;
}

}  // namespace ldpc
