// capi.cpp -- the extern "C" boundary declared in include/ldpc_amd.h.
//
// Host side of the drop-in for ldpc.exe: graph handles (immutable, shared),
// a per-graph pool of device engines + pinned staging buffers (so repeated
// calls from decoder.py do not re-allocate), host-side exp() exactly as the
// reference (DNA_main.cpp:1344), and one host thread per GPU for multi-device
// calls -- contiguous codeword shards, no collective (the reference's dormant
// per-rank frame split, DNA_main.cpp:629-651, with its MPI_Reduce of counters,
// DNA_main.cpp:1187-1193, reduced to a host gather).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ldpc_amd.h"
#include "engine.hpp"
#include "graph.hpp"
#include "host_simd.hpp"

using ldpc::Engine;
using ldpc::HostGraph;
using ldpc::set_error;

constexpr int kMaxDevices = 64;       // opts.n_devices bound (one host thread per device)
constexpr int kMaxHostThreads = 256;  // opts.host_threads clamp
// shards up to this many codewords get a lane pool holding all of them
// (the 272-codeword DNA batch: 248k cw/s grouped vs 194k through the
// resident pool); larger ones use the engine's own pool
constexpr int64_t kExplicitPoolMax = 1024;
constexpr int64_t kXferChunk = 4096;  // codewords per PCIe chunk (at least); shards of <= kExplicitPoolMax
                                      // cross in one chunk (A/B on the DNA batch: chunks of 128 or 192
                                      // within noise of one, 64 slower)

namespace {

// Persistent host workers (one set per device context): the host-side passes
// over a chunk (exp, LLR encoding, copies) split into `n` row ranges, run by
// the workers and the calling thread, with no thread creation per call.
class Workers {
  public:
    explicit Workers(int n) : n_(std::max(1, n))
    {
        for (int t = 1; t < n_; t++) th_.emplace_back([this, t] { loop(t); });
    }
    ~Workers()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    // f(t) for t = 0..n_-1, t = 0 on the calling thread; returns when all are
    // done.  Callers on different threads take turns.
    void run(const std::function<void(int)>& f)
    {
        if (n_ == 1) { f(0); return; }
        std::lock_guard<std::mutex> turn(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            left_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int t)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
            }
            (*f)(t);
            std::lock_guard<std::mutex> lk(mu_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Code table path (DNA batches): an LLR that is an exact multiple k * unit,
// |k| <= kCodeMax, crosses PCIe as the byte k and the engine decodes the codes
// (Engine::decode_codes) with table[k + 128] = k * unit: BP's LR is the host
// libm's exp of that value -- the same bits as exp(LLR), DNA_main.cpp:1344 --
// and min-sum reads the value itself.
constexpr int kCodeMax = 127;
constexpr int kTable = 256;

// the unit: the smallest nonzero |LLR| among the chunk's first rows (a guess;
// every value is checked against it)
double llr_unit(const double* src, int64_t rows, size_t N)
{
    double u = 0;
    const size_t n = (size_t)std::min<int64_t>(rows, 4) * N;
    for (size_t i = 0; i < n; i++) {
        const double a = std::fabs(src[i]);
        if (a > 0 && std::isfinite(a) && (u == 0 || a < u)) u = a;
    }
    return u;
}

// codes of LLRs [i0, i1) (host_simd.cpp)
bool encode_rows(const double* __restrict__ src, int8_t* __restrict__ code, size_t i0, size_t i1, double unit,
                 bool msa)
{
    return ldpc::host_encode_lattice(src, code, i0, i1, unit, kCodeMax, /*keep_neg_zero=*/msa);
}

// byte x -> 8 bytes, byte r = bit r of x (unpacking the device's packed hard bits)
struct BitBytes {
    uint64_t t[256];
    BitBytes()
    {
        for (int x = 0; x < 256; x++) {
            uint64_t v = 0;
            for (int r = 0; r < 8; r++) v |= (uint64_t)((x >> r) & 1) << (8 * r);
            t[x] = v;
        }
    }
};
const BitBytes kBitBytes;

// One reusable device context for host-buffer decodes: an engine plus two
// sets of pinned / device staging buffers of `xfer` codewords each, so that
// the host-side exp and the PCIe copies of one chunk overlap the decode of
// the previous one.  The engine decodes each chunk through its lane pool
// (pool codewords, 0: its own choice -- the resident pool for BP), by
// continuous refill when the chunk is larger.
struct Slot {
    std::unique_ptr<Engine> eng;
    int device = 0, algo = 0;
    int64_t pool = 0, xfer = 0;
    ldpc_schedule sched{};  // resolved (ldpc::resolve_schedule): the engine's schedule
    hipStream_t copy = nullptr, copy_out = nullptr;  // H2D / D2H streams (the engine computes on its own)
    hipEvent_t ev_h2d[2] = {}, ev_dec[2] = {}, ev_d2h[2] = {};
    double* h_in[2] = {};
    double* h_post[2] = {};
    uint8_t* h_hard[2] = {};
    int32_t* h_iters[2] = {};
    uint8_t* h_valid[2] = {};
    double* d_in[2] = {};
    double* d_post[2] = {};
    uint8_t* d_hard[2] = {};
    int32_t* d_iters[2] = {};
    uint8_t* d_valid[2] = {};
    uint8_t* h_hbits[2] = {};  // hard bits packed 8 per byte (N % 8 == 0)
    uint8_t* d_hbits[2] = {};
    int8_t* h_code[2] = {};   // code table path: one byte per LLR
    int8_t* d_code[2] = {};
    std::vector<double> h_table[2];  // [kTable] LLR (or, BP, LR: table_kind) of code k at k + 128
    int table_kind[2] = {LDPC_IN_LLR, LDPC_IN_LLR};
    bool coded[2] = {};              // the staging buffer holds codes (else fp64 input)
    std::unique_ptr<Workers> workers;

    ~Slot()
    {
        workers.reset();
        if (eng) hipSetDevice(device);
        for (int k = 0; k < 2; k++) {
            hipHostFree(h_in[k]); hipHostFree(h_post[k]); hipHostFree(h_hard[k]); hipHostFree(h_iters[k]);
            hipHostFree(h_valid[k]); hipHostFree(h_code[k]); hipHostFree(h_hbits[k]);
            hipFree(d_in[k]); hipFree(d_post[k]); hipFree(d_hard[k]); hipFree(d_iters[k]); hipFree(d_valid[k]);
            hipFree(d_code[k]); hipFree(d_hbits[k]);
            if (ev_h2d[k]) hipEventDestroy(ev_h2d[k]);
            if (ev_dec[k]) hipEventDestroy(ev_dec[k]);
            if (ev_d2h[k]) hipEventDestroy(ev_d2h[k]);
        }
        if (copy) hipStreamDestroy(copy);
        if (copy_out) hipStreamDestroy(copy_out);
        eng.reset();
    }
    // code staging of the integer decoders (ldpc_decode_codes): on first use
    int want_codes(size_t N)
    {
        for (int k = 0; k < 2 && !h_code[k]; k++) {
            LDPC_HIP(hipHostMalloc((void**)&h_code[k], (size_t)xfer * N, hipHostMallocDefault));
            LDPC_HIP(hipMalloc((void**)&d_code[k], (size_t)xfer * N));
            h_table[k].assign(kTable, 0.0);
        }
        return LDPC_OK;
    }
    // posterior staging is allocated on the first call that asks for it
    int want_post(size_t N)
    {
        for (int k = 0; k < 2 && !h_post[k]; k++) {
            LDPC_HIP(hipHostMalloc((void**)&h_post[k], (size_t)xfer * N * sizeof(double), hipHostMallocDefault));
            LDPC_HIP(hipMalloc((void**)&d_post[k], (size_t)xfer * N * sizeof(double)));
        }
        return LDPC_OK;
    }
};

int make_slot(const HostGraph* g, int device, int algo, int64_t pool, int64_t xfer, const ldpc_schedule& sched,
              std::unique_ptr<Slot>& out)
{
    auto s = std::make_unique<Slot>();
    s->device = device;
    s->algo = algo;
    s->sched = sched;
    s->eng = std::make_unique<Engine>();
    int rc = s->eng->init(g, device, algo, pool, &sched, /*resolved=*/true);
    if (rc) return rc;
    s->pool = pool;
    s->xfer = xfer;
    const size_t N = (size_t)g->N, C = (size_t)s->xfer;
    LDPC_HIP(hipStreamCreateWithFlags(&s->copy, hipStreamNonBlocking));
    LDPC_HIP(hipStreamCreateWithFlags(&s->copy_out, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++) {
        LDPC_HIP(hipEventCreateWithFlags(&s->ev_h2d[k], hipEventDisableTiming));
        LDPC_HIP(hipEventCreateWithFlags(&s->ev_dec[k], hipEventDisableTiming));
        LDPC_HIP(hipEventCreateWithFlags(&s->ev_d2h[k], hipEventDisableTiming));
        LDPC_HIP(hipHostMalloc((void**)&s->h_in[k], C * N * sizeof(double), hipHostMallocDefault));
        LDPC_HIP(hipHostMalloc((void**)&s->h_hard[k], C * N, hipHostMallocDefault));
        LDPC_HIP(hipHostMalloc((void**)&s->h_iters[k], C * sizeof(int32_t), hipHostMallocDefault));
        LDPC_HIP(hipHostMalloc((void**)&s->h_valid[k], C, hipHostMallocDefault));
        LDPC_HIP(hipMalloc((void**)&s->d_in[k], C * N * sizeof(double)));
        LDPC_HIP(hipMalloc((void**)&s->d_hard[k], C * N));
        LDPC_HIP(hipMalloc((void**)&s->d_iters[k], C * sizeof(int32_t)));
        LDPC_HIP(hipMalloc((void**)&s->d_valid[k], C));
        if (N % 8 == 0) {
            LDPC_HIP(hipHostMalloc((void**)&s->h_hbits[k], C * N / 8, hipHostMallocDefault));
            LDPC_HIP(hipMalloc((void**)&s->d_hbits[k], C * N / 8));
        }
        if (algo == LDPC_ALGO_BP || algo == LDPC_ALGO_MSA) {
            LDPC_HIP(hipHostMalloc((void**)&s->h_code[k], C * N, hipHostMallocDefault));
            LDPC_HIP(hipMalloc((void**)&s->d_code[k], C * N));
            s->h_table[k].assign(kTable, 0.0);
        }
    }
    out = std::move(s);
    return LDPC_OK;
}

// f(r0, r1) over n rows split across the slot's workers
template <typename F>
void parallel_rows(Workers& W, int64_t n, F&& f)
{
    const int T = W.size();
    if (T == 1 || n < 2) { f(0, n); return; }
    W.run([&](int t) {
        const int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        if (r1 > r0) f(r0, r1);
    });
}

}  // namespace

struct ldpc_graph {
    HostGraph h;
    std::mutex mu;
    std::vector<std::unique_ptr<Slot>> free_slots;

    // a slot with the same lane pool (0: the engine's own) and staging for
    // at least `xfer` codewords per chunk
    // (small: any small-batch pool of at least `pool` lanes will do -- the
    // extra tiles stay empty -- so calls of varying small sizes share one)
    std::unique_ptr<Slot> take(int device, int algo, int64_t pool, int64_t xfer, bool small, const ldpc_schedule& sched)
    {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = 0; i < free_slots.size(); i++) {
            auto& s = free_slots[i];
            const bool pool_ok = small ? (s->pool >= pool && s->pool <= kExplicitPoolMax) : s->pool == pool;
            if (s->device == device && s->algo == algo && pool_ok && s->xfer >= xfer &&
                std::memcmp(&s->sched, &sched, sizeof(sched)) == 0) {
                auto r = std::move(s);
                free_slots.erase(free_slots.begin() + (long)i);
                return r;
            }
        }
        return nullptr;
    }
    void give(std::unique_ptr<Slot> s)
    {
        std::lock_guard<std::mutex> lk(mu);
        // keep at most a few idle slots per graph
        if (free_slots.size() >= 8) free_slots.erase(free_slots.begin());
        free_slots.push_back(std::move(s));
    }
};

struct ldpc_engine {
    std::unique_ptr<Engine> e;
};

static int fail(int rc, int* err)
{
    if (err) *err = rc;
    return rc;
}

extern "C" {

int ldpc_abi_version(void) { return LDPC_AMD_ABI_VERSION; }

const char* ldpc_last_error(void) { return ldpc::last_error(); }

int ldpc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

ldpc_graph* ldpc_graph_load(const char* pchk_path, int* err)
{
    if (!pchk_path) { set_error("null path"); fail(LDPC_ERR_ARG, err); return nullptr; }
    auto g = std::make_unique<ldpc_graph>();
    std::string msg;
    int rc = ldpc::load_pchk(pchk_path, g->h, &msg);
    if (rc) { set_error(msg); fail(rc, err); return nullptr; }
    if (err) *err = LDPC_OK;
    return g.release();
}

ldpc_graph* ldpc_graph_from_edges(int32_t M, int32_t N, const int32_t* rows, const int32_t* cols, int64_t n_edges,
                                  int* err)
{
    if ((!rows || !cols) && n_edges > 0) { set_error("null edge arrays"); fail(LDPC_ERR_ARG, err); return nullptr; }
    auto g = std::make_unique<ldpc_graph>();
    std::string msg;
    int rc = ldpc::build_graph(M, N, rows, cols, n_edges, g->h, &msg);
    if (rc) { set_error(msg); fail(rc, err); return nullptr; }
    if (err) *err = LDPC_OK;
    return g.release();
}

ldpc_graph* ldpc_graph_load_alist(const char* alist_path, int32_t transpose, int* err)
{
    if (!alist_path) { set_error("null path"); fail(LDPC_ERR_ARG, err); return nullptr; }
    auto g = std::make_unique<ldpc_graph>();
    std::string msg;
    int rc = ldpc::load_alist(alist_path, transpose != 0, g->h, &msg);
    if (rc) { set_error(msg); fail(rc, err); return nullptr; }
    if (err) *err = LDPC_OK;
    return g.release();
}

ldpc_graph* ldpc_graph_rs_ldpc(int32_t s, int32_t rho, int32_t gamma, int32_t* gen_poly, int32_t* coset,
                              int* err)
{
    auto g = std::make_unique<ldpc_graph>();
    std::string msg;
    std::vector<int> gp, cs;
    int rc = ldpc::build_rs_ldpc(s, rho, gamma, g->h, &gp, &cs, &msg);
    if (rc) { set_error(msg); fail(rc, err); return nullptr; }
    if (gen_poly) std::copy(gp.begin(), gp.end(), gen_poly);
    if (coset) std::copy(cs.begin(), cs.end(), coset);
    if (err) *err = LDPC_OK;
    return g.release();
}

int ldpc_graph_save_pchk(const ldpc_graph* g, const char* pchk_path)
{
    if (!g || !pchk_path) { set_error("null argument"); return LDPC_ERR_ARG; }
    std::string msg;
    int rc = ldpc::save_pchk(g->h, pchk_path, &msg);
    if (rc) set_error(msg);
    return rc;
}

int ldpc_graph_save_alist(const ldpc_graph* g, const char* alist_path)
{
    if (!g || !alist_path) { set_error("null argument"); return LDPC_ERR_ARG; }
    std::string msg;
    int rc = ldpc::save_alist(g->h, alist_path, &msg);
    if (rc) set_error(msg);
    return rc;
}

void ldpc_graph_free(ldpc_graph* g) { delete g; }

int ldpc_graph_info(const ldpc_graph* g, int32_t* M, int32_t* N, int64_t* E, int32_t* dv_max, int32_t* regular_dv,
                    int32_t* dc_max, int32_t* regular_dc)
{
    if (!g) { set_error("null graph"); return LDPC_ERR_ARG; }
    if (M) *M = g->h.M;
    if (N) *N = g->h.N;
    if (E) *E = g->h.E;
    if (dv_max) *dv_max = g->h.dv_max;
    if (regular_dv) *regular_dv = g->h.regular_dv;
    if (dc_max) *dc_max = g->h.dc_max;
    if (regular_dc) *regular_dc = g->h.regular_dc;
    return LDPC_OK;
}

int ldpc_graph_blocks(const ldpc_graph* g, int32_t* Q, int32_t* row_blocks, int32_t* col_blocks, int32_t* col_block)
{
    if (!g) { set_error("null graph"); return LDPC_ERR_ARG; }
    const ldpc::BlockLayout* L = ldpc::block_layout_of(g->h);
    if (Q) *Q = L ? L->Q : 0;
    if (row_blocks) *row_blocks = L ? L->GA : 0;
    if (col_blocks) *col_blocks = L ? L->RB : 0;
    if (L && col_block)
        for (size_t q = 0; q < L->col_orig.size(); q++) col_block[L->col_orig[q]] = (int32_t)(q / (size_t)L->Q);
    return LDPC_OK;
}

int ldpc_graph_edges(const ldpc_graph* g, int32_t* row_ptr, int32_t* col_idx, int32_t* col_ptr, int32_t* col_edge)
{
    if (!g) { set_error("null graph"); return LDPC_ERR_ARG; }
    const auto& h = g->h;
    if (row_ptr) std::memcpy(row_ptr, h.row_ptr.data(), h.row_ptr.size() * 4);
    if (col_idx) std::memcpy(col_idx, h.col_idx.data(), h.col_idx.size() * 4);
    if (col_ptr) std::memcpy(col_ptr, h.col_ptr.data(), h.col_ptr.size() * 4);
    if (col_edge) std::memcpy(col_edge, h.col_edge.data(), h.col_edge.size() * 4);
    return LDPC_OK;
}

int ldpc_graph_syndrome(const ldpc_graph* g, const uint8_t* dblk, uint8_t* pchk)
{
    if (!g || !dblk) { set_error("null argument"); return LDPC_ERR_ARG; }
    return ldpc::syndrome_host(g->h, dblk, pchk);
}

// The channel input of a host-buffer decode: fp64 LLRs (ldpc_decode) or int8
// codes with their 256-entry table (ldpc_decode_codes).
struct HostInput {
    const double* llr = nullptr;
    const int8_t* codes = nullptr;
    const double* table = nullptr;
    int table_kind = LDPC_IN_LLR;
};

static int host_decode(const ldpc_graph* gc, const HostInput& in, int64_t B, int32_t max_iter, int32_t algo,
                       uint8_t* hard_out, double* post_out, int32_t* iters_out, uint8_t* valid_out,
                       const ldpc_opts* opts)
{
    ldpc_graph* g = const_cast<ldpc_graph*>(gc);
    const double* llr = in.llr;
    if (!g) { set_error("null graph"); return LDPC_ERR_ARG; }
    if (B < 0 || max_iter < 0) { set_error("B and max_iter must be >= 0"); return LDPC_ERR_ARG; }
    if (B > 0 && ((!llr && !in.codes) || !hard_out)) { set_error("the channel input and hard_out are required"); return LDPC_ERR_ARG; }
    if (in.codes && !in.table) { set_error("ldpc_decode_codes: null table"); return LDPC_ERR_ARG; }
    if (in.codes && in.table_kind != LDPC_IN_LLR && !(in.table_kind == LDPC_IN_LR && algo == LDPC_ALGO_BP)) {
        set_error("table kind: LDPC_IN_LLR, or LDPC_IN_LR for BP");
        return LDPC_ERR_ARG;
    }
    if (algo < LDPC_ALGO_BP || algo > LDPC_ALGO_GALLAGER_B2) { set_error("unknown algorithm"); return LDPC_ERR_ARG; }
    ldpc_opts o{};
    o.exp_on_host = 1;
    if (opts) o = *opts;
    // quantized min-sum parameters: 0 selects the engine defaults (q 6, step 0.5)
    const int32_t q_prec = o.msa_precision > 0 ? o.msa_precision : 6;
    const double q_step = o.msa_step > 0 ? o.msa_step : 0.5;
    if (algo == LDPC_ALGO_QMSA && (q_prec < 2 || q_prec > 16 || o.msa_offset < 0)) {
        set_error("quantized min-sum needs 2 <= msa_precision <= 16 and msa_offset >= 0");
        return LDPC_ERR_ARG;
    }
    if (algo != LDPC_ALGO_BP && post_out && o.post_kind == LDPC_POST_RATIO) {
        set_error("LDPC_POST_RATIO is BP-only");
        return LDPC_ERR_ARG;
    }
    // B [B][N] fp64 values must be addressable (the host code forms B * N * 8)
    if (B > (int64_t)(PTRDIFF_MAX / 8) / (int64_t)std::max<int32_t>(1, g->h.N)) {
        set_error("batch too large: B * N * 8 bytes overflow the address space");
        return LDPC_ERR_ARG;
    }
    if (o.n_devices > kMaxDevices) {
        set_error("opts.n_devices above " + std::to_string(kMaxDevices));
        return LDPC_ERR_ARG;
    }
    if (B == 0) return LDPC_OK;

    std::vector<int> devs;
    const int ndev = std::max(1, (int)o.n_devices);
    for (int i = 0; i < ndev; i++) {
        devs.push_back(o.devices ? o.devices[i] : i);
        if (devs.back() < 0) { set_error("negative device ordinal"); return LDPC_ERR_ARG; }
    }
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    // host threads for exp / packing: the caller's count, clamped (each is an
    // OS thread of this call's worker pool)
    const int host_threads = o.host_threads > 0 ? std::min(o.host_threads, kMaxHostThreads)
                                                : std::min(16, std::max(1, hw / ndev));
    const ldpc_schedule sched = ldpc::resolve_schedule(o.schedule);
    const bool lr_table = ldpc::sched_flag(sched, LDPC_SCHED_LR_TABLE);
    // the only environment variable the library reads: a debug print of the
    // host-leg split (never changes what is computed)
    const char* pev = std::getenv("LDPC_API_TIMING");
    const bool api_timing = pev && *pev && std::atoi(pev) != 0;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const size_t N = (size_t)g->h.N;

    // codes in pinned host memory (ldpc_host_alloc / hipHostMalloc: mapped
    // for every device) cross PCIe straight from the caller's array; the
    // tested case is ldpc_host_alloc memory
    bool codes_pinned = false;
    if (in.codes) {
        hipPointerAttribute_t a0{}, a1{};
        codes_pinned = hipPointerGetAttributes(&a0, in.codes) == hipSuccess && a0.type == hipMemoryTypeHost &&
                       hipPointerGetAttributes(&a1, in.codes + (size_t)B * N - 1) == hipSuccess &&
                       a1.type == hipMemoryTypeHost;
        (void)hipGetLastError();  // pageable memory: the attribute query's error is not sticky
    }
    std::vector<int> rcs(devs.size(), LDPC_OK);
    std::vector<std::string> msgs(devs.size());
    auto work = [&](size_t di) {
        const int dev = devs[di];
        const int64_t s0 = B * (int64_t)di / (int64_t)devs.size();
        const int64_t s1 = B * (int64_t)(di + 1) / (int64_t)devs.size();
        const int64_t shard = s1 - s0;
        if (shard <= 0) return;
        // lane pool: the caller's chunk; else for small shards (the DNA batch)
        // one holding all of them (every codeword in flight at once), else the
        // engine's own (0: the resident pool for BP).  Codewords move through
        // PCIe in double-buffered chunks of `xfer`.
        const int64_t sh64 = (shard + 63) / 64 * 64;
        const int64_t pool = o.chunk > 0 ? o.chunk : (shard <= kExplicitPoolMax ? sh64 : 0);
        const int64_t xfer = std::min<int64_t>(sh64, std::max<int64_t>(kXferChunk, (pool + 63) / 64 * 64));
        std::unique_ptr<Slot> slot = g->take(dev, algo, pool, xfer, o.chunk <= 0 && pool > 0, sched);
        int rc = LDPC_OK;
        if (!slot) rc = make_slot(&g->h, dev, algo, pool, xfer, sched, slot);
        if (!rc && post_out) rc = slot->want_post(N);
        if (!rc && in.codes) rc = slot->want_codes(N);
        if (rc) { rcs[di] = rc; msgs[di] = ldpc::last_error(); return; }
        if (!slot->workers || slot->workers->size() != host_threads) slot->workers = std::make_unique<Workers>(host_threads);
        Slot& S = *slot;
        Workers& W = *S.workers;
        Engine& E = *S.eng;
        const bool host_exp = (algo == LDPC_ALGO_BP) && o.exp_on_host;
        const int in_kind = (algo == LDPC_ALGO_BP && host_exp) ? LDPC_IN_LR : LDPC_IN_LLR;
        const int64_t X = xfer, nch = (shard + X - 1) / X;  // (the slot's staging holds >= xfer)
        auto c0 = [&](int64_t c) { return s0 + c * X; };
        auto cn = [&](int64_t c) { return std::min<int64_t>(X, s1 - c0(c)); };
        // host side of chunk c: exp (DNA_main.cpp:1344  g_received_LR[i] =
        // exp(g_received_LLR[i])) or copy into pinned staging, then H2D on the
        // copy stream once the decode that last read that device buffer is done
        auto prep = [&](int64_t c) -> int {
            const int k = (int)(c & 1);
            const int64_t Bc = cn(c);
            LDPC_HIP(hipSetDevice(dev));
            if (c >= 2) LDPC_HIP(hipEventSynchronize(S.ev_h2d[k]));  // staging buffer free again
            const double tp0 = api_timing ? now() : 0;
            if (in.codes) {
                // the caller's codes: into pinned staging and across PCIe in
                // pieces (each crossing while the next is copied)
                const int8_t* src = in.codes + (size_t)c0(c) * N;
                if (c >= 2) LDPC_HIP(hipStreamWaitEvent(S.copy, S.ev_dec[k], 0));
                const int64_t pieces = codes_pinned ? 0 : std::min<int64_t>(4, Bc);
                if (codes_pinned)
                    LDPC_HIP(hipMemcpyAsync(S.d_code[k], src, (size_t)Bc * N, hipMemcpyHostToDevice, S.copy));
                for (int64_t pc = 0; pc < pieces; pc++) {
                    const int64_t p0 = Bc * pc / pieces, p1 = Bc * (pc + 1) / pieces;
                    parallel_rows(W, p1 - p0, [&](int64_t r0, int64_t r1) {
                        std::memcpy(S.h_code[k] + (size_t)(p0 + r0) * N, src + (size_t)(p0 + r0) * N,
                                    (size_t)(r1 - r0) * N);
                    });
                    LDPC_HIP(hipMemcpyAsync(S.d_code[k] + (size_t)p0 * N, S.h_code[k] + (size_t)p0 * N,
                                            (size_t)(p1 - p0) * N, hipMemcpyHostToDevice, S.copy));
                }
                std::copy(in.table, in.table + kTable, S.h_table[k].begin());
                S.table_kind[k] = in.table_kind;
                S.coded[k] = true;
                const double tp1 = api_timing ? now() : 0;
                LDPC_HIP(hipEventRecord(S.ev_h2d[k], S.copy));
                if (api_timing) {
                    LDPC_HIP(hipEventSynchronize(S.ev_h2d[k]));
                    std::fprintf(stderr, "api chunk %lld: codes copy %.3f ms, + H2D %.3f ms\n", (long long)c,
                                 tp1 - tp0, now() - tp1);
                }
                return LDPC_OK;
            }
            const double* src = llr + (size_t)c0(c) * N;
            // code table path: all of the chunk's LLRs exact multiples of one unit
            bool coded = false;
            if ((host_exp || algo == LDPC_ALGO_MSA) && lr_table && S.h_code[k]) {
                const double unit = llr_unit(src, Bc, N);
                if (unit > 0) {
                    // in pieces, each crossing PCIe while the next is encoded
                    if (c >= 2) LDPC_HIP(hipStreamWaitEvent(S.copy, S.ev_dec[k], 0));
                    const int64_t pieces = std::min<int64_t>(4, Bc);
                    std::atomic<bool> ok{true};
                    for (int64_t pc = 0; pc < pieces && ok; pc++) {
                        const int64_t p0 = Bc * pc / pieces, p1 = Bc * (pc + 1) / pieces;
                        parallel_rows(W, p1 - p0, [&](int64_t r0, int64_t r1) {
                            if (!encode_rows(src, S.h_code[k], (size_t)(p0 + r0) * N, (size_t)(p0 + r1) * N, unit,
                                             algo == LDPC_ALGO_MSA))
                                ok = false;
                        });
                        if (ok)
                            LDPC_HIP(hipMemcpyAsync(S.d_code[k] + (size_t)p0 * N, S.h_code[k] + (size_t)p0 * N,
                                                    (size_t)(p1 - p0) * N, hipMemcpyHostToDevice, S.copy));
                    }
                    if (ok) {
                        for (int q = -kCodeMax; q <= kCodeMax; q++) S.h_table[k][q + 128] = (double)q * unit;
                        S.table_kind[k] = LDPC_IN_LLR;
                        coded = true;
                    }
                }
            }
            if (!coded) {
                if (host_exp)
                    parallel_rows(W, Bc, [&](int64_t r0, int64_t r1) {
                        for (size_t i = (size_t)r0 * N; i < (size_t)r1 * N; i++) S.h_in[k][i] = std::exp(src[i]);
                    });
                else
                    parallel_rows(W, Bc, [&](int64_t r0, int64_t r1) {
                        std::memcpy(S.h_in[k] + (size_t)r0 * N, src + (size_t)r0 * N, (size_t)(r1 - r0) * N * 8);
                    });
            }
            const double tp1 = api_timing ? now() : 0;
            if (c >= 2) LDPC_HIP(hipStreamWaitEvent(S.copy, S.ev_dec[k], 0));
            S.coded[k] = coded;
            if (!coded) {  // (codes are on their way already; their table goes with the decode)
                LDPC_HIP(hipMemcpyAsync(S.d_in[k], S.h_in[k], (size_t)Bc * N * 8, hipMemcpyHostToDevice, S.copy));
            }
            LDPC_HIP(hipEventRecord(S.ev_h2d[k], S.copy));
            if (api_timing) {
                LDPC_HIP(hipEventSynchronize(S.ev_h2d[k]));
                std::fprintf(stderr, "api chunk %lld: %s %.3f ms, + H2D %.3f ms\n", (long long)c,
                             coded ? "encode" : "exp/copy", tp1 - tp0, now() - tp1);
            }
            return LDPC_OK;
        };
        // outputs of chunk c, once its D2H copies are done
        auto finish = [&](int64_t c) -> int {
            const int k = (int)(c & 1);
            const int64_t b0 = c0(c), Bc = cn(c);
            const double tf0 = api_timing ? now() : 0;
            LDPC_HIP(hipEventSynchronize(S.ev_d2h[k]));
            const double tf1 = api_timing ? now() : 0;
            parallel_rows(W, Bc, [&](int64_t r0, int64_t r1) {
                if (S.h_hbits[k]) {  // packed: 8 hard bits per byte
                    uint64_t* o = reinterpret_cast<uint64_t*>(hard_out + (size_t)(b0 + r0) * N);
                    const uint8_t* in = S.h_hbits[k] + (size_t)r0 * N / 8;
                    const size_t nb = (size_t)(r1 - r0) * N / 8;
                    if (((uintptr_t)o & 7) == 0)
                        for (size_t q = 0; q < nb; q++) o[q] = kBitBytes.t[in[q]];
                    else
                        for (size_t q = 0; q < nb; q++) std::memcpy((uint8_t*)o + 8 * q, &kBitBytes.t[in[q]], 8);
                } else {
                    std::memcpy(hard_out + (size_t)(b0 + r0) * N, S.h_hard[k] + (size_t)r0 * N, (size_t)(r1 - r0) * N);
                }
                if (post_out)
                    std::memcpy(post_out + (size_t)(b0 + r0) * N, S.h_post[k] + (size_t)r0 * N, (size_t)(r1 - r0) * N * 8);
            });
            if (iters_out) std::memcpy(iters_out + b0, S.h_iters[k], (size_t)Bc * 4);
            if (valid_out) std::memcpy(valid_out + b0, S.h_valid[k], (size_t)Bc);
            if (api_timing)
                std::fprintf(stderr, "api chunk %lld: wait decode + D2H %.3f ms, copy out %.3f ms\n", (long long)c,
                             tf1 - tf0, now() - tf1);
            return LDPC_OK;
        };
        auto decode = [&](int64_t c) -> int {
            const int k = (int)(c & 1);
            const int64_t Bc = cn(c);
            LDPC_HIP(hipSetDevice(dev));
            if (algo == LDPC_ALGO_QMSA) {
                int r = E.set_params(q_prec, q_step, o.msa_offset, o.tie_seed);
                if (r) return r;
            }
            E.tie_base = c0(c);  // tie hash keyed by the codeword's index in this call
            LDPC_HIP(hipStreamWaitEvent(E.stream, S.ev_h2d[k], 0));
            const double td0 = api_timing ? now() : 0;
            int r = S.coded[k] ? E.decode_codes(S.d_code[k], S.h_table[k].data(), S.table_kind[k], Bc, max_iter, S.d_hard[k],
                                                post_out ? S.d_post[k] : nullptr, o.post_kind, S.d_iters[k], S.d_valid[k],
                                                S.d_in[k])
                               : E.decode(S.d_in[k], in_kind, Bc, max_iter, S.d_hard[k],
                                          post_out ? S.d_post[k] : nullptr, o.post_kind, S.d_iters[k], S.d_valid[k]);
            if (r) return r;
            if (api_timing)
                std::fprintf(stderr, "api chunk %lld: decode enqueue + drain wait %.3f ms\n", (long long)c, now() - td0);
            LDPC_HIP(hipEventRecord(S.ev_dec[k], E.stream));
            LDPC_HIP(hipStreamWaitEvent(S.copy_out, S.ev_dec[k], 0));
            if (S.d_hbits[k]) {  // 1/8 of the bytes across PCIe
                r = E.pack_bits(S.d_hard[k], S.d_hbits[k], Bc * (int64_t)N / 8);
                if (r) return r;
                LDPC_HIP(hipEventRecord(S.ev_dec[k], E.stream));
                LDPC_HIP(hipStreamWaitEvent(S.copy_out, S.ev_dec[k], 0));
                LDPC_HIP(hipMemcpyAsync(S.h_hbits[k], S.d_hbits[k], (size_t)Bc * N / 8, hipMemcpyDeviceToHost,
                                        S.copy_out));
            } else {
                LDPC_HIP(hipMemcpyAsync(S.h_hard[k], S.d_hard[k], (size_t)Bc * N, hipMemcpyDeviceToHost, S.copy_out));
            }
            if (post_out)
                LDPC_HIP(hipMemcpyAsync(S.h_post[k], S.d_post[k], (size_t)Bc * N * 8, hipMemcpyDeviceToHost,
                                        S.copy_out));
            LDPC_HIP(hipMemcpyAsync(S.h_iters[k], S.d_iters[k], (size_t)Bc * 4, hipMemcpyDeviceToHost, S.copy_out));
            LDPC_HIP(hipMemcpyAsync(S.h_valid[k], S.d_valid[k], (size_t)Bc, hipMemcpyDeviceToHost, S.copy_out));
            LDPC_HIP(hipEventRecord(S.ev_d2h[k], S.copy_out));
            return LDPC_OK;
        };
        const double t_call = api_timing ? now() : 0;
        rc = prep(0);
        for (int64_t c = 0; c < nch && rc == LDPC_OK; c++) {
            // the next chunk's host work and H2D run on a helper thread while
            // this thread drives the decode of chunk c
            int rc_next = LDPC_OK;
            std::string err_next;
            std::thread next;
            if (c + 1 < nch)
                next = std::thread([&, c] {
                    rc_next = prep(c + 1);
                    if (rc_next) err_next = ldpc::last_error();
                });
            rc = decode(c);
            if (rc == LDPC_OK && c >= 1) rc = finish(c - 1);
            if (next.joinable()) next.join();
            if (rc == LDPC_OK && rc_next) { rc = rc_next; set_error(err_next); }
        }
        if (rc == LDPC_OK) rc = finish(nch - 1);
        if (api_timing) std::fprintf(stderr, "api shard %zu: %.3f ms\n", di, now() - t_call);
        if (rc == LDPC_OK) rc = E.sync();  // surplus steps of the last decode; a device fault report
        if (rc) { rcs[di] = rc; msgs[di] = ldpc::last_error(); return; }
        g->give(std::move(slot));
    };
    if (devs.size() == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (size_t i = 0; i < devs.size(); i++) th.emplace_back(work, i);
        for (auto& t : th) t.join();
    }
    for (size_t i = 0; i < devs.size(); i++)
        if (rcs[i]) { set_error("device " + std::to_string(devs[i]) + ": " + msgs[i]); return rcs[i]; }
    return LDPC_OK;
}

int ldpc_decode(const ldpc_graph* g, const double* llr, int64_t B, int32_t max_iter, int32_t algo, uint8_t* hard_out,
                double* post_out, int32_t* iters_out, uint8_t* valid_out, const ldpc_opts* opts)
{
    HostInput in;
    in.llr = llr;
    return host_decode(g, in, B, max_iter, algo, hard_out, post_out, iters_out, valid_out, opts);
}

int ldpc_decode_codes(const ldpc_graph* g, const int8_t* codes, const double* table, int32_t table_kind, int64_t B,
                      int32_t max_iter, int32_t algo, uint8_t* hard_out, double* post_out, int32_t* iters_out,
                      uint8_t* valid_out, const ldpc_opts* opts)
{
    HostInput in;
    in.codes = codes;
    in.table = table;
    in.table_kind = table_kind;
    if (B > 0 && !codes) { set_error("null codes"); return LDPC_ERR_ARG; }
    return host_decode(g, in, B, max_iter, algo, hard_out, post_out, iters_out, valid_out, opts);
}

int ldpc_engine_set_params(ldpc_engine* e, int32_t msa_precision, double msa_step, int32_t msa_offset,
                           uint64_t tie_seed)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    return e->e->set_params(msa_precision, msa_step, msa_offset, tie_seed);
}

ldpc_engine* ldpc_engine_create_ex(const ldpc_graph* g, int32_t device, int32_t algo, int64_t chunk,
                                   const ldpc_schedule* schedule, int* err)
{
    if (!g) { set_error("null graph"); fail(LDPC_ERR_ARG, err); return nullptr; }
    auto e = std::make_unique<ldpc_engine>();
    e->e = std::make_unique<Engine>();
    int rc = e->e->init(&g->h, device, algo, chunk, schedule);
    if (rc) { fail(rc, err); return nullptr; }
    if (err) *err = LDPC_OK;
    return e.release();
}

ldpc_engine* ldpc_engine_create(const ldpc_graph* g, int32_t device, int32_t algo, int64_t chunk, int* err)
{
    return ldpc_engine_create_ex(g, device, algo, chunk, nullptr, err);
}

int ldpc_engine_info(ldpc_engine* e, int64_t* cap, int64_t* group_tiles, int32_t* flags)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    if (cap) *cap = e->e->cap;
    if (group_tiles) *group_tiles = e->e->group_tiles;
    if (flags) *flags = e->e->flags();
    return LDPC_OK;
}

void ldpc_engine_free(ldpc_engine* e) { delete e; }

int ldpc_engine_decode(ldpc_engine* e, const double* d_in, int32_t in_kind, int64_t B, int32_t max_iter,
                       uint8_t* d_hard, double* d_post, int32_t post_kind, int32_t* d_iters, uint8_t* d_valid)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    if (B > 0 && !d_in) { set_error("null input"); return LDPC_ERR_ARG; }
    return e->e->decode(d_in, in_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
}

int ldpc_engine_decode_codes(ldpc_engine* e, const int8_t* d_codes, const double* table, int32_t table_kind,
                             int64_t B, int32_t max_iter, uint8_t* d_hard, double* d_post, int32_t post_kind,
                             int32_t* d_iters, uint8_t* d_valid)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    return e->e->decode_codes(d_codes, table, table_kind, B, max_iter, d_hard, d_post, post_kind, d_iters, d_valid);
}

int ldpc_engine_sync(ldpc_engine* e)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    return e->e->sync();
}

void* ldpc_engine_stream(ldpc_engine* e) { return e ? (void*)e->e->stream : nullptr; }

int ldpc_engine_gen_bsc(ldpc_engine* e, double* d_out, int32_t out_kind, int64_t b0, int64_t B,
                        const uint8_t* d_codewords, int32_t n_cw, uint64_t seed, double p, double llr_mag)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    return e->e->gen_bsc(d_out, out_kind, b0, B, d_codewords, n_cw, seed, p, llr_mag);
}

int ldpc_engine_gen_bsc_codes(ldpc_engine* e, int8_t* d_out, int64_t b0, int64_t B, const uint8_t* d_codewords,
                              int32_t n_cw, uint64_t seed, double p)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    return e->e->gen_bsc_codes(d_out, b0, B, d_codewords, n_cw, seed, p);
}

int ldpc_engine_profile(ldpc_engine* e, int32_t stride)
{
    if (!e) { set_error("null engine"); return LDPC_ERR_ARG; }
    int rc = e->e->collect_stats();
    if (rc) return rc;
    for (int c = 0; c < ldpc::K_NCLASS; c++) { e->e->launches[c] = 0; e->e->ms[c] = 0; e->e->sampled[c] = 0; }
    e->e->profile_stride = stride > 0 ? stride : 0;
    return LDPC_OK;
}

int ldpc_engine_stats(ldpc_engine* e, ldpc_kernel_stats* out)
{
    if (!e || !out) { set_error("null argument"); return LDPC_ERR_ARG; }
    int rc = e->e->collect_stats();
    if (rc) return rc;
    std::memset(out, 0, sizeof(*out));
    for (int c = 0; c < ldpc::K_NCLASS; c++) {
        out->launches[c] = e->e->launches[c];
        out->sampled[c] = e->e->sampled[c];
        out->ms[c] = e->e->ms[c];
    }
    return LDPC_OK;
}

void* ldpc_host_alloc(size_t bytes)
{
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) { set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e)); return nullptr; }
    return p;
}

int ldpc_host_free(void* p)
{
    if (p) LDPC_HIP(hipHostFree(p));
    return LDPC_OK;
}

void* ldpc_dev_malloc(int32_t device, size_t bytes)
{
    void* p = nullptr;
    if (hipSetDevice(device) != hipSuccess) { set_error("hipSetDevice failed"); return nullptr; }
    hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 1));
    if (e != hipSuccess) { set_error(std::string("hipMalloc: ") + hipGetErrorString(e)); return nullptr; }
    return p;
}

int ldpc_dev_free(int32_t device, void* p)
{
    LDPC_HIP(hipSetDevice(device));
    LDPC_HIP(hipFree(p));
    return LDPC_OK;
}

int ldpc_dev_memcpy(int32_t device, void* dst, const void* src, size_t bytes, int32_t kind)
{
    hipMemcpyKind k = kind == LDPC_H2D ? hipMemcpyHostToDevice : kind == LDPC_D2H ? hipMemcpyDeviceToHost
                                                                                   : hipMemcpyDeviceToDevice;
    LDPC_HIP(hipSetDevice(device));
    LDPC_HIP(hipMemcpy(dst, src, bytes, k));
    return LDPC_OK;
}

}  // extern "C"
