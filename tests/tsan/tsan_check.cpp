// tsan_check.cpp -- TEST INFRASTRUCTURE: race detection on the C ABI's host
// side.  Linked against tests/tsan/build/
// libldpc_amd_tsan.so -- every host unit of lib/libldpc_amd.so under
// ThreadSanitizer (hipcc -Xarch_host -fsanitize=thread), the gfx950 device
// code as usual -- and run on an MI355X by tests/test_tsan_gpu.py.
//
// The threading contract (include/ldpc_amd.h): a graph is
// shareable, calls are reentrant, errors are per thread.  Eight threads at
// once, two rounds each, on ONE graph:
//   0, 1  ldpc_decode BP (host exp; one with posteriors), different batches
//   2     ldpc_decode min-sum
//   3     ldpc_decode_codes (int8 codes + table)
//   4, 5  4160 codewords each (BP fp64, min-sum codes): two PCIe chunks, so
//         the helper thread that prepares the next chunk runs too
//   6     the device-resident engine: create, gen_bsc on device, decode, sync
//   7     graph loads that fail and succeed, host syndromes, error strings
// plus one call with two shards on device 0 (the per-device worker threads).
// Every decode result must equal the same call made alone first.  A race is
// a ThreadSanitizer report (the test fails on it); a wrong result prints
// MISMATCH and exits 3.
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ldpc_amd.h"

namespace {

std::atomic<int> g_bad{0};

void fail(const std::string& what)
{
    std::printf("MISMATCH %s (%s)\n", what.c_str(), ldpc_last_error());
    g_bad = 1;
}

uint64_t mix(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// BSC(p) LLRs around the all-zero codeword (a codeword of every linear code)
std::vector<double> bsc(int64_t B, int64_t N, double p, uint64_t seed)
{
    const double mag = std::log((1 - p) / p);
    std::vector<double> v((size_t)(B * N));
    for (size_t i = 0; i < v.size(); i++) v[i] = (double)(mix(seed * 1000003ull + i) >> 11) * 0x1p-53 < p ? -mag : mag;
    return v;
}

struct Out {
    std::vector<uint8_t> hard, valid;
    std::vector<int32_t> iters;
    std::vector<double> post;
    bool operator==(const Out& o) const
    {
        return hard == o.hard && valid == o.valid && iters == o.iters &&
               (post.size() == o.post.size() &&
                (post.empty() || std::memcmp(post.data(), o.post.data(), post.size() * 8) == 0));
    }
};

struct Job {
    int kind;  // 0 decode, 1 decode_codes
    int algo;
    int64_t B;
    int max_iter;
    bool want_post;
    std::vector<double> llr;
    std::vector<int8_t> codes;
};

Out run(const ldpc_graph* g, const Job& j, int64_t N, const ldpc_opts* o = nullptr)
{
    Out r;
    r.hard.resize((size_t)(j.B * N));
    r.valid.resize((size_t)j.B);
    r.iters.resize((size_t)j.B);
    if (j.want_post) r.post.resize((size_t)(j.B * N));
    int rc;
    if (j.kind == 0) {
        rc = ldpc_decode(g, j.llr.data(), j.B, j.max_iter, j.algo, r.hard.data(), j.want_post ? r.post.data() : nullptr,
                         r.iters.data(), r.valid.data(), o);
    } else {
        std::vector<double> table(256);
        const double unit = std::log(49.0);
        for (int k = 0; k < 256; k++) table[(size_t)k] = (k - 128) * unit;
        rc = ldpc_decode_codes(g, j.codes.data(), table.data(), LDPC_IN_LLR, j.B, j.max_iter, j.algo, r.hard.data(),
                               j.want_post ? r.post.data() : nullptr, r.iters.data(), r.valid.data(), o);
    }
    if (rc != LDPC_OK) fail("decode status " + std::to_string(rc));
    return r;
}

Out engine_run(const ldpc_graph* g, int64_t B, int64_t N, int max_iter)
{
    Out r;
    int err = 0;
    ldpc_engine* e = ldpc_engine_create(g, 0, LDPC_ALGO_BP, 0, &err);
    if (!e) { fail("engine create"); return r; }
    std::vector<uint8_t> cw((size_t)N, 0);
    void* d_cw = ldpc_dev_malloc(0, (size_t)N);
    void* d_in = ldpc_dev_malloc(0, (size_t)(B * N * 8));
    void* d_h = ldpc_dev_malloc(0, (size_t)(B * N));
    void* d_i = ldpc_dev_malloc(0, (size_t)B * 4);
    void* d_v = ldpc_dev_malloc(0, (size_t)B);
    if (!d_cw || !d_in || !d_h || !d_i || !d_v) { fail("dev malloc"); return r; }
    if (ldpc_dev_memcpy(0, d_cw, cw.data(), (size_t)N, LDPC_H2D) ||
        ldpc_engine_gen_bsc(e, (double*)d_in, LDPC_IN_LR, 0, B, (const uint8_t*)d_cw, 1, 77, 0.004,
                            std::log(0.996 / 0.004)) ||
        ldpc_engine_decode(e, (const double*)d_in, LDPC_IN_LR, B, max_iter, (uint8_t*)d_h, nullptr, LDPC_POST_LLR,
                           (int32_t*)d_i, (uint8_t*)d_v) ||
        ldpc_engine_sync(e))
        fail("engine decode");
    r.hard.resize((size_t)(B * N));
    r.iters.resize((size_t)B);
    r.valid.resize((size_t)B);
    if (ldpc_dev_memcpy(0, r.hard.data(), d_h, r.hard.size(), LDPC_D2H) ||
        ldpc_dev_memcpy(0, r.iters.data(), d_i, (size_t)B * 4, LDPC_D2H) ||
        ldpc_dev_memcpy(0, r.valid.data(), d_v, (size_t)B, LDPC_D2H))
        fail("engine download");
    for (void* p : {d_cw, d_in, d_h, d_i, d_v}) ldpc_dev_free(0, p);
    ldpc_engine_free(e);
    return r;
}

}  // namespace

// a deliberate data race: `tsan_check --selftest` must draw a
// ThreadSanitizer report, which shows the detector is live where the test runs
int g_racy = 0;

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: tsan_check PCHK | --selftest\n");
        return 2;
    }
    if (std::string(argv[1]) == "--selftest") {
        std::thread a([] { for (int i = 0; i < 1000; i++) g_racy++; });
        std::thread b([] { for (int i = 0; i < 1000; i++) g_racy++; });
        a.join();
        b.join();
        std::printf("selftest %d\n", g_racy > 0);
        return 0;
    }
    const std::string pchk = argv[1];
    if (ldpc_device_count() < 1) {
        std::printf("no GPU\n");
        return 4;
    }
    int err = 0;
    ldpc_graph* g = ldpc_graph_load(pchk.c_str(), &err);
    if (!g) { std::printf("load failed\n"); return 4; }
    int32_t M32, N32;
    int64_t E;
    ldpc_graph_info(g, &M32, &N32, &E, nullptr, nullptr, nullptr, nullptr);
    const int64_t N = N32;

    // jobs 4 and 5 span two PCIe chunks (> 4096 codewords): the helper thread
    // that prepares chunk c + 1 while chunk c decodes
    const int NJ = 6;
    std::vector<Job> jobs(NJ);
    jobs[0] = {0, LDPC_ALGO_BP, 64, 20, true, bsc(64, N, 0.004, 1), {}};
    jobs[1] = {0, LDPC_ALGO_BP, 130, 30, false, bsc(130, N, 0.02, 2), {}};
    jobs[2] = {0, LDPC_ALGO_MSA, 80, 25, true, bsc(80, N, 0.002, 3), {}};
    jobs[3] = {1, LDPC_ALGO_BP, 96, 20, false, {}, {}};
    jobs[4] = {0, LDPC_ALGO_BP, 4160, 3, false, bsc(4160, N, 0.01, 5), {}};
    jobs[5] = {1, LDPC_ALGO_MSA, 4160, 3, false, {}, {}};
    for (int j : {3, 5}) {
        const std::vector<double> x = bsc(jobs[(size_t)j].B, N, 0.003, 4 + (uint64_t)j);
        jobs[(size_t)j].codes.resize(x.size());
        for (size_t i = 0; i < x.size(); i++) jobs[(size_t)j].codes[i] = x[i] > 0 ? 1 : -1;
    }
    // alone first
    std::vector<Out> alone;
    for (const Job& j : jobs) alone.push_back(run(g, j, N));
    const Out eng_alone = engine_run(g, 70, N, 15);

    std::vector<std::thread> th;
    for (int t = 0; t < NJ + 2; t++)
        th.emplace_back([&, t] {
            for (int rep = 0; rep < 2; rep++) {
                if (t < NJ) {
                    if (!(run(g, jobs[(size_t)t], N) == alone[(size_t)t])) fail("thread " + std::to_string(t));
                } else if (t == NJ) {
                    if (!(engine_run(g, 70, N, 15) == eng_alone)) fail("engine thread");
                } else {
                    int e2 = 0;
                    if (ldpc_graph_load("/nonexistent/x.pchk", &e2) || e2 != LDPC_ERR_IO) fail("missing-file status");
                    if (std::strstr(ldpc_last_error(), "x.pchk") == nullptr) fail("per-thread error string");
                    ldpc_graph* g2 = ldpc_graph_load(pchk.c_str(), &e2);
                    std::vector<uint8_t> zero((size_t)N, 0);
                    if (!g2 || ldpc_graph_syndrome(g, zero.data(), nullptr) != 0 ||
                        ldpc_graph_syndrome(g2, zero.data(), nullptr) != 0)
                        fail("graph thread");
                    ldpc_graph_free(g2);
                }
            }
        });
    for (auto& t : th) t.join();

    // two shards on device 0: the host API's per-device worker threads
    ldpc_opts o{};
    o.exp_on_host = 1;
    o.n_devices = 2;
    const int32_t devs[2] = {0, 0};
    o.devices = devs;
    if (!(run(g, jobs[1], N, &o) == alone[1])) fail("two shards on device 0");

    ldpc_graph_free(g);
    std::printf("ok tsan: 8 threads x 2 rounds + a two-shard call, results equal the single-thread calls\n");
    return g_bad ? 3 : 0;
}
