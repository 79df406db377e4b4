// abi_check.cpp -- TEST INFRASTRUCTURE: the C ABI (include/ldpc_amd.h) of a
// host-sanitized build of lib/libldpc_amd.so (tests/asan/Makefile `abi`:
// every host unit under -fsanitize=address,undefined, the gfx950 device code
// as usual), called the way a careless binding would call it -- null
// pointers, negative and oversized counts, malformed files, bad enums.  Runs
// on a machine without a GPU (this container): every call must either refuse
// its arguments (LDPC_ERR_ARG / _FORMAT / _IO / _UNSUPPORTED) or get as far
// as the device and report LDPC_ERR_DEVICE, with no sanitizer report.
// Usage: abi_check PCHK TMPDIR.  Output: "ok ..." lines; exit 3 on a wrong
// status ("MISMATCH ...").
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ldpc_amd.h"

namespace {

int g_bad = 0;
int g_n = 0;

void expect(const char* what, int got, int want)
{
    g_n++;
    if (got != want) {
        std::printf("MISMATCH %s: status %d, want %d (%s)\n", what, got, want, ldpc_last_error());
        g_bad = 1;
    }
}

void expect_any(const char* what, int got, std::initializer_list<int> want)
{
    g_n++;
    for (int w : want)
        if (got == w) return;
    std::printf("MISMATCH %s: status %d (%s)\n", what, got, ldpc_last_error());
    g_bad = 1;
}

void write_file(const std::string& path, const void* p, size_t n)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return;
    if (n) std::fwrite(p, 1, n, f);
    std::fclose(f);
}

uint64_t mix(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// with a GPU (tests/test_asan_gpu.py): every host buffer path of the decode
// entry points runs for real under ASan -- staging copies, the next-chunk
// helper thread, packed hard bits unpacked into aligned and unaligned output,
// posteriors, coded input from pageable and pinned memory, two shards, the
// integer decoders, an irregular graph whose N is not a multiple of 8, the
// engine, the DNA kernels.  Consistency: valid <=> zero syndrome, identical
// results through the different entry points.
void gpu_section(const std::string& pchk)
{
    int err = 0;
    // irregular graph: N = 13, an empty column, degree-1 and empty rows
    const int32_t rr[] = {0, 0, 0, 1, 1, 2, 3, 3, 3, 3, 4};
    const int32_t cc[] = {0, 3, 7, 1, 12, 5, 2, 6, 8, 11, 9};
    ldpc_graph* ig = ldpc_graph_from_edges(6, 13, rr, cc, 11, &err);
    if (!ig) { expect("irregular graph", err, LDPC_OK); return; }
    ldpc_graph* g = ldpc_graph_load(pchk.c_str(), &err);
    if (!g) { expect("load", err, LDPC_OK); return; }
    auto check_valid = [&](const std::string& what, const ldpc_graph* gg, int64_t B, int64_t N, const uint8_t* hard,
                           const uint8_t* valid) {
        for (int64_t b = 0; b < B; b++) {
            const int syn = ldpc_graph_syndrome(gg, hard + b * N, nullptr);
            if ((syn == 0) != (valid[b] != 0)) {
                std::printf("MISMATCH %s: codeword %lld syndrome %d valid %d\n", what.c_str(), (long long)b, syn,
                            (int)valid[b]);
                g_bad = 1;
                return;
            }
        }
        g_n++;
    };
    for (int algo : {LDPC_ALGO_BP, LDPC_ALGO_MSA, LDPC_ALGO_QMSA, LDPC_ALGO_GALLAGER_A, LDPC_ALGO_GALLAGER_B2}) {
        const int64_t B = 5, N = 13;
        std::vector<double> x((size_t)(B * N));
        for (size_t i = 0; i < x.size(); i++) x[i] = ((mix(i + 99) >> 40) % 7 == 0 ? -2.0 : 2.5) + (double)(i % 3);
        std::vector<uint8_t> h((size_t)(B * N + 1)), v((size_t)B);
        std::vector<int32_t> it((size_t)B);
        std::vector<double> post((size_t)(B * N));
        expect(("irregular decode, algo " + std::to_string(algo)).c_str(), ldpc_decode(ig, x.data(), B, 7, algo, h.data() + 1,
                                               algo <= LDPC_ALGO_MSA ? post.data() : nullptr, it.data(), v.data(),
                                               nullptr), LDPC_OK);
        check_valid("irregular valid, algo " + std::to_string(algo), ig, B, N, h.data() + 1, v.data());
    }
    const int64_t N = 18432;
    // two PCIe chunks (> 4096 codewords), coded input and fp64 input of the same values
    const int64_t B = 4100;
    const double unit = std::log(49.0);
    std::vector<int8_t> codes((size_t)(B * N));
    for (size_t i = 0; i < codes.size(); i++) codes[i] = (mix(i) >> 11) * 0x1p-53 < 0.01 ? -1 : 1;
    std::vector<double> table(256), x((size_t)(B * N));
    for (int k = 0; k < 256; k++) table[(size_t)k] = (k - 128) * unit;
    for (size_t i = 0; i < x.size(); i++) x[i] = table[(size_t)(codes[i] + 128)];
    std::vector<uint8_t> h1((size_t)(B * N)), h2((size_t)(B * N + 3)), v1((size_t)B), v2((size_t)B);
    std::vector<int32_t> i1((size_t)B), i2((size_t)B);
    expect("big decode", ldpc_decode(g, x.data(), B, 4, LDPC_ALGO_BP, h1.data(), nullptr, i1.data(), v1.data(),
                                     nullptr), LDPC_OK);
    expect("big decode_codes", ldpc_decode_codes(g, codes.data(), table.data(), LDPC_IN_LLR, B, 4, LDPC_ALGO_BP,
                                                 h2.data() + 3, nullptr, i2.data(), v2.data(), nullptr), LDPC_OK);
    expect("fp64 == codes", std::memcmp(h1.data(), h2.data() + 3, h1.size()) == 0 && i1 == i2 && v1 == v2, 1);
    check_valid("big valid", g, B, N, h1.data(), v1.data());
    // pinned codes, posteriors, two shards on device 0
    const int64_t Bp = 300;
    int8_t* pc = (int8_t*)ldpc_host_alloc((size_t)(Bp * N));
    if (!pc) { expect("host alloc", 0, 1); return; }
    std::memcpy(pc, codes.data(), (size_t)(Bp * N));
    std::vector<double> post((size_t)(Bp * N));
    ldpc_opts o{};
    o.exp_on_host = 1;
    o.n_devices = 2;
    const int32_t devs[2] = {0, 0};
    o.devices = devs;
    std::vector<uint8_t> h3((size_t)(Bp * N)), v3((size_t)Bp);
    std::vector<int32_t> i3((size_t)Bp);
    expect("pinned two-shard decode", ldpc_decode_codes(g, pc, table.data(), LDPC_IN_LLR, Bp, 4, LDPC_ALGO_MSA,
                                                        h3.data(), post.data(), i3.data(), v3.data(), &o), LDPC_OK);
    check_valid("pinned valid", g, Bp, N, h3.data(), v3.data());
    ldpc_host_free(pc);
    // the engine: device BSC codes, coded decode, stats
    ldpc_engine* e = ldpc_engine_create(g, 0, LDPC_ALGO_BP, 0, &err);
    expect("engine", e ? 0 : err, 0);
    if (e) {
        const int64_t Be = 200;
        std::vector<uint8_t> cw((size_t)N, 0);
        void* d_cw = ldpc_dev_malloc(0, (size_t)N);
        void* d_c = ldpc_dev_malloc(0, (size_t)(Be * N));
        void* d_h = ldpc_dev_malloc(0, (size_t)(Be * N));
        void* d_i = ldpc_dev_malloc(0, (size_t)Be * 4);
        void* d_v = ldpc_dev_malloc(0, (size_t)Be);
        ldpc_kernel_stats st{};
        expect("engine run", ldpc_dev_memcpy(0, d_cw, cw.data(), (size_t)N, LDPC_H2D) ||
                                  ldpc_engine_profile(e, 1) ||
                                  ldpc_engine_gen_bsc_codes(e, (int8_t*)d_c, 0, Be, (const uint8_t*)d_cw, 1, 5, 0.004) ||
                                  ldpc_engine_decode_codes(e, (const int8_t*)d_c, table.data(), LDPC_IN_LLR, Be, 10,
                                                           (uint8_t*)d_h, nullptr, LDPC_POST_LLR, (int32_t*)d_i,
                                                           (uint8_t*)d_v) ||
                                  ldpc_engine_sync(e) || ldpc_engine_stats(e, &st),
               LDPC_OK);
        std::vector<uint8_t> he((size_t)(Be * N)), ve((size_t)Be);
        ldpc_dev_memcpy(0, he.data(), d_h, he.size(), LDPC_D2H);
        ldpc_dev_memcpy(0, ve.data(), d_v, ve.size(), LDPC_D2H);
        check_valid("engine valid", g, Be, N, he.data(), ve.data());
        for (void* p : {d_cw, d_c, d_h, d_i, d_v}) ldpc_dev_free(0, p);
        ldpc_engine_free(e);
    }
    // the DNA kernels: one strand read twice, one read once (short), codes
    const int32_t kind[3] = {1, 2, 0};
    const int64_t rptr[4] = {0, 2, 3, 3};
    std::vector<uint8_t> rows(3 * 136, 'A');
    rows[136 + 5] = 'T';
    const int32_t q[3] = {70, 40, 80};
    std::vector<double> dl(2 * 136 * 3);
    std::vector<uint8_t> dm(dl.size());
    std::vector<int8_t> dc(dl.size());
    int32_t exact = -1;
    expect("dna llr codes", ldpc_dna_llr_codes(3, kind, rptr, rows.data(), q, 136, unit, dl.data(), dm.data(),
                                               dc.data(), &exact, 0), LDPC_OK);
    bool same = exact == 1;
    for (size_t i = 0; i < dl.size(); i++) same = same && dl[i] == dc[i] * unit;
    expect("dna codes == llr / unit", same ? 1 : 0, 1);
    const char* sq = "ACGTACGTTTACGAACGT";
    const int64_t off[3] = {0, 4, 9};
    const int32_t len[3] = {4, 5, 9}, pa[2] = {0, 1}, pb[2] = {1, 2};
    int32_t dist[2] = {-1, -1};
    expect("edit distance", ldpc_dna_edit_distance((const uint8_t*)sq, off, len, 3, pa, pb, 2, dist, 0), LDPC_OK);
    expect("edit distance values", dist[0] == 1 && dist[1] == 5, 1);  // Levenshtein, def_func.edit_dist
    ldpc_graph_free(g);
    ldpc_graph_free(ig);
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: abi_check PCHK TMPDIR\n");
        return 2;
    }
    const std::string pchk = argv[1], tmp = argv[2];
    expect("abi version", ldpc_abi_version(), LDPC_AMD_ABI_VERSION);
    const int ndev = ldpc_device_count();
    const int DEV = ndev > 0 ? LDPC_OK : LDPC_ERR_DEVICE;  // a decode with good arguments
    int err = 0;

    // ---- graph constructors ----
    expect("load null path", ldpc_graph_load(nullptr, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    ldpc_graph_load(nullptr, nullptr);  // err may be NULL
    expect("load missing", ldpc_graph_load((tmp + "/none.pchk").c_str(), &err) == nullptr ? err : 0, LDPC_ERR_IO);
    const int32_t hdr[] = {('P' << 8) + 0x80, 0x7fffffff, 0x7fffffff, 0};
    write_file(tmp + "/huge.pchk", hdr, sizeof hdr);
    expect("load huge header", ldpc_graph_load((tmp + "/huge.pchk").c_str(), &err) == nullptr ? err : 0,
           LDPC_ERR_UNSUPPORTED);
    write_file(tmp + "/trunc.pchk", hdr, 7);
    expect("load truncated", ldpc_graph_load((tmp + "/trunc.pchk").c_str(), &err) == nullptr ? err : 0,
           LDPC_ERR_FORMAT);
    expect("alist null", ldpc_graph_load_alist(nullptr, 0, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    write_file(tmp + "/bad.alist", "3 3\n1 1\n1 1 x\n", 15);
    expect("alist malformed", ldpc_graph_load_alist((tmp + "/bad.alist").c_str(), 1, &err) == nullptr ? err : 0,
           LDPC_ERR_FORMAT);
    const int32_t rows[] = {0, 1, 1}, cols[] = {0, 0, 2}, badc[] = {0, 3, 1};
    expect("edges null arrays", ldpc_graph_from_edges(2, 3, nullptr, cols, 3, &err) == nullptr ? err : 0,
           LDPC_ERR_ARG);
    expect("edges negative n", ldpc_graph_from_edges(2, 3, rows, cols, -1, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    expect("edges M = 0", ldpc_graph_from_edges(0, 3, rows, cols, 3, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    expect("edges column = N", ldpc_graph_from_edges(2, 3, rows, badc, 3, &err) == nullptr ? err : 0,
           LDPC_ERR_FORMAT);
    expect("edges above LDPC_MAX_DIM",
           ldpc_graph_from_edges(LDPC_MAX_DIM + 1, 3, rows, cols, 3, &err) == nullptr ? err : 0,
           LDPC_ERR_UNSUPPORTED);
    ldpc_graph* small = ldpc_graph_from_edges(2, 3, rows, cols, 3, &err);
    expect("edges ok", small ? err : -99, LDPC_OK);
    expect("rs bad s", ldpc_graph_rs_ldpc(1, 3, 1, nullptr, nullptr, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    expect("rs bad rho", ldpc_graph_rs_ldpc(3, 99, 1, nullptr, nullptr, &err) == nullptr ? err : 0, LDPC_ERR_ARG);
    std::vector<int32_t> gp(5), coset(64);
    ldpc_graph* rs = ldpc_graph_rs_ldpc(3, 6, 3, gp.data(), coset.data(), &err);
    expect("rs ok", rs ? err : -99, LDPC_OK);

    // ---- graph queries ----
    expect("info null graph", ldpc_graph_info(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr),
           LDPC_ERR_ARG);
    expect("info null outs", ldpc_graph_info(small, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr),
           LDPC_OK);
    expect("blocks null graph", ldpc_graph_blocks(nullptr, nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    int32_t Q = -1, rb = 0, cb = 0;
    std::vector<int32_t> colb(48);
    expect("blocks rs", ldpc_graph_blocks(rs, &Q, &rb, &cb, colb.data()), LDPC_OK);
    expect("blocks rs Q", Q, 8);
    expect("blocks irregular", ldpc_graph_blocks(small, &Q, nullptr, nullptr, nullptr), LDPC_OK);
    expect("blocks irregular Q", Q, 0);
    expect("edges null graph", ldpc_graph_edges(nullptr, nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    std::vector<int32_t> rp(3), ci(3), cp(4), ce(3);
    expect("edges copy", ldpc_graph_edges(small, rp.data(), ci.data(), cp.data(), ce.data()), LDPC_OK);
    expect("edges copy nulls", ldpc_graph_edges(small, nullptr, nullptr, nullptr, nullptr), LDPC_OK);
    const uint8_t word[3] = {1, 0, 1};
    uint8_t par[2];
    expect("syndrome null word", ldpc_graph_syndrome(small, nullptr, par), LDPC_ERR_ARG);
    expect("syndrome", ldpc_graph_syndrome(small, word, par), 1);
    expect("syndrome null out", ldpc_graph_syndrome(small, word, nullptr), 1);
    expect("save null", ldpc_graph_save_pchk(nullptr, (tmp + "/x.pchk").c_str()), LDPC_ERR_ARG);
    expect("save no dir", ldpc_graph_save_pchk(small, (tmp + "/no/dir/x.pchk").c_str()), LDPC_ERR_IO);
    expect("save alist", ldpc_graph_save_alist(rs, (tmp + "/rs.alist").c_str()), LDPC_OK);
    ldpc_graph* back = ldpc_graph_load_alist((tmp + "/rs.alist").c_str(), 0, &err);
    expect("alist round trip", back ? err : -99, LDPC_OK);
    ldpc_graph_free(back);
    ldpc_graph_free(nullptr);

    // ---- host decode entry points: argument checks, then the device ----
    ldpc_graph* g = ldpc_graph_load(pchk.c_str(), &err);
    expect("load DNA code", g ? err : -99, LDPC_OK);
    const int64_t N = 18432;
    std::vector<double> llr(2 * N, 3.8918202981106265);
    std::vector<uint8_t> hard(2 * N), valid(2);
    std::vector<int32_t> iters(2);
    std::vector<double> post(2 * N);
    std::vector<int8_t> codes(2 * N, 1);
    std::vector<double> table(256);
    for (int k = 0; k < 256; k++) table[(size_t)k] = (k - 128) * 3.8918202981106265;
    expect("decode null graph", ldpc_decode(nullptr, llr.data(), 2, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr,
                                            nullptr, nullptr), LDPC_ERR_ARG);
    expect("decode B < 0", ldpc_decode(g, llr.data(), -1, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr, nullptr,
                                       nullptr), LDPC_ERR_ARG);
    expect("decode max_iter < 0", ldpc_decode(g, llr.data(), 2, -5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr,
                                              nullptr, nullptr), LDPC_ERR_ARG);
    expect("decode null llr", ldpc_decode(g, nullptr, 2, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr, nullptr,
                                          nullptr), LDPC_ERR_ARG);
    expect("decode null hard", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_BP, nullptr, nullptr, nullptr, nullptr,
                                           nullptr), LDPC_ERR_ARG);
    expect("decode bad algo", ldpc_decode(g, llr.data(), 2, 5, 99, hard.data(), nullptr, nullptr, nullptr, nullptr),
           LDPC_ERR_ARG);
    expect("decode B = 0", ldpc_decode(g, nullptr, 0, 5, LDPC_ALGO_BP, nullptr, nullptr, nullptr, nullptr, nullptr),
           LDPC_OK);
    ldpc_opts o{};
    o.exp_on_host = 1;
    o.post_kind = LDPC_POST_RATIO;
    expect("decode ratio min-sum", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_MSA, hard.data(), post.data(), nullptr,
                                               nullptr, &o), LDPC_ERR_ARG);
    o.post_kind = LDPC_POST_LLR;
    o.msa_precision = 40;
    expect("decode qmsa precision", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_QMSA, hard.data(), nullptr, nullptr,
                                                nullptr, &o), LDPC_ERR_ARG);
    o.msa_precision = 0;
    o.n_devices = 1 << 30;  // no such machine
    expect("decode n_devices", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr, nullptr,
                                           &o), LDPC_ERR_ARG);
    o.n_devices = 1;
    const int32_t neg_dev = -3;
    o.devices = &neg_dev;
    expect("decode device < 0", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr, nullptr,
                                            &o), LDPC_ERR_ARG);
    o.devices = nullptr;
    o.host_threads = 1 << 30;  // clamped, not 2^30 threads
    expect_any("decode host_threads", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_BP, hard.data(), nullptr, nullptr,
                                                  nullptr, &o), {DEV});
    o.host_threads = 0;
    o.chunk = -7;  // <= 0: auto
    expect("decode good args", ldpc_decode(g, llr.data(), 2, 5, LDPC_ALGO_BP, hard.data(), post.data(), iters.data(),
                                           valid.data(), &o), DEV);
    expect("decode B * N overflows", ldpc_decode(g, llr.data(), INT64_MAX / 4, 5, LDPC_ALGO_BP, hard.data(), nullptr,
                                                 nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    expect("codes null", ldpc_decode_codes(g, nullptr, table.data(), LDPC_IN_LLR, 2, 5, LDPC_ALGO_BP, hard.data(),
                                           nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    expect("codes null table", ldpc_decode_codes(g, codes.data(), nullptr, LDPC_IN_LLR, 2, 5, LDPC_ALGO_BP,
                                                 hard.data(), nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    expect("codes LR table min-sum", ldpc_decode_codes(g, codes.data(), table.data(), LDPC_IN_LR, 2, 5, LDPC_ALGO_MSA,
                                                       hard.data(), nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    expect("codes B * N overflows", ldpc_decode_codes(g, codes.data(), table.data(), LDPC_IN_LLR, INT64_MAX / 2, 5,
                                                      LDPC_ALGO_BP, hard.data(), nullptr, nullptr, nullptr, nullptr),
           LDPC_ERR_ARG);
    expect("codes good args", ldpc_decode_codes(g, codes.data(), table.data(), LDPC_IN_LLR, 2, 5, LDPC_ALGO_MSA,
                                                hard.data(), nullptr, iters.data(), valid.data(), nullptr), DEV);

    // ---- engine and memory entry points ----
    expect("engine null graph", ldpc_engine_create(nullptr, 0, LDPC_ALGO_BP, 0, &err) == nullptr ? err : 0,
           LDPC_ERR_ARG);
    ldpc_engine* e = ldpc_engine_create(g, 0, LDPC_ALGO_BP, 0, &err);
    if (ndev == 0) expect("engine without a device", e == nullptr ? err : 0, LDPC_ERR_DEVICE);
    ldpc_engine_free(e);
    ldpc_schedule bad_sched{};
    bad_sched.flags_set = -1;
    bad_sched.flags = -1;
    bad_sched.group_tiles = -5;
    bad_sched.var_cpw = 1000;
    ldpc_engine* e2 = ldpc_engine_create_ex(g, 0, LDPC_ALGO_MSA, -1, &bad_sched, &err);
    if (ndev == 0) expect_any("engine_ex odd schedule", e2 == nullptr ? err : 0, {LDPC_ERR_DEVICE, LDPC_ERR_ARG});
    ldpc_engine_free(e2);
    expect("engine info null", ldpc_engine_info(nullptr, nullptr, nullptr, nullptr), LDPC_ERR_ARG);
    expect("engine decode null", ldpc_engine_decode(nullptr, nullptr, 0, 1, 5, nullptr, nullptr, 0, nullptr, nullptr),
           LDPC_ERR_ARG);
    expect("engine codes null", ldpc_engine_decode_codes(nullptr, nullptr, table.data(), 0, 1, 5, nullptr, nullptr, 0,
                                                         nullptr, nullptr), LDPC_ERR_ARG);
    expect("engine sync null", ldpc_engine_sync(nullptr), LDPC_ERR_ARG);
    expect("engine stream null", ldpc_engine_stream(nullptr) == nullptr ? 0 : 1, 0);
    expect("engine gen null", ldpc_engine_gen_bsc(nullptr, nullptr, 0, 0, 1, nullptr, 1, 1, 0.1, 3.9), LDPC_ERR_ARG);
    expect("engine gen codes null", ldpc_engine_gen_bsc_codes(nullptr, nullptr, 0, 1, nullptr, 1, 1, 0.1),
           LDPC_ERR_ARG);
    expect("engine params null", ldpc_engine_set_params(nullptr, 6, 0.5, 1, 0), LDPC_ERR_ARG);
    expect("engine profile null", ldpc_engine_profile(nullptr, 1), LDPC_ERR_ARG);
    expect("engine stats null", ldpc_engine_stats(nullptr, nullptr), LDPC_ERR_ARG);
    void* hp = ldpc_host_alloc(64);
    if (ndev == 0) expect("host alloc without a device", hp == nullptr ? 0 : 1, 0);
    expect("host free", ldpc_host_free(hp), LDPC_OK);
    expect("host free null", ldpc_host_free(nullptr), LDPC_OK);
    if (ndev == 0) {
        expect("dev malloc", ldpc_dev_malloc(0, 64) == nullptr ? 0 : 1, 0);
        expect("dev free", ldpc_dev_free(0, nullptr), LDPC_ERR_DEVICE);
        expect("dev memcpy", ldpc_dev_memcpy(0, hard.data(), llr.data(), 8, LDPC_D2D), LDPC_ERR_DEVICE);
    }

    // ---- DNA stage ----
    const int32_t kind[2] = {1, 0};
    const int64_t rptr[3] = {0, 1, 1}, bad_rptr[3] = {0, 2, 1};
    const uint8_t seq[136] = {'A'};
    const int32_t q[1] = {70};
    std::vector<double> dl(2 * 136 * 2);
    std::vector<uint8_t> dm(dl.size());
    std::vector<int8_t> dc(dl.size());
    int32_t exact = -1;
    expect("dna llr null", ldpc_dna_llr(2, nullptr, rptr, seq, q, 136, 3.89, dl.data(), dm.data(), 0), LDPC_ERR_ARG);
    expect("dna llr nt = 0", ldpc_dna_llr(2, kind, rptr, seq, q, 0, 3.89, dl.data(), dm.data(), 0), LDPC_ERR_ARG);
    expect("dna llr row_ptr", ldpc_dna_llr(2, kind, bad_rptr, seq, q, 136, 3.89, dl.data(), dm.data(), 0),
           LDPC_ERR_ARG);
    const int32_t bad_kind[2] = {7, 0};
    expect("dna llr kind", ldpc_dna_llr(2, bad_kind, rptr, seq, q, 136, 3.89, dl.data(), dm.data(), 0), LDPC_ERR_ARG);
    expect("dna codes no exact", ldpc_dna_llr_codes(2, kind, rptr, seq, q, 136, 3.89, dl.data(), dm.data(), dc.data(),
                                                    nullptr, 0), LDPC_ERR_ARG);
    expect("dna codes empty", ldpc_dna_llr_codes(0, kind, rptr, seq, q, 136, 3.89, dl.data(), nullptr, dc.data(),
                                                 &exact, 0), LDPC_OK);
    expect("dna codes empty exact", exact, 1);
    expect("dna codes good args", ldpc_dna_llr_codes(2, kind, rptr, seq, q, 136, 3.89, dl.data(), dm.data(),
                                                     dc.data(), &exact, 0), DEV);
    const int64_t off[2] = {0, 5};
    const int32_t len[2] = {5, 900}, pa[1] = {0}, pb[1] = {1};
    int32_t dist[1];
    expect("edit distance null", ldpc_dna_edit_distance(nullptr, off, len, 2, pa, pb, 1, dist, 0),
           LDPC_ERR_UNSUPPORTED);  // (the 900-nt length is refused first)
    expect("edit distance too long", ldpc_dna_edit_distance((const uint8_t*)"ACGTACGTAC", off, len, 2, pa, pb, 1,
                                                            dist, 0), LDPC_ERR_UNSUPPORTED);
    const int64_t off_big[2] = {0, INT64_MAX - 2};
    const int32_t len_ok[2] = {5, 5};
    expect("edit distance null seqs", ldpc_dna_edit_distance(nullptr, off, len_ok, 2, pa, pb, 1, dist, 0),
           LDPC_ERR_ARG);
    expect("edit distance offset overflow", ldpc_dna_edit_distance((const uint8_t*)"ACGTACGTAC", off_big, len_ok, 2,
                                                                   pa, pb, 1, dist, 0), LDPC_ERR_ARG);
    const int32_t far[1] = {5};
    expect("edit distance index", ldpc_dna_edit_distance((const uint8_t*)"ACGTACGTAC", off, len, 2, pa, far, 1, dist,
                                                         0), LDPC_ERR_ARG);
    expect("soft files null", ldpc_write_soft_files(nullptr, 1, dl.data(), nullptr, 1, 1), LDPC_ERR_ARG);
    expect("soft files negative", ldpc_write_soft_files(tmp.c_str(), 1, dl.data(), nullptr, -1, 1), LDPC_ERR_ARG);
    char rb2[4];
    expect("repr small buffer", ldpc_py_float_repr(-1.2345678901234567e-300, rb2, 4), LDPC_ERR_ARG);
    char rb3[40];
    expect("repr", ldpc_py_float_repr(-1.2345678901234567e-300, rb3, 40), 24);
    expect("repr text", std::strcmp(rb3, "-1.2345678901234568e-300"), 0);  // Python repr()
    expect("repr null", ldpc_py_float_repr(1.0, nullptr, 40), LDPC_ERR_ARG);

    ldpc_graph_free(g);
    ldpc_graph_free(small);
    ldpc_graph_free(rs);
    if (ndev > 0) gpu_section(pchk);
    std::printf("ok abi %d checks, %d device(s)\n", g_n, ndev);
    return g_bad ? 3 : 0;
}
