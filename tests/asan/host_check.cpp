// host_check.cpp -- TEST INFRASTRUCTURE: driver of the host ASan/UBSan build
// (tests/asan/Makefile, run by tests/test_asan_host.py).  Not part of the
// product.
//
// Every subcommand exercises host-only product code on untrusted input and,
// where the oracle restates the same reference function, checks the two agree:
//   pchk FILE                 load_pchk vs oracle_graph_load (rcode.cpp:54-85,
//                             mod2sparse.cpp:381-427); accepted graphs
//                             round-trip through save_pchk / save_alist
//   alist FILE                load_alist (alist-to-pchk.cpp:36-160), both
//                             orientations; accepted graphs round-trip
//   ints FILE N SHORT | doubles FILE N
//                             the CLI's codeword / soft-file readers
//                             (cli_io.cpp; DNA_main.cpp:1322-1345)
//   fuzz-pchk | fuzz-alist | fuzz-text  SEED COUNT DIR
//                             seeded mutations of valid files / token streams
//   repr SEED COUNT DIR       py_float_repr round trip + ldpc_write_soft_files
//   lattice SEED              host_encode_lattice against a scalar restatement
//   rs                        build_rs_ldpc / find_block_layout, valid and
//                             invalid parameters
//   decode FILE ALGO ITERS SEED P
//                             one oracle BP (0) or min-sum (1) decode of a BSC
//                             word, plus a threaded batch; syndrome_host vs
//                             oracle_check
// Output: one "ok ..." / "err ..." line per check; exit 0, or 3 on a
// disagreement ("MISMATCH ...").  A sanitizer report aborts with its own code.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../dna-ldpc-codes_amd/csrc/cli_io.hpp"
#include "../../dna-ldpc-codes_amd/csrc/graph.hpp"
#include "../../dna-ldpc-codes_amd/csrc/host_io.hpp"
#include "../../dna-ldpc-codes_amd/csrc/host_simd.hpp"
#include "../../include/ldpc_amd.h"
#include "../../oracle/ldpc_oracle.h"

extern "C" int ldpc_write_soft_files(const char* dir, int32_t rs, const double* llr, const uint8_t* int_mask,
                                     int32_t n_files, int32_t n_strands);

namespace ldpc {
static std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace ldpc

namespace {

int g_bad = 0;

void mismatch(const std::string& what)
{
    std::printf("MISMATCH %s\n", what.c_str());
    g_bad = 1;
}

struct Rng {  // splitmix64
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

std::vector<unsigned char> slurp(const std::string& path)
{
    std::vector<unsigned char> b;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return b;
    unsigned char tmp[4096];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + got);
    std::fclose(f);
    return b;
}

void spit(const std::string& path, const void* p, size_t n)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    if (n && std::fwrite(p, 1, n, f) != n) { std::perror(path.c_str()); std::exit(2); }
    std::fclose(f);
}

bool same_graph(const ldpc::HostGraph& a, const ldpc::HostGraph& b)
{
    return a.M == b.M && a.N == b.N && a.E == b.E && a.row_ptr == b.row_ptr && a.col_idx == b.col_idx &&
           a.col_ptr == b.col_ptr && a.col_edge == b.col_edge && a.edge_row == b.edge_row;
}

bool same_as_oracle(const ldpc::HostGraph& g, const oracle_graph& o)
{
    if (g.M != o.M || g.N != o.N || g.E != o.E) return false;
    for (int32_t i = 0; i <= g.M; i++)
        if (g.row_ptr[(size_t)i] != o.row_ptr[i]) return false;
    for (int32_t j = 0; j <= g.N; j++)
        if (g.col_ptr[(size_t)j] != o.col_ptr[j]) return false;
    for (int64_t e = 0; e < g.E; e++)
        if (g.col_idx[(size_t)e] != o.col_idx[e] || g.col_edge[(size_t)e] != o.col_edge[e]) return false;
    return true;
}

// structural invariants every accepted graph must satisfy
bool well_formed(const ldpc::HostGraph& g)
{
    if (g.M <= 0 || g.N <= 0 || g.E < 0) return false;
    if (g.row_ptr.size() != (size_t)g.M + 1 || g.col_ptr.size() != (size_t)g.N + 1) return false;
    if (g.row_ptr[0] != 0 || g.row_ptr[(size_t)g.M] != g.E || g.col_ptr[0] != 0 || g.col_ptr[(size_t)g.N] != g.E)
        return false;
    for (int32_t i = 0; i < g.M; i++) {
        if (g.row_ptr[(size_t)i] > g.row_ptr[(size_t)i + 1]) return false;
        for (int32_t e = g.row_ptr[(size_t)i]; e < g.row_ptr[(size_t)i + 1]; e++) {
            const int32_t c = g.col_idx[(size_t)e];
            if (c < 0 || c >= g.N || g.edge_row[(size_t)e] != i) return false;
            if (e > g.row_ptr[(size_t)i] && g.col_idx[(size_t)e - 1] >= c) return false;  // ascending, no duplicates
        }
    }
    for (int32_t j = 0; j < g.N; j++)
        for (int32_t q = g.col_ptr[(size_t)j]; q < g.col_ptr[(size_t)j + 1]; q++) {
            const int32_t e = g.col_edge[(size_t)q];
            if (e < 0 || e >= g.E || g.col_idx[(size_t)e] != j) return false;
            if (q > g.col_ptr[(size_t)j] && g.edge_row[(size_t)g.col_edge[(size_t)q - 1]] >= g.edge_row[(size_t)e])
                return false;
        }
    return true;
}

// header dimensions of a .pchk (0 when the file is too short or not one)
void pchk_header(const std::vector<unsigned char>& b, int64_t* M, int64_t* N)
{
    *M = *N = 0;
    if (b.size() < 12) return;
    auto w = [&](size_t k) {
        return (int32_t)((uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
                         ((uint32_t)b[4 * k + 3] << 24));
    };
    if (w(0) != ('P' << 8) + 0x80) return;
    *M = w(1);
    *N = w(2);
}

// load one .pchk with the product and (when its header is within the cap, so
// that the restatement's unbounded allocation stays small) the oracle; both
// must accept or reject it together and build the same arrays
int check_pchk(const std::string& path, bool roundtrip, bool quiet)
{
    ldpc::HostGraph g;
    std::string msg;
    const int rc = ldpc::load_pchk(path, g, &msg);
    int64_t hM, hN;
    pchk_header(slurp(path), &hM, &hN);
    const bool big = hM > LDPC_MAX_DIM || hN > LDPC_MAX_DIM;
    if (big) {
        if (rc != LDPC_ERR_UNSUPPORTED) mismatch(path + ": header above LDPC_MAX_DIM not refused");
    } else {
        oracle_graph o;
        const int orc = oracle_graph_load(path.c_str(), &o);
        if ((rc == LDPC_OK) != (orc == 0)) mismatch(path + ": product rc " + std::to_string(rc) + ", oracle rc " +
                                                    std::to_string(orc));
        else if (rc == LDPC_OK && !same_as_oracle(g, o)) mismatch(path + ": graph differs from the oracle's");
        if (orc == 0) oracle_graph_free(&o);
    }
    if (rc == LDPC_OK) {
        if (!well_formed(g)) mismatch(path + ": accepted graph is malformed");
        if (roundtrip) {
            ldpc::HostGraph r;
            if (ldpc::save_pchk(g, path + ".rt.pchk", &msg) != LDPC_OK ||
                ldpc::load_pchk(path + ".rt.pchk", r, &msg) != LDPC_OK || !same_graph(g, r))
                mismatch(path + ": .pchk round trip");
            // empty columns/rows make an alist the reader refuses (degree 0 is
            // legal there only with max degree 0), so only check full graphs
            if (ldpc::save_alist(g, path + ".rt.alist", &msg) != LDPC_OK) mismatch(path + ": save_alist");
            else if (ldpc::load_alist(path + ".rt.alist", false, r, &msg) == LDPC_OK && !same_graph(g, r))
                mismatch(path + ": alist round trip");
            std::remove((path + ".rt.pchk").c_str());
            std::remove((path + ".rt.alist").c_str());
        }
    }
    if (!quiet) {
        if (rc == LDPC_OK) std::printf("ok pchk %d %d %lld\n", g.M, g.N, (long long)g.E);
        else std::printf("err pchk %d %s\n", rc, msg.c_str());
    }
    return rc;
}

int check_alist(const std::string& path, bool quiet)
{
    int rc0 = 0;
    for (int t = 0; t < 2; t++) {
        ldpc::HostGraph g, r;
        std::string msg;
        const int rc = ldpc::load_alist(path, t != 0, g, &msg);
        if (t == 0) rc0 = rc;
        if (rc == LDPC_OK) {
            if (!well_formed(g)) mismatch(path + ": accepted alist graph is malformed");
            if (ldpc::save_alist(g, path + ".rt", &msg) != LDPC_OK ||
                ldpc::load_alist(path + ".rt", false, r, &msg) != LDPC_OK || !same_graph(g, r))
                mismatch(path + ": alist round trip");
            std::remove((path + ".rt").c_str());
        }
        if (!quiet) {
            if (rc == LDPC_OK) std::printf("ok alist%s %d %d %lld\n", t ? "-t" : "", g.M, g.N, (long long)g.E);
            else std::printf("err alist%s %d %s\n", t ? "-t" : "", rc, msg.c_str());
        }
    }
    return rc0;
}

// a small full-weight code to mutate: RS-LDPC(3, 6, 3), M = 24, N = 48
ldpc::HostGraph small_code()
{
    ldpc::HostGraph g;
    if (ldpc::build_rs_ldpc(3, 6, 3, g, nullptr, nullptr, nullptr) != LDPC_OK) {
        std::printf("MISMATCH build_rs_ldpc(3,6,3) failed\n");
        std::exit(3);
    }
    return g;
}

void put_le32(std::vector<unsigned char>& b, size_t at, int32_t v)
{
    const uint32_t u = (uint32_t)v;
    for (int k = 0; k < 4; k++) b[at + (size_t)k] = (unsigned char)(u >> (8 * k));
}

int fuzz_pchk(uint64_t seed, int count, const std::string& dir)
{
    const std::string base = dir + "/fz_base.pchk", path = dir + "/fz.pchk";
    std::string msg;
    ldpc::HostGraph g = small_code();
    if (ldpc::save_pchk(g, base, &msg) != LDPC_OK) { std::printf("MISMATCH save_pchk\n"); return 3; }
    const std::vector<unsigned char> orig = slurp(base);
    Rng r{seed};
    int acc = 0;
    // (accepted dimensions stay small: a header near LDPC_MAX_DIM is valid and
    // only costs time; above it must be refused before any allocation)
    static const int32_t special[] = {0, 1, -1, 2, -2, INT32_MIN, INT32_MAX, 24, 25, -24, -25, 48, 49, 4096,
                                      LDPC_MAX_DIM + 1};
    for (int it = 0; it < count; it++) {
        std::vector<unsigned char> b = orig;
        const int op = (int)r.below(7);
        const size_t nw = b.size() / 4;
        if (op == 0) {  // flip 1-4 bytes
            for (int k = 1 + (int)r.below(4); k > 0; k--) b[r.below(b.size())] ^= (unsigned char)(1 + r.below(255));
        } else if (op == 1) {  // truncate anywhere (odd lengths included)
            b.resize(r.below(b.size() + 1));
        } else if (op == 2) {  // overwrite a word with a special value
            put_le32(b, 4 * r.below(nw), special[r.below(sizeof special / sizeof special[0])]);
        } else if (op == 3) {  // delete a word
            const size_t w = r.below(nw);
            b.erase(b.begin() + (long)(4 * w), b.begin() + (long)(4 * w + 4));
        } else if (op == 4) {  // duplicate a word (duplicate entries / rows)
            const size_t w = r.below(nw);
            std::vector<unsigned char> word(b.begin() + (long)(4 * w), b.begin() + (long)(4 * w + 4));
            b.insert(b.begin() + (long)(4 * w), word.begin(), word.end());
        } else if (op == 5) {  // header M / N: small, negative or above the cap
            const int32_t v = r.below(4) ? (int32_t)r.below(4100) - 4 : LDPC_MAX_DIM + 1 + (int32_t)r.below(1u << 30);
            put_le32(b, 4 + 4 * r.below(2), v);
        } else {  // trailing garbage after the terminator
            for (int k = 1 + (int)r.below(7); k > 0; k--) b.push_back((unsigned char)r.below(256));
        }
        spit(path, b.data(), b.size());
        int64_t hM, hN;
        pchk_header(b, &hM, &hN);
        const bool small = hM <= 4096 && hN <= 4096;  // byte flips can make a valid 16M-row header: load, skip the round trip
        acc += check_pchk(path, small && (it & 3) == 0, true) == LDPC_OK;
    }
    std::printf("ok fuzz-pchk %d mutations, %d accepted\n", count, acc);
    return 0;
}

std::vector<std::string> split_ws(const std::vector<unsigned char>& b)
{
    std::vector<std::string> t;
    std::string cur;
    for (unsigned char c : b) {
        if (c == ' ' || c == '\n' || c == '\t' || c == '\r') {
            if (!cur.empty()) { t.push_back(cur); cur.clear(); }
        } else {
            cur.push_back((char)c);
        }
    }
    if (!cur.empty()) t.push_back(cur);
    return t;
}

int fuzz_alist(uint64_t seed, int count, const std::string& dir)
{
    const std::string base = dir + "/fz_base.alist", path = dir + "/fz.alist";
    std::string msg;
    ldpc::HostGraph g = small_code();
    if (ldpc::save_alist(g, base, &msg) != LDPC_OK) { std::printf("MISMATCH save_alist\n"); return 3; }
    const std::vector<std::string> orig = split_ws(slurp(base));
    static const char* junk[] = {"x", "1x", "+", "-", "-0", "+3", "99999999999", "-99999999999", "0x10", "", "1.5"};
    Rng r{seed};
    int acc = 0;
    for (int it = 0; it < count; it++) {
        std::vector<std::string> t = orig;
        const int op = (int)r.below(6);
        const size_t k = r.below(t.size());
        if (op == 0) t[k] = std::to_string((int)r.below(52) - 2);
        else if (op == 1) t[k] = junk[r.below(sizeof junk / sizeof junk[0])];
        else if (op == 2) t.erase(t.begin() + (long)k);
        else if (op == 3) t.insert(t.begin() + (long)k, t[k]);
        else if (op == 4) std::swap(t[k], t[r.below(t.size())]);
        else t.resize(k);
        std::string text;
        for (size_t i = 0; i < t.size(); i++) text += t[i] + ((i & 15) == 15 ? "\n" : " ");
        if (op == 5 && r.below(2)) text.resize(r.below(text.size() + 1));  // cut inside a token too
        spit(path, text.data(), text.size());
        acc += check_alist(path, true) == LDPC_OK;
    }
    std::printf("ok fuzz-alist %d mutations, %d accepted\n", count, acc);
    return 0;
}

int do_ints(const std::string& path, size_t n, bool allow_short)
{
    std::vector<int> v;
    std::string msg;
    if (!ldpc_cli::read_int_file(path, n, allow_short, v, &msg)) {
        std::printf("err ints %s\n", msg.c_str());
        return 0;
    }
    long long sum = 0;
    for (int x : v) sum += x;
    std::printf("ok ints %zu %lld\n", v.size(), sum);
    return 0;
}

int do_doubles(const std::string& path, size_t n)
{
    std::vector<double> v;
    std::string msg;
    if (!ldpc_cli::read_double_file(path, n, v, &msg)) {
        std::printf("err doubles %s\n", msg.c_str());
        return 0;
    }
    int nan = 0, inf = 0;
    for (double x : v) { nan += std::isnan(x); inf += std::isinf(x); }
    std::printf("ok doubles %zu nan=%d inf=%d first=%.17g\n", v.size(), nan, inf, v.empty() ? 0.0 : v[0]);
    return 0;
}

// random token streams through both readers; valid tokens must parse to what
// strtol / strtod give, invalid ones must be refused
int fuzz_text(uint64_t seed, int count, const std::string& dir)
{
    static const char* tokens[] = {"0", "1", "-1", "+7", "2147483647", "-2147483648", "2147483648", "-99999999999999",
                                   "3.8918202981106265", "-3.8918202981106265", "1e-05", "-0.0", "nan", "-nan",
                                   "inf", "-inf", "Infinity", "1e999", "-1e999", "4.9e-324", "0x1p3", "1.", ".5",
                                   "abc", "1,2", "--1", "+-1", "1e", "e5", "0x", "\x01\x02", "\xff\xfe"};
    const size_t ntok = sizeof tokens / sizeof tokens[0];
    const std::string path = dir + "/fz.txt";
    Rng r{seed};
    int ok_i = 0, ok_d = 0;
    for (int it = 0; it < count; it++) {
        const size_t n = 1 + r.below(40);
        std::vector<std::string> t;
        std::string text;
        const size_t len = r.below(4) ? n + r.below(4) : r.below(n + 6);
        // mode 0: integer tokens, 1: number tokens, 2: anything; one stray
        // token in 8 files of modes 0 and 1
        const int mode = (int)r.below(3);
        const size_t stray = r.below(8) == 0 ? r.below(len + 1) : (size_t)-1;
        for (size_t i = 0; i < len; i++) {
            const size_t pick = (mode == 2 || i == stray) ? r.below(ntok) : r.below(mode == 0 ? 7 : 23);
            std::string s = tokens[pick];
            if (r.below(50) == 0) s = std::string(400 + r.below(400), "12345.e"[r.below(7)]);  // long tokens
            t.push_back(s);
            text += s;
            static const char* seps[] = {" ", "\n", "\t", "\r\n", "  ", "\v", "\f"};
            text += seps[r.below(7)];
        }
        if (r.below(4) == 0 && !text.empty()) text.pop_back();  // no trailing separator
        spit(path, text.data(), text.size());
        // expected, token by token
        auto valid_d = [](const std::string& s) {
            char* end;
            (void)std::strtod(s.c_str(), &end);
            return !s.empty() && s.size() <= ldpc_cli::kMaxToken && *end == 0;
        };
        auto valid_i = [](const std::string& s) {
            const size_t p = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
            if (p >= s.size() || s.size() > ldpc_cli::kMaxToken) return false;
            for (size_t k = p; k < s.size(); k++)
                if (s[k] < '0' || s[k] > '9') return false;
            return true;
        };
        bool exp_i = t.size() >= n, exp_d = t.size() >= n, exp_short = true;
        for (size_t i = 0; i < std::min(n, t.size()); i++) {
            exp_d = exp_d && valid_d(t[i]);
            exp_i = exp_i && valid_i(t[i]);
        }
        for (size_t i = 0; i < std::min(n + 3, t.size()); i++) exp_short = exp_short && valid_i(t[i]);
        std::vector<int> vi;
        std::vector<double> vd;
        std::string msg;
        const bool gi = ldpc_cli::read_int_file(path, n, false, vi, &msg);
        const bool gd = ldpc_cli::read_double_file(path, n, vd, &msg);
        if (gi != exp_i) mismatch("fuzz-text ints iteration " + std::to_string(it));
        if (gd != exp_d) mismatch("fuzz-text doubles iteration " + std::to_string(it));
        if (gd)
            for (size_t i = 0; i < n; i++) {
                const double want = std::strtod(t[i].c_str(), nullptr);
                if (std::memcmp(&want, &vd[i], sizeof want) != 0 && !(std::isnan(want) && std::isnan(vd[i])))
                    mismatch("fuzz-text double value");
            }
        if (gi)
            for (size_t i = 0; i < n; i++) {
                const long x = std::strtol(t[i].c_str(), nullptr, 10);
                const int want = x > INT32_MAX ? INT32_MAX : x < INT32_MIN ? INT32_MIN : (int)x;
                if (vi[i] != want) mismatch("fuzz-text int value");
            }
        // the side-file reader pads a short file with zeros
        if (ldpc_cli::read_int_file(path, n + 3, true, vi, &msg) != exp_short || vi.size() != n + 3)
            mismatch("fuzz-text allow_short");
        ok_i += gi;
        ok_d += gd;
    }
    std::printf("ok fuzz-text %d files, %d int / %d double accepted\n", count, ok_i, ok_d);
    return 0;
}

int do_repr(uint64_t seed, int count, const std::string& dir)
{
    Rng r{seed};
    std::vector<double> v = {0.0, -0.0, 1.0, -1.0, 0.1, 1e16, 1e15, 9.999999999999999e15, 1e-4, 9.9e-5, 1e-5,
                             5e-324, -5e-324, 1.7976931348623157e308, -1.7976931348623157e308, INFINITY, -INFINITY,
                             NAN, 3.8918202981106265, 2.2250738585072014e-308, 123456789012345678.0};
    for (int i = 0; i < count; i++) {
        uint64_t bits = r.next();
        double x;
        std::memcpy(&x, &bits, sizeof x);
        v.push_back(x);
        v.push_back(std::ldexp(r.unit(), (int)r.below(120) - 60));
    }
    char buf[64];
    for (double x : v) {
        std::memset(buf, 0, sizeof buf);
        const size_t n = ldpc::py_float_repr(x, buf);
        if (n == 0 || n >= 32) { mismatch("py_float_repr length"); continue; }
        const double back = std::strtod(buf, nullptr);
        if (std::isnan(x) ? !std::isnan(back) || std::strcmp(buf, "nan") != 0
                          : std::memcmp(&back, &x, sizeof x) != 0)
            mismatch(std::string("py_float_repr round trip ") + buf);
    }
    // the soft-file writer: a few files with int-marked zeros
    const int nf = 3, ns = 17;
    std::vector<double> llr((size_t)nf * ns);
    std::vector<uint8_t> mask((size_t)nf * ns, 0);
    for (size_t i = 0; i < llr.size(); i++) {
        llr[i] = (i % 5 == 0) ? 0.0 : v[i % v.size()];
        mask[i] = (i % 5 == 0) && (i % 2 == 0);
    }
    if (ldpc_write_soft_files(dir.c_str(), 7, llr.data(), mask.data(), nf, ns) != LDPC_OK)
        mismatch("ldpc_write_soft_files: " + ldpc::g_err);
    llr[0] = 1.0;  // int-marked but nonzero: refused
    if (ldpc_write_soft_files(dir.c_str(), 7, llr.data(), mask.data(), nf, ns) != LDPC_ERR_ARG)
        mismatch("ldpc_write_soft_files accepted a nonzero int-marked value");
    if (ldpc_write_soft_files((dir + "/no/such/dir").c_str(), 7, llr.data(), nullptr, nf, ns) != LDPC_ERR_IO)
        mismatch("ldpc_write_soft_files into a missing directory");
    std::printf("ok repr %zu values\n", v.size());
    return 0;
}

// host_encode_lattice (host_simd.cpp) against a scalar restatement of its
// contract: code = round(x / unit) clamped to +-kmax; false when any x in
// [i0, i1) is not exactly code * unit (or is -0.0 with keep_neg_zero)
int do_lattice(uint64_t seed)
{
    Rng r{seed};
    const double unit = std::log(49.0);
    for (int rep = 0; rep < 200; rep++) {
        const size_t n = 1 + r.below(300);
        std::vector<double> x(n);
        for (size_t i = 0; i < n; i++) x[i] = (double)((int)r.below(13) - 6) * unit;
        const int kind = (int)r.below(8);
        if (kind >= 1) {
            static const double bad[] = {NAN, INFINITY, -INFINITY, -0.0, 1e300, -1e300, 0.5, 7 * 3.8918202981106265};
            x[r.below(n)] = bad[kind - 1];
        }
        const size_t i0 = r.below(n), i1 = i0 + r.below(n - i0 + 1);
        for (int keep = 0; keep < 2; keep++) {
            const int kmax = 1 + (int)r.below(8);
            std::vector<int8_t> code(n, 99);
            const bool got = ldpc::host_encode_lattice(x.data(), code.data(), i0, i1, unit, kmax, keep != 0);
            bool want = true;
            for (size_t i = i0; i < i1; i++) {
                const double k = std::nearbyint(x[i] / unit);
                if (!(k * unit == x[i]) || !(std::fabs(k) <= kmax) || (keep && std::signbit(x[i]) && x[i] == 0))
                    want = false;
                else if (code[i] != (int8_t)k) mismatch("host_encode_lattice code");
            }
            for (size_t i = 0; i < n; i++)
                if ((i < i0 || i >= i1) && code[i] != 99) mismatch("host_encode_lattice wrote outside [i0, i1)");
            if (got != want) mismatch("host_encode_lattice verdict");
        }
    }
    std::printf("ok lattice\n");
    return 0;
}

int do_rs()
{
    static const int cases[][3] = {{3, 6, 3}, {4, 8, 3}, {4, 16, 16}, {5, 12, 4}, {2, 4, 4}, {8, 72, 8},
                                   {1, 3, 1}, {11, 3, 1}, {3, 2, 1}, {3, 9, 1}, {3, 4, 0}, {3, 4, 9}, {-1, -1, -1}};
    for (auto& c : cases) {
        ldpc::HostGraph g;
        std::vector<int> gp, coset;
        std::string msg;
        const int rc = ldpc::build_rs_ldpc(c[0], c[1], c[2], g, &gp, &coset, &msg);
        if (rc == LDPC_OK) {
            if (!well_formed(g) || g.M != c[2] << c[0] || g.N != c[1] << c[0]) mismatch("build_rs_ldpc shape");
            ldpc::BlockLayout L;
            if (!ldpc::find_block_layout(g, L) || L.Q != 1 << c[0] || L.RB != c[1] || L.GA != c[2])
                mismatch("find_block_layout on an RS-LDPC code");
            if (!ldpc::block_layout_of(g)) mismatch("block_layout_of");
            std::printf("ok rs %d %d %d E=%lld\n", c[0], c[1], c[2], (long long)g.E);
        } else {
            std::printf("err rs %d %d %d %d %s\n", c[0], c[1], c[2], rc, msg.c_str());
        }
    }
    // a graph with no block structure
    const int32_t rows[] = {0, 0, 1, 2, 2}, cols[] = {0, 3, 1, 2, 0};
    ldpc::HostGraph h;
    std::string msg;
    if (ldpc::build_graph(3, 4, rows, cols, 5, h, &msg) != LDPC_OK || ldpc::block_layout_of(h))
        mismatch("irregular graph block layout");
    if (ldpc::build_graph(LDPC_MAX_DIM + 1, 4, rows, cols, 0, h, &msg) != LDPC_ERR_UNSUPPORTED)
        mismatch("build_graph above LDPC_MAX_DIM");
    if (ldpc::build_graph(0, 4, rows, cols, 0, h, &msg) != LDPC_ERR_ARG) mismatch("build_graph M = 0");
    const int32_t badc[] = {4};
    if (ldpc::build_graph(3, 4, rows, badc, 1, h, &msg) != LDPC_ERR_FORMAT) mismatch("build_graph column = N");
    return 0;
}

int do_decode(const std::string& path, int algo, int iters, uint64_t seed, double p)
{
    ldpc::HostGraph g;
    std::string msg;
    if (ldpc::load_pchk(path, g, &msg) != LDPC_OK) { std::printf("MISMATCH %s\n", msg.c_str()); return 3; }
    oracle_graph o;
    if (oracle_graph_load(path.c_str(), &o) != 0) { std::printf("MISMATCH oracle load\n"); return 3; }
    const int N = g.N, B = 4;
    Rng r{seed};
    // BSC(p) on the all-zero codeword, LLR = +-ln((1-p)/p) (synth.bsc_llrs)
    const double mag = std::log((1 - p) / p);
    std::vector<double> llr((size_t)B * N), lr((size_t)N);
    for (auto& x : llr) x = r.unit() < p ? -mag : mag;
    for (int j = 0; j < N; j++) lr[(size_t)j] = std::exp(llr[(size_t)j]);
    std::vector<uint8_t> dblk((size_t)N), pchk_a((size_t)g.M), pchk_b((size_t)g.M);
    std::vector<double> post((size_t)N);
    int valid = 0;
    const int it = algo == 0 ? oracle_bp(&o, lr.data(), iters, dblk.data(), post.data(), &valid)
                             : oracle_msa(&o, llr.data(), iters, dblk.data(), post.data(), &valid);
    const int sa = ldpc::syndrome_host(g, dblk.data(), pchk_a.data());
    const int sb = oracle_check(&o, dblk.data(), pchk_b.data());
    if (sa != sb || pchk_a != pchk_b) mismatch("syndrome_host vs oracle_check");
    if ((sa == 0) != (valid != 0)) mismatch("valid flag vs syndrome");
    int flips = 0;
    for (int j = 0; j < N; j++) flips += dblk[(size_t)j];
    // the threaded batch path must give the single decode's answer for row 0
    std::vector<uint8_t> hard((size_t)B * N), vb((size_t)B);
    std::vector<int32_t> ib((size_t)B);
    oracle_decode_batch(&o, llr.data(), B, iters, algo == 0 ? ORACLE_ALGO_BP : ORACLE_ALGO_MSA, ORACLE_POST_LLR, 2,
                        hard.data(), nullptr, ib.data(), vb.data());
    if (ib[0] != it || (vb[0] != 0) != (valid != 0) || std::memcmp(hard.data(), dblk.data(), (size_t)N) != 0)
        mismatch("oracle_decode_batch row 0 vs single decode");
    std::printf("ok decode algo=%d iters=%d valid=%d ones=%d syndrome=%d\n", algo, it, valid, flips, sa);
    // the integer-message decoders of the oracle (quantized / offset min-sum,
    // Gallager A / B1 / B2): valid flags must agree with the host syndrome
    // (with infinite, NaN and huge inputs: the quantizer's out-of-range
    // conversion and the wrapping int sums, defined in the oracle)
    std::vector<double> xl(llr);
    xl[5] = INFINITY;
    xl[6] = -INFINITY;
    xl[(size_t)N + 7] = NAN;
    xl[(size_t)N + 8] = 1e300;
    for (int ialgo = 2; ialgo <= 5; ialgo++) {
        oracle_decode_int_batch(&o, xl.data(), B, iters, ialgo, 6, 0.5, 1, seed, 2, hard.data(), nullptr, ib.data(),
                                vb.data());
        for (int b = 0; b < B; b++)
            if ((ldpc::syndrome_host(g, hard.data() + (size_t)b * N, nullptr) == 0) != (vb[(size_t)b] != 0))
                mismatch("integer decoder valid flag vs syndrome");
        std::printf("ok decode-int algo=%d iters=%d valid=%d\n", ialgo, ib[0], vb[0]);
    }
    oracle_graph_free(&o);
    return 0;
}

void usage()
{
    std::fprintf(stderr, "usage: host_check pchk|alist|ints|doubles|fuzz-pchk|fuzz-alist|fuzz-text|repr|lattice|rs|"
                         "decode ...\n");
    std::exit(2);
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) usage();
    const std::string cmd = argv[1];
    auto need = [&](int n) {
        if (argc < n + 2) usage();
    };
    if (cmd == "pchk") { need(1); check_pchk(argv[2], true, false); }
    else if (cmd == "alist") { need(1); check_alist(argv[2], false); }
    else if (cmd == "ints") { need(3); do_ints(argv[2], std::strtoul(argv[3], nullptr, 10), std::atoi(argv[4]) != 0); }
    else if (cmd == "doubles") { need(2); do_doubles(argv[2], std::strtoul(argv[3], nullptr, 10)); }
    else if (cmd == "fuzz-pchk") { need(3); fuzz_pchk(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), argv[4]); }
    else if (cmd == "fuzz-alist") { need(3); fuzz_alist(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), argv[4]); }
    else if (cmd == "fuzz-text") { need(3); fuzz_text(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), argv[4]); }
    else if (cmd == "repr") { need(3); do_repr(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), argv[4]); }
    else if (cmd == "lattice") { need(1); do_lattice(std::strtoull(argv[2], nullptr, 10)); }
    else if (cmd == "rs") { do_rs(); }
    else if (cmd == "decode") {
        need(5);
        do_decode(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::strtoull(argv[5], nullptr, 10),
                  std::strtod(argv[6], nullptr));
    } else usage();
    return g_bad ? 3 : 0;
}
