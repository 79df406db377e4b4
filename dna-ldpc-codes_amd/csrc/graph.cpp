// graph.cpp -- .pchk reader and CSR/CSC edge-array builder.
//
// Reference behaviour reproduced (LDPC_dec/ldpc/):
//   * intio_read (intio.cpp:35-50): 4-byte little-endian two's complement.
//   * read_pchk  (rcode.cpp:54-85): magic ('P'<<8)+0x80, then mod2sparse_read.
//   * mod2sparse_read (mod2sparse.cpp:381-427): M, N > 0; records: negative
//     v selects row -v-1, positive v inserts column v-1 into the current row,
//     0 terminates; out-of-range rows/cols, a column before any row, or EOF
//     before the terminator are errors.
//   * mod2sparse_insert (mod2sparse.cpp:502-604): row lists ascend by column,
//     column lists ascend by row, duplicate entries are ignored.
// Unlike the reference, errors are returned (no exit()) and the whole file
// is read with one fread instead of ~150k 1-byte freads.
#include "graph.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <set>

#include "../../include/ldpc_amd.h"

namespace ldpc {

static inline int32_t le32(const unsigned char* b)
{
    uint32_t u = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    return (int32_t)u;
}

int build_graph(int32_t M, int32_t N, const int32_t* rows, const int32_t* cols, int64_t n,
                HostGraph& g, std::string* msg)
{
    if (M <= 0 || N <= 0 || n < 0) {
        if (msg) *msg = "graph dimensions must be positive";
        return LDPC_ERR_ARG;
    }
    if (M > LDPC_MAX_DIM || N > LDPC_MAX_DIM) {
        if (msg) *msg = "graph dimensions above LDPC_MAX_DIM";
        return LDPC_ERR_UNSUPPORTED;
    }
    std::vector<uint64_t> key((size_t)n);
    for (int64_t i = 0; i < n; i++) {
        if (rows[i] < 0 || rows[i] >= M || cols[i] < 0 || cols[i] >= N) {
            if (msg) *msg = "row or column index out of bounds";  // mod2sparse.cpp:511-515
            return LDPC_ERR_FORMAT;
        }
        key[(size_t)i] = ((uint64_t)(uint32_t)rows[i] << 32) | (uint32_t)cols[i];
    }
    std::sort(key.begin(), key.end());
    key.erase(std::unique(key.begin(), key.end()), key.end());
    const int64_t E = (int64_t)key.size();
    if (E > INT32_MAX) {
        if (msg) *msg = "too many edges";
        return LDPC_ERR_UNSUPPORTED;
    }
    g = HostGraph{};
    g.M = M; g.N = N; g.E = E;
    g.row_ptr.assign((size_t)M + 1, 0);
    g.col_ptr.assign((size_t)N + 1, 0);
    g.col_idx.resize((size_t)E);
    g.edge_row.resize((size_t)E);
    g.col_edge.resize((size_t)E);
    for (int64_t e = 0; e < E; e++) {
        int32_t r = (int32_t)(key[(size_t)e] >> 32), c = (int32_t)(key[(size_t)e] & 0xffffffffu);
        g.row_ptr[(size_t)r + 1]++;
        g.col_ptr[(size_t)c + 1]++;
        g.col_idx[(size_t)e] = c;
        g.edge_row[(size_t)e] = r;
    }
    for (int32_t i = 0; i < M; i++) g.row_ptr[(size_t)i + 1] += g.row_ptr[(size_t)i];
    for (int32_t j = 0; j < N; j++) g.col_ptr[(size_t)j + 1] += g.col_ptr[(size_t)j];
    std::vector<int32_t> fill(g.col_ptr.begin(), g.col_ptr.end() - 1);
    for (int64_t e = 0; e < E; e++) g.col_edge[(size_t)fill[(size_t)g.col_idx[(size_t)e]]++] = (int32_t)e;

    // CheckRegular (dec.cpp:138-189)
    g.dv_max = -1; g.dc_max = -1; g.regular_dv = true; g.regular_dc = true;
    for (int32_t j = 0; j < N; j++) {
        int32_t t = g.col_ptr[(size_t)j + 1] - g.col_ptr[(size_t)j];
        if (g.dv_max == -1) g.dv_max = t;
        else { if (t != g.dv_max) g.regular_dv = false; if (t > g.dv_max) g.dv_max = t; }
    }
    for (int32_t i = 0; i < M; i++) {
        int32_t t = g.row_ptr[(size_t)i + 1] - g.row_ptr[(size_t)i];
        if (g.dc_max == -1) g.dc_max = t;
        else { if (t != g.dc_max) g.regular_dc = false; if (t > g.dc_max) g.dc_max = t; }
    }
    return LDPC_OK;
}

int load_pchk(const std::string& path, HostGraph& g, std::string* msg)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        if (msg) *msg = "Can't open parity check file: " + path;  // rcode.cpp:62-64
        return LDPC_ERR_IO;
    }
    std::vector<unsigned char> buf;
    unsigned char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    std::fclose(f);

    const size_t nwords = buf.size() / 4;  // a trailing partial word reads as EOF
    size_t pos = 0;
    auto next = [&](int32_t* v) -> bool {
        if (pos >= nwords) return false;
        *v = le32(&buf[4 * pos++]);
        return true;
    };
    int32_t magic = 0;
    if (!next(&magic) || magic != ('P' << 8) + 0x80) {
        if (msg) *msg = "File " + path + " doesn't contain a parity check matrix";  // rcode.cpp:67-71
        return LDPC_ERR_FORMAT;
    }
    int32_t M = 0, N = 0;
    if (!next(&M) || M <= 0 || !next(&N) || N <= 0) {
        if (msg) *msg = "Error reading parity check matrix from " + path;  // rcode.cpp:75-79
        return LDPC_ERR_FORMAT;
    }
    if (M > LDPC_MAX_DIM || N > LDPC_MAX_DIM) {
        if (msg) *msg = "Parity check matrix in " + path + " is larger than LDPC_MAX_DIM";
        return LDPC_ERR_UNSUPPORTED;
    }
    std::vector<int32_t> rows, cols;
    rows.reserve(nwords);
    cols.reserve(nwords);
    int32_t row = -1;
    bool ok = false;
    for (;;) {
        int32_t v;
        if (!next(&v)) break;
        if (v == 0) { ok = true; break; }
        if (v < 0) {
            if (v == INT32_MIN) break;
            row = -v - 1;
            if (row >= M) break;
        } else {
            int32_t col = v - 1;
            if (col >= N || row == -1) break;
            rows.push_back(row);
            cols.push_back(col);
        }
    }
    if (!ok) {
        if (msg) *msg = "Error reading parity check matrix from " + path;
        return LDPC_ERR_FORMAT;
    }
    return build_graph(M, N, rows.data(), cols.data(), (int64_t)rows.size(), g, msg);
}

int syndrome_host(const HostGraph& g, const uint8_t* dblk, uint8_t* pchk)
{
    int c = 0;
    for (int32_t i = 0; i < g.M; i++) {
        uint8_t p = 0;
        for (int32_t e = g.row_ptr[(size_t)i]; e < g.row_ptr[(size_t)i + 1]; e++) p ^= (dblk[g.col_idx[(size_t)e]] != 0);
        if (pchk) pchk[i] = p;
        c += p;
    }
    return c;
}

// ---------------------------------------------------------------------------
// alist / pchk writers and the alist reader
// ---------------------------------------------------------------------------

namespace {

// fscanf("%d") on a whitespace-separated stream: 1 = got a value, 0 = a
// non-numeric token (not EOF), -1 = end of input.
struct IntScanner {
    std::vector<char> buf;
    size_t pos = 0;
    int next(int* v)
    {
        while (pos < buf.size() && std::isspace((unsigned char)buf[pos])) pos++;
        if (pos >= buf.size()) return -1;
        size_t p = pos;
        if (buf[p] == '+' || buf[p] == '-') p++;
        if (p >= buf.size() || !std::isdigit((unsigned char)buf[p])) return 0;
        long long x = 0;
        const bool neg = buf[pos] == '-';
        while (p < buf.size() && std::isdigit((unsigned char)buf[p])) {
            x = x * 10 + (buf[p] - '0');
            if (x > 0x7fffffffLL) x = 0x7fffffffLL;
            p++;
        }
        pos = p;
        *v = (int)(neg ? -x : x);
        return 1;
    }
};

bool write_le32(FILE* f, int32_t v)
{
    const uint32_t u = (uint32_t)v;
    const unsigned char b[4] = {(unsigned char)(u & 0xff), (unsigned char)((u >> 8) & 0xff),
                                (unsigned char)((u >> 16) & 0xff), (unsigned char)((u >> 24) & 0xff)};
    return std::fwrite(b, 1, 4, f) == 4;
}

}  // namespace

int load_alist(const std::string& path, bool transpose, HostGraph& g, std::string* msg)
{
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) {
        if (msg) *msg = "Can't open alist file: " + path;  // alist-to-pchk.cpp:72-76
        return LDPC_ERR_IO;
    }
    IntScanner sc;
    char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) sc.buf.insert(sc.buf.end(), tmp, tmp + got);
    std::fclose(f);
    auto bad = [&]() {
        if (msg) *msg = "Alist file doesn't have the right format";  // bad_alist_file :164-168
        return LDPC_ERR_FORMAT;
    };
    int M, N, mxrw, mxcw;
    if (sc.next(&M) != 1 || M < 1 || sc.next(&N) != 1 || N < 1 || sc.next(&mxrw) != 1 || mxrw < 0 || mxrw > N ||
        sc.next(&mxcw) != 1 || mxcw < 0 || mxcw > M)
        return bad();
    // the M + N degrees that follow take two bytes each at least: a header
    // larger than the file cannot be right, and must not size the allocations
    if ((size_t)M + (size_t)N > sc.buf.size() / 2) return bad();
    std::vector<int> rw((size_t)M), cw((size_t)N);
    for (int i = 0; i < M; i++)
        if (sc.next(&rw[(size_t)i]) != 1 || rw[(size_t)i] < 0 || rw[(size_t)i] > N) return bad();
    for (int j = 0; j < N; j++)
        if (sc.next(&cw[(size_t)j]) != 1 || cw[(size_t)j] < 0 || cw[(size_t)j] > M) return bad();
    std::set<std::pair<int, int>> ent;
    std::vector<int32_t> rows, cols;
    long long tot = 0;
    for (int i = 0; i < M; i++) {
        for (int k = 0; k < mxrw; k++) {
            int j;
            if (sc.next(&j) != 1 || j < 0 || j > N || (k >= rw[(size_t)i] && j != 0) || (k < rw[(size_t)i] && j == 0))
                return bad();
            if (j == 0) continue;
            if (!ent.insert({i, j - 1}).second) return bad();  // duplicate (mod2sparse_find)
            rows.push_back(i);
            cols.push_back(j - 1);
            tot++;
        }
    }
    for (int j = 0; j < N; j++) {
        for (int k = 0; k < mxcw; k++) {
            int i;
            if (sc.next(&i) != 1 || i < 0 || i > M || (k >= cw[(size_t)j] && i != 0) || (k < cw[(size_t)j] && i == 0))
                return bad();
            if (i == 0) continue;
            if (!ent.count({i - 1, j})) return bad();
            tot--;
        }
    }
    if (tot != 0) return bad();
    int extra;
    if (sc.next(&extra) != -1) return bad();  // more numbers, or trailing garbage
    if (transpose) return build_graph(N, M, cols.data(), rows.data(), (int64_t)rows.size(), g, msg);
    return build_graph(M, N, rows.data(), cols.data(), (int64_t)rows.size(), g, msg);
}

int save_pchk(const HostGraph& g, const std::string& path, std::string* msg)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) {
        if (msg) *msg = "Can't create parity check file: " + path;
        return LDPC_ERR_IO;
    }
    bool ok = write_le32(f, ('P' << 8) + 0x80) && write_le32(f, g.M) && write_le32(f, g.N);
    for (int32_t i = 0; ok && i < g.M; i++) {
        const int32_t a = g.row_ptr[(size_t)i], b = g.row_ptr[(size_t)i + 1];
        if (a == b) continue;  // empty rows are not written (mod2sparse.cpp:357-359)
        ok = write_le32(f, -(i + 1));
        for (int32_t e = a; ok && e < b; e++) ok = write_le32(f, g.col_idx[(size_t)e] + 1);
    }
    ok = ok && write_le32(f, 0);
    if (std::fclose(f) != 0) ok = false;
    if (!ok) {
        if (msg) *msg = "Error writing to parity check file " + path;
        return LDPC_ERR_IO;
    }
    return LDPC_OK;
}

int save_alist(const HostGraph& g, const std::string& path, std::string* msg)
{
    // Layout of the alist files RS_LDPC.c:434-474 writes (every number
    // followed by a space, one line per list), zero-padded to the maximum
    // degree for irregular graphs as alist-to-pchk.cpp:104-124 expects.
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) {
        if (msg) *msg = "Can't create alist file: " + path;
        return LDPC_ERR_IO;
    }
    const int mxrw = std::max(0, g.dc_max), mxcw = std::max(0, g.dv_max);
    std::fprintf(f, "%d %d\n%d %d\n", g.M, g.N, mxrw, mxcw);
    for (int32_t i = 0; i < g.M; i++) std::fprintf(f, "%d ", g.row_ptr[(size_t)i + 1] - g.row_ptr[(size_t)i]);
    std::fprintf(f, "\n");
    for (int32_t j = 0; j < g.N; j++) std::fprintf(f, "%d ", g.col_ptr[(size_t)j + 1] - g.col_ptr[(size_t)j]);
    std::fprintf(f, "\n");
    for (int32_t i = 0; i < g.M; i++) {
        int k = 0;
        for (int32_t e = g.row_ptr[(size_t)i]; e < g.row_ptr[(size_t)i + 1]; e++, k++)
            std::fprintf(f, "%d ", g.col_idx[(size_t)e] + 1);
        for (; k < mxrw; k++) std::fprintf(f, "0 ");
        std::fprintf(f, "\n");
    }
    for (int32_t j = 0; j < g.N; j++) {
        int k = 0;
        for (int32_t q = g.col_ptr[(size_t)j]; q < g.col_ptr[(size_t)j + 1]; q++, k++)
            std::fprintf(f, "%d ", g.edge_row[(size_t)g.col_edge[(size_t)q]] + 1);
        for (; k < mxcw; k++) std::fprintf(f, "0 ");
        std::fprintf(f, "\n");
    }
    if (std::fclose(f) != 0) {
        if (msg) *msg = "Error writing alist file " + path;
        return LDPC_ERR_IO;
    }
    return LDPC_OK;
}

// ---------------------------------------------------------------------------
// RS-based LDPC construction (RS_LDPC.c)
// ---------------------------------------------------------------------------
//
// GF(2^s) elements are carried as exponents (alpha^k, -1 = zero) exactly as
// in the reference; addition goes through an antilog/log table pair instead
// of its linear search over gf_table (RS_LDPC.c:119-160), which yields the
// same exponent because the primitive polynomials make alpha^0..alpha^(q-2)
// distinct.  Codewords are generated on the fly, and the reference's search
// for "the first codeword equal to this coset row" (RS_LDPC.c:334-347,
// 368-382) is an O(rho) solve: codeword index (a+1)*q + (b+1) has
// a = cw[0] / g1[0] and b = cw[rho-1] / g2[rho-1], then a full compare.

namespace {

struct RsField {
    int s = 0, q = 0, level = 0;
    std::vector<int> tab, log;  // tab[k] = bit vector of alpha^k; log[vec] = k

    bool init(int s_)
    {
        // RS_LDPC.c:14-93 polynominal(): low-order coefficients p0..p(s-1)
        static const unsigned poly[11] = {0, 0, 0x3, 0x3, 0x3, 0x5, 0x3, 0x9, 0x1d, 0x11, 0x9};
        if (s_ < 2 || s_ > 10) return false;
        s = s_;
        q = 1 << s;
        level = q - 1;
        tab.assign((size_t)level, 0);
        log.assign((size_t)q, -1);
        tab[0] = 1;  // RS_LDPC.c:95-117 make_table()
        for (int i = 1; i < level; i++) {
            int v = (tab[(size_t)i - 1] << 1) & (q - 1);
            if (tab[(size_t)i - 1] & (1 << (s - 1))) v ^= (int)poly[s];
            tab[(size_t)i] = v;
        }
        for (int i = 0; i < level; i++) {
            if (log[(size_t)tab[(size_t)i]] != -1) return false;
            log[(size_t)tab[(size_t)i]] = i;
        }
        return true;
    }
    int add(int i, int j) const  // gf_add, RS_LDPC.c:119-160 (C % semantics)
    {
        if (i == -1) return j % level;
        if (j == -1) return i % level;
        i %= level;
        j %= level;
        if (i == j) return -1;
        return log[(size_t)(tab[(size_t)i] ^ tab[(size_t)j])];
    }
    int mult(int i, int j) const { return (i == -1 || j == -1) ? -1 : (i + j) % level; }  // :162-174
    int div(int a, int b) const { return ((a - b) % level + level) % level; }  // alpha^a / alpha^b
};

}  // namespace

int build_rs_ldpc(int s, int rho, int gamma, HostGraph& g, std::vector<int>* gen_poly_out,
                  std::vector<int>* coset_out, std::string* msg)
{
    auto arg = [&](const char* m) {
        if (msg) *msg = m;
        return LDPC_ERR_ARG;
    };
    RsField F;
    if (!F.init(s)) return arg("RS-LDPC: s must be in 2..10 (RS_LDPC.c:14-93 polynomial table)");
    const int q = F.q;
    if (rho < 3 || rho > q) return arg("RS-LDPC: rho must be in 3..2^s");
    if (gamma < 1 || gamma > q) return arg("RS-LDPC: gamma must be in 1..2^s");

    // generator polynomial (x+alpha)(x+alpha^2)... (RS_LDPC.c:176-200)
    std::vector<int> gp((size_t)rho, 0);  // one spare slot: poly[n+1] is written at n = rho-3
    gp[0] = 1;
    gp[1] = 0;
    for (int i = 1; i < rho - 2; i++) {
        const int b = 1 + i, n = i;
        gp[(size_t)n + 1] = gp[(size_t)n];
        for (int k = n; k > 0; k--) gp[(size_t)k] = F.add(gp[(size_t)k - 1], F.mult(b, gp[(size_t)k]));
        gp[0] = F.mult(b, gp[0]);
    }
    gp.resize((size_t)rho - 1);
    std::vector<int> g1((size_t)rho, 0), g2((size_t)rho, 0);  // RS_LDPC.c:316-324
    for (int i = 0; i < rho - 1; i++) {
        g1[(size_t)i] = gp[(size_t)i];
        g2[(size_t)i + 1] = gp[(size_t)i];
    }
    g1[(size_t)rho - 1] = -1;
    g2[0] = -1;
    if (g1[0] == -1 || g2[(size_t)rho - 1] == -1) return arg("RS-LDPC: degenerate generator polynomial");

    auto codeword = [&](int idx, int* out) {  // encode(), RS_LDPC.c:202-217
        const int a = idx / q - 1, b = idx % q - 1;
        for (int k = 0; k < rho; k++) out[k] = F.add(F.mult(a, g1[(size_t)k]), F.mult(b, g2[(size_t)k]));
    };
    std::vector<int> tmp((size_t)rho);
    auto find = [&](const int* v) -> int {  // index of the codeword equal to v, or -1
        const int a = v[0] == -1 ? -1 : F.div(v[0], g1[0]);
        const int b = v[rho - 1] == -1 ? -1 : F.div(v[rho - 1], g2[(size_t)rho - 1]);
        const int idx = (a + 1) * q + (b + 1);
        codeword(idx, tmp.data());
        for (int k = 0; k < rho; k++)
            if (tmp[(size_t)k] != v[k]) return -1;
        return idx;
    };

    const int64_t ncw = (int64_t)q * q;
    int selected = -1;
    std::vector<int> cw((size_t)rho);
    for (int64_t i = 0; i < ncw && selected < 0; i++) {  // RS_LDPC.c:311-329
        codeword((int)i, cw.data());
        int cnt = 0;
        for (int k = 0; k < rho; k++) cnt += cw[(size_t)k] != -1;
        if (cnt == rho) selected = (int)i;
    }
    if (selected < 0) return arg("RS-LDPC: no codeword of full weight rho");
    std::vector<int> coset((size_t)ncw, -1);
    std::vector<int> Cb((size_t)gamma * q * rho);
    codeword(selected, cw.data());
    for (int i = 0; i < q; i++)  // RS_LDPC.c:331-336
        for (int k = 0; k < rho; k++) Cb[(size_t)i * rho + k] = F.mult(i - 1, cw[(size_t)k]);
    for (int i = 0; i < q; i++) {
        const int idx = find(&Cb[(size_t)i * rho]);
        if (idx >= 0) coset[(size_t)idx] = 0;
    }
    for (int c = 1; c < gamma; c++) {  // RS_LDPC.c:352-385
        selected = -1;
        for (int64_t j = 0; j < ncw; j++)
            if (coset[(size_t)j] == -1) { selected = (int)j; break; }
        if (selected < 0) return arg("RS-LDPC: ran out of cosets");
        codeword(selected, cw.data());
        for (int j = 0; j < q; j++)
            for (int k = 0; k < rho; k++)
                Cb[((size_t)j + (size_t)c * q) * rho + k] = F.add(Cb[(size_t)j * rho + k], cw[(size_t)k]);
        for (int j = 0; j < q; j++) {
            const int idx = find(&Cb[((size_t)j + (size_t)c * q) * rho]);
            if (idx >= 0) coset[(size_t)idx] = c;
        }
    }
    // H[i][j*q + Cb[i][j] + 1] = 1 (RS_LDPC.c:389-398)
    const int M = gamma * q, N = rho * q;
    std::vector<int32_t> rows((size_t)M * rho), cols((size_t)M * rho);
    for (int i = 0; i < M; i++)
        for (int k = 0; k < rho; k++) {
            rows[(size_t)i * rho + k] = i;
            cols[(size_t)i * rho + k] = k * q + Cb[(size_t)i * rho + k] + 1;
        }
    if (gen_poly_out) *gen_poly_out = gp;
    if (coset_out) *coset_out = std::move(coset);
    return build_graph(M, N, rows.data(), cols.data(), (int64_t)rows.size(), g, msg);
}

namespace {

// cls[j] = column block of column j: every row must hold exactly one column of
// every block, and every block Q columns
bool check_col_blocks(const HostGraph& g, const std::vector<int32_t>& cls, int32_t RB, int32_t Q)
{
    std::vector<int32_t> cnt((size_t)RB, 0);
    for (int32_t j = 0; j < g.N; j++) {
        if (cls[(size_t)j] < 0 || cls[(size_t)j] >= RB) return false;
        cnt[(size_t)cls[(size_t)j]]++;
    }
    for (int32_t b = 0; b < RB; b++)
        if (cnt[(size_t)b] != Q) return false;
    std::vector<int32_t> seen((size_t)RB, -1);
    for (int32_t i = 0; i < g.M; i++)
        for (int32_t e = g.row_ptr[(size_t)i]; e < g.row_ptr[(size_t)i + 1]; e++) {
            const int32_t b = cls[(size_t)g.col_idx[(size_t)e]];
            if (seen[(size_t)b] == i) return false;
            seen[(size_t)b] = i;
        }
    return true;
}

}  // namespace

bool find_block_layout(const HostGraph& g, BlockLayout& L)
{
    if (!g.regular_dv || !g.regular_dc || g.dv_max < 1 || g.dc_max < 2) return false;
    const int32_t GA = g.dv_max, RB = g.dc_max;
    if (g.M % GA != 0) return false;
    const int32_t Q = g.M / GA;
    if ((int64_t)g.N != (int64_t)RB * Q) return false;
    // row blocks: rows a*Q .. a*Q+Q-1 cover every column exactly once
    std::vector<int32_t> seen((size_t)g.N, -1);
    for (int32_t i = 0; i < g.M; i++)
        for (int32_t e = g.row_ptr[(size_t)i]; e < g.row_ptr[(size_t)i + 1]; e++) {
            const int32_t j = g.col_idx[(size_t)e];
            if (seen[(size_t)j] == i / Q) return false;
            seen[(size_t)j] = i / Q;
        }
    // column blocks: contiguous blocks of Q columns, else the blocks of the
    // RS-LDPC code (build_rs_ldpc) with the same rows, matched by row sets
    std::vector<int32_t> cls((size_t)g.N);
    for (int32_t j = 0; j < g.N; j++) cls[(size_t)j] = j / Q;
    if (!check_col_blocks(g, cls, RB, Q)) {
        int s = 0;
        while ((1 << s) < Q) s++;
        HostGraph rs;
        if ((1 << s) != Q || build_rs_ldpc(s, RB, GA, rs, nullptr, nullptr, nullptr) != LDPC_OK) return false;
        if (rs.M != g.M || rs.N != g.N) return false;
        std::map<std::vector<int32_t>, int32_t> key;
        std::vector<int32_t> k((size_t)GA);
        for (int32_t j = 0; j < rs.N; j++) {
            for (int32_t s2 = 0; s2 < GA; s2++)
                k[(size_t)s2] = rs.edge_row[(size_t)rs.col_edge[(size_t)rs.col_ptr[(size_t)j] + s2]];
            key[k] = j;
        }
        for (int32_t j = 0; j < g.N; j++) {
            for (int32_t s2 = 0; s2 < GA; s2++)
                k[(size_t)s2] = g.edge_row[(size_t)g.col_edge[(size_t)g.col_ptr[(size_t)j] + s2]];
            auto it = key.find(k);
            if (it == key.end()) return false;
            cls[(size_t)j] = it->second / Q;
        }
        if (!check_col_blocks(g, cls, RB, Q)) return false;
    }
    // position of each column inside its block (ascending column index)
    std::vector<int32_t> fill((size_t)RB, 0);
    L.Q = Q;
    L.GA = GA;
    L.RB = RB;
    L.col_orig.assign((size_t)RB * Q, 0);
    for (int32_t j = 0; j < g.N; j++) {
        const int32_t b = cls[(size_t)j];
        L.col_orig[(size_t)b * Q + fill[(size_t)b]++] = j;
    }
    return true;
}

const BlockLayout* block_layout_of(const HostGraph& g)
{
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (g.blk_state == 0) {
        auto L = std::make_shared<BlockLayout>();
        g.blk_state = find_block_layout(g, *L) ? 1 : -1;
        if (g.blk_state > 0) g.blk_cache = L;
    }
    return g.blk_state > 0 ? g.blk_cache.get() : nullptr;
}

}  // namespace ldpc
