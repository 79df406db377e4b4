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
#include <cstdio>
#include <cstring>

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

}  // namespace ldpc
