// graph.hpp -- host-side parity-check graph (CSR + CSC edge arrays).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace ldpc {

// Sparse GF(2) parity-check matrix laid out once as flat edge arrays.
// Replaces the reference's doubly-linked mod2sparse lists (mod2sparse.h:42-93):
//   CSR (check-major) edge ids  e = row_ptr[i] + k, k ascending by column;
//   CSC col_edge[col_ptr[j] + s] = CSR edge id of the s-th entry of column j,
//   s ascending by row  -- exactly the traversal orders of
//   mod2sparse_first_in_row/next_in_row and first_in_col/next_in_col.
struct HostGraph {
    int32_t M = 0, N = 0;
    int64_t E = 0;
    std::vector<int32_t> row_ptr, col_idx, col_ptr, col_edge, edge_row;
    int32_t dv_max = 0, dc_max = 0;
    bool regular_dv = true, regular_dc = true;
};

// Parse a .pchk (rcode.cpp:54-85 / mod2sparse.cpp:381-427).  Returns an
// LDPC_* status and fills *msg on error.
int load_pchk(const std::string& path, HostGraph& g, std::string* msg);

// Build from (row, col) pairs with mod2sparse_insert ordering + dedup.
int build_graph(int32_t M, int32_t N, const int32_t* rows, const int32_t* cols, int64_t n,
                HostGraph& g, std::string* msg);

// check.cpp:28-45 on the host.
int syndrome_host(const HostGraph& g, const uint8_t* dblk, uint8_t* pchk);

}  // namespace ldpc
