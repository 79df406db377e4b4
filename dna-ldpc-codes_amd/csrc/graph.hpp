// graph.hpp -- host-side parity-check graph (CSR + CSC edge arrays).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace ldpc {

struct BlockLayout;

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
    // block structure (block_layout_of), found once per graph
    mutable int blk_state = 0;  // 0 not looked for, 1 found, -1 none
    mutable std::shared_ptr<BlockLayout> blk_cache;
};

// Parse a .pchk (rcode.cpp:54-85 / mod2sparse.cpp:381-427).  Returns an
// LDPC_* status and fills *msg on error.
int load_pchk(const std::string& path, HostGraph& g, std::string* msg);

// Build from (row, col) pairs with mod2sparse_insert ordering + dedup.
int build_graph(int32_t M, int32_t N, const int32_t* rows, const int32_t* cols, int64_t n,
                HostGraph& g, std::string* msg);

// check.cpp:28-45 on the host.
int syndrome_host(const HostGraph& g, const uint8_t* dblk, uint8_t* pchk);

// alist -> graph with the validation rules of alist-to-pchk.cpp:36-160
// (transpose = its -t option).
int load_alist(const std::string& path, bool transpose, HostGraph& g, std::string* msg);

// graph -> .pchk: magic, then mod2sparse_write (mod2sparse.cpp:338-376):
// M, N, for every non-empty row -(i+1) and its columns+1, terminator 0.
int save_pchk(const HostGraph& g, const std::string& path, std::string* msg);

// graph -> alist (the format alist-to-pchk reads; rows then columns, 1-based,
// zero-padded to the maximum degree).
int save_alist(const HostGraph& g, const std::string& path, std::string* msg);

// RS-based LDPC code of RS_LDPC.c (RS LDPC encode/RS_LDPC/RS_LDPC.c:221-431):
// q = 2^s, M = gamma*q, N = rho*q.  gen_poly (rho-1 exponents, -1 = zero) and
// coset (q*q entries) are the tables its H_pri=0 mode prints; either may be null.
int build_rs_ldpc(int s, int rho, int gamma, HostGraph& g, std::vector<int>* gen_poly,
                  std::vector<int>* coset, std::string* msg);

// Block structure of array (RS / quasi-cyclic) codes (ldpc_graph_blocks):
// rows in GA = dv contiguous blocks of Q, columns in RB = dc blocks of Q,
// every (row block, column block) submatrix a Q x Q permutation.
struct BlockLayout {
    int32_t Q = 0, GA = 0, RB = 0;
    std::vector<int32_t> col_orig;  // [RB][Q]: column index of position jp of column block b (ascending)
};

// Column blocks: contiguous blocks of Q, else the RS-LDPC(log2 Q, dc, dv)
// code's blocks when H is that code with permuted columns.  False when H has
// no such structure.
bool find_block_layout(const HostGraph& g, BlockLayout& L);

// find_block_layout once per graph (thread-safe); nullptr when H has no such structure
const BlockLayout* block_layout_of(const HostGraph& g);

}  // namespace ldpc
