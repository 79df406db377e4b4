// cli_io.hpp -- readers of the ldpc CLI's text inputs (codeword, soft and
// side files), host-only so that they also build under the sanitizer harness
// (tests/asan/host_check.cpp).
//
// The reference reads these with fscanf into fixed arrays, unchecked
// (DNA_main.cpp:1322-1345 codeword / soft files, SetUp :355-478 side files):
// a missing file is a NULL FILE*, a short file leaves earlier values, and a
// non-numeric token stalls every later fscanf.  Here every such case is an
// error with a message, except a short side file, which keeps the reference's
// calloc'd zeros (the SC-code multiplicities of a plain code are all 0).
#pragma once
#include <cstddef>
#include <string>
#include <vector>

namespace ldpc_cli {

// Longest token kept; longer ones are truncated and never parse (no fscanf
// number is this long).
constexpr size_t kMaxToken = 512;

// First `need` tokens of a file separated by space, tab, CR, LF, VT or FF.
// False when the file cannot be opened.
bool read_tokens(const std::string& path, std::vector<std::string>& out, size_t need);

// fscanf "%d" over a whole token: optional sign, decimal digits, nothing
// else.  Out-of-range values saturate to INT_MIN / INT_MAX (strtol's rule).
bool parse_int(const std::string& tok, int* v);

// fscanf "%lf" over a whole token (strtod: decimal, hex, inf, nan).
bool parse_double(const std::string& tok, double* v);

// n integers (codeword file, DNA_main.cpp:1322-1328).  allow_short: missing
// values are 0 (side files, SetUp :355-431).  Returns false with *msg set.
bool read_int_file(const std::string& path, size_t n, bool allow_short, std::vector<int>& out, std::string* msg);

// n doubles (soft file of channel LLRs, DNA_main.cpp:1335-1345).
bool read_double_file(const std::string& path, size_t n, std::vector<double>& out, std::string* msg);

}  // namespace ldpc_cli
