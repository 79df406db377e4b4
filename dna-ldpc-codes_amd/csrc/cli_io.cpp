// cli_io.cpp -- see cli_io.hpp.
#include "cli_io.hpp"

#include <climits>
#include <cstdio>
#include <cstdlib>

namespace ldpc_cli {

static inline bool is_sep(unsigned char c)
{
    return c == ' ' || c == '\n' || c == '\r' || c == '\t' || c == '\v' || c == '\f';
}

bool read_tokens(const std::string& path, std::vector<std::string>& out, size_t need)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::string cur;
    bool in_tok = false;
    unsigned char buf[1 << 16];
    size_t got;
    while (out.size() < need && (got = std::fread(buf, 1, sizeof buf, f)) > 0) {
        for (size_t i = 0; i < got && out.size() < need; i++) {
            if (is_sep(buf[i])) {
                if (in_tok) { out.push_back(cur); cur.clear(); in_tok = false; }
            } else {
                in_tok = true;
                if (cur.size() < kMaxToken) cur.push_back((char)buf[i]);
                else cur.back() = '\x01';  // marks truncation: never a number
            }
        }
    }
    if (in_tok && out.size() < need) out.push_back(cur);
    std::fclose(f);
    return true;
}

bool parse_int(const std::string& tok, int* v)
{
    size_t p = 0;
    if (p < tok.size() && (tok[p] == '+' || tok[p] == '-')) p++;
    if (p >= tok.size()) return false;
    for (size_t i = p; i < tok.size(); i++)
        if (tok[i] < '0' || tok[i] > '9') return false;
    const long x = std::strtol(tok.c_str(), nullptr, 10);  // LONG_MIN / LONG_MAX out of range
    *v = x > INT_MAX ? INT_MAX : x < INT_MIN ? INT_MIN : (int)x;
    return true;
}

bool parse_double(const std::string& tok, double* v)
{
    if (tok.empty()) return false;
    char* end = nullptr;
    const double x = std::strtod(tok.c_str(), &end);
    if (end != tok.c_str() + tok.size()) return false;
    *v = x;  // overflow gives +-HUGE_VAL, as fscanf stores
    return true;
}

static std::string at(const std::string& path, size_t i)
{
    return path + ": token " + std::to_string(i + 1);
}

bool read_int_file(const std::string& path, size_t n, bool allow_short, std::vector<int>& out, std::string* msg)
{
    out.assign(n, 0);
    if (n == 0) return true;
    std::vector<std::string> tok;
    if (!read_tokens(path, tok, n)) {
        if (msg) *msg = "cannot open " + path;
        return false;
    }
    if (tok.size() < n && !allow_short) {
        if (msg) *msg = path + ": " + std::to_string(tok.size()) + " values, the code needs " + std::to_string(n);
        return false;
    }
    for (size_t i = 0; i < tok.size(); i++)
        if (!parse_int(tok[i], &out[i])) {
            if (msg) *msg = at(path, i) + " is not an integer";
            return false;
        }
    return true;
}

bool read_double_file(const std::string& path, size_t n, std::vector<double>& out, std::string* msg)
{
    out.assign(n, 0.0);
    if (n == 0) return true;
    std::vector<std::string> tok;
    if (!read_tokens(path, tok, n)) {
        if (msg) *msg = "cannot open " + path;
        return false;
    }
    if (tok.size() < n) {
        if (msg) *msg = path + ": " + std::to_string(tok.size()) + " values, the code needs " + std::to_string(n);
        return false;
    }
    for (size_t i = 0; i < n; i++)
        if (!parse_double(tok[i], &out[i])) {
            if (msg) *msg = at(path, i) + " is not a number";
            return false;
        }
    return true;
}

}  // namespace ldpc_cli
