// dna_io.cpp -- soft-input files of the DNA pipeline (decoder.py:511-516 +
// def_func.write_codeword def_func.py:54-57): file i+1 holds bit i of every
// strand as `str(value) + ' '` tokens, no newline.  A value the reference
// never assigned a float to (int 0) is written "0"; a float is written the
// way Python's repr prints it (shortest round-trip digits, fixed notation for
// decimal exponents -4..15 with at least one fractional digit, otherwise
// d.ddde+XX).
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/ldpc_amd.h"
#include "host_io.hpp"

namespace ldpc {

// Python repr(float) (float_repr_style 'short').
size_t py_float_repr(double v, char* out)
{
    char* o = out;
    if (std::isnan(v)) { std::memcpy(o, "nan", 3); return 3; }
    if (std::signbit(v)) { *o++ = '-'; v = -v; }
    if (std::isinf(v)) { std::memcpy(o, "inf", 3); return (size_t)(o - out) + 3; }
    if (v == 0.0) { std::memcpy(o, "0.0", 3); return (size_t)(o - out) + 3; }
    char sci[64];
    auto r = std::to_chars(sci, sci + sizeof sci, v, std::chars_format::scientific);
    *r.ptr = 0;
    // sci = d[.ddd]e[+-]XX
    char digits[32];
    int nd = 0;
    const char* p = sci;
    for (; *p && *p != 'e'; p++)
        if (*p != '.') digits[nd++] = *p;
    const int e = std::atoi(p + 1);
    if (e >= -4 && e < 16) {
        if (e >= 0) {
            for (int i = 0; i <= e; i++) *o++ = i < nd ? digits[i] : '0';
            *o++ = '.';
            if (nd > e + 1) for (int i = e + 1; i < nd; i++) *o++ = digits[i];
            else *o++ = '0';
        } else {
            *o++ = '0';
            *o++ = '.';
            for (int i = 0; i < -e - 1; i++) *o++ = '0';
            for (int i = 0; i < nd; i++) *o++ = digits[i];
        }
    } else {
        *o++ = digits[0];
        if (nd > 1) {
            *o++ = '.';
            for (int i = 1; i < nd; i++) *o++ = digits[i];
        }
        o += std::snprintf(o, 8, "e%c%02d", e < 0 ? '-' : '+', e < 0 ? -e : e);
    }
    return (size_t)(o - out);
}

}  // namespace ldpc

using ldpc::set_error;

extern "C" {

int ldpc_write_soft_files(const char* dir, int32_t rs, const double* llr, const uint8_t* int_mask,
                          int32_t n_files, int32_t n_strands)
{
    if (!dir || !llr || n_files < 0 || n_strands < 0) {
        set_error("ldpc_write_soft_files: bad arguments");
        return LDPC_ERR_ARG;
    }
    std::string buf;
    buf.reserve((size_t)n_strands * 21);
    char tok[40];
    for (int32_t i = 0; i < n_files; i++) {
        buf.clear();
        const double* row = llr + (size_t)i * n_strands;
        const uint8_t* m = int_mask ? int_mask + (size_t)i * n_strands : nullptr;
        for (int32_t s = 0; s < n_strands; s++) {
            if (m && m[s]) {
                if (row[s] != 0.0) {
                    set_error("ldpc_write_soft_files: int-marked value is not 0");
                    return LDPC_ERR_ARG;
                }
                buf += "0 ";
            } else {
                const size_t n = ldpc::py_float_repr(row[s], tok);
                buf.append(tok, n);
                buf += ' ';
            }
        }
        char name[64];
        std::snprintf(name, sizeof name, "/soft%d_n18432_m1860_%d.txt", rs, i + 1);  // decoder.py:515
        const std::string path = std::string(dir) + name;
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) {
            set_error("can't create " + path);
            return LDPC_ERR_IO;
        }
        const bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
        if (std::fclose(f) != 0 || !ok) {
            set_error("error writing " + path);
            return LDPC_ERR_IO;
        }
    }
    return LDPC_OK;
}

int ldpc_py_float_repr(double v, char* out, int32_t cap)
{
    char tok[40];
    const size_t n = ldpc::py_float_repr(v, tok);
    if (!out || cap < (int32_t)n + 1) {
        set_error("ldpc_py_float_repr: buffer too small");
        return LDPC_ERR_ARG;
    }
    std::memcpy(out, tok, n);
    out[n] = 0;
    return (int)n;
}

}  // extern "C"
