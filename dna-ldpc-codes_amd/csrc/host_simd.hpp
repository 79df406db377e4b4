// host_simd.hpp -- host-side vector loops of the C ABI (compiled by the host
// compiler alone, with run-time ISA dispatch).
#pragma once
#include <cstddef>
#include <cstdint>

namespace ldpc {

// code[i] = k for src[i] == k * unit exactly, |k| <= kmax, i in [i0, i1);
// false when some value is not on that lattice (the LR table path of
// ldpc_decode, capi.cpp).  With keep_neg_zero, -0.0 counts as off the lattice
// (min-sum sums keep the sign of a zero; BP's exp(-0.0) == exp(0.0)).
bool host_encode_lattice(const double* __restrict__ src, int8_t* __restrict__ code, size_t i0, size_t i1, double unit,
                         int kmax, bool keep_neg_zero);

}  // namespace ldpc
