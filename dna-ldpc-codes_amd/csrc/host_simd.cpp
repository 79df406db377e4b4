// host_simd.cpp -- host-side vector loops of the C ABI, built by the host
// compiler (not hipcc) so that target_clones can pick an AVX2 version at run
// time where the host has it; the default clone is the baseline x86-64 one.
// Both clones execute the same IEEE operations in the same order per
// element, so they produce the same codes.
#include "host_simd.hpp"


namespace ldpc {

// Branch-free (round to nearest by the 1.5 * 2^52 trick, |q| < 2^51 here), so
// the compiler vectorises it.
__attribute__((target_clones("avx2", "default"))) bool host_encode_lattice(const double* __restrict__ src,
                                                                             int8_t* __restrict__ code, size_t i0,
                                                                             size_t i1, double unit, int kmax,
                                                                             bool keep_neg_zero)
{
    const double inv = 1.0 / unit, magic = 6755399441055744.0, lim = kmax;
    // -0.0 compares equal to 0 * unit but is not its bits: off the lattice
    // when the decoder can see the sign of a zero (min-sum)
    const unsigned long long negz = keep_neg_zero ? 0x8000000000000000ull : 1ull;  // 1: a denormal, never k * unit
    int bad = 0;
    for (size_t i = i0; i < i1; i++) {
        const double x = src[i];
        const double kd = (x * inv + magic) - magic;
        bad |= (int)(kd * unit != x) | (int)!(kd <= lim && kd >= -lim) |
               (int)(__builtin_bit_cast(unsigned long long, x) == negz);
        // clamp with plain compares (vectorise to blends; fmin / fmax would be
        // library calls here): NaN becomes -lim, and such a value is flagged bad
        double kc = kd >= -lim ? kd : -lim;
        kc = kc <= lim ? kc : lim;
        code[i] = (int8_t)(int)kc;
    }
    return bad == 0;
}

}  // namespace ldpc
