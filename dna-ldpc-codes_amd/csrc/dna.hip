// dna.hip -- the step before the decoder: per-strand
// read candidates -> the 272 x 18432 LLR matrix the first decode consumes,
// plus the pairwise edit distances that pick which ragged candidates go to
// the aligner.
//
// Reference: ex_decoder/decoder.py:142-519 (the strand loop; count rule
// :266-320 and :442-497), def_func.py:10-26 (edit_dist), :97-117
// (DNA2binary).  The host mirror (dna_llr.py) classifies every strand into a
// `kind` and lays the candidates out as fixed-width rows; these kernels do
// the arithmetic:
//
//   kind 0  no LLRs              -> every bit int 0 (decoder.py:507-510 fill)
//   kind 1  count                -> bit b: (count0 - count1) * L over the rows,
//                                   bit 2*nt-1 skips rows with q < 53 and has
//                                   the one-vs-one tie rule (:290-299)
//   kind 2  one short candidate  -> only the last bit: +-L from the low bit of
//                                   the candidate's last base if q > 63 (:247-251)
//   kind 3  alignment failed     -> only the last bit: (count0 - count1) * L
//                                   over the failed rows' last bases with
//                                   q > 63 (:266-282)
//
// Bit values follow DNA2binary: A=00 C=01 G=10 T=11, any other character
// gives '2', which the count loop treats as a one (it tests == '0').
// Arithmetic is the reference's: (double)(c0 - c1) * L, +-2 * L, +-L.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ldpc_amd.h"
#include "engine.hpp"

namespace ldpc {
namespace {

constexpr int kQSkip = 53;  // decoder.py:285 (i==271 and q < 53: skip)
constexpr int kQHigh = 63;  // decoder.py:247, :270, :292-295

// DNA2binary bit of character c: hi = first bit, else second bit.
// Returns true when the bit is '0'.
__device__ __forceinline__ bool bit_is_zero(uint8_t c, bool hi)
{
    if (hi) return c == 'A' || c == 'C';
    return c == 'A' || c == 'G';
}

// Every entry is k * L for an integer count difference k (decoder.py:297-314;
// the +-2L / +-L special cases included), so the kernel can hand the decoder
// its int8 codes directly (codes != nullptr): k saturated to [-127, 127], and
// *overflow set (a plain store of 1) when some |k| > 127.
__global__ void __launch_bounds__(256) k_dna_llr(const int32_t* __restrict__ kind, const int64_t* __restrict__ row_ptr,
                                                 const uint8_t* __restrict__ rows, const int32_t* __restrict__ row_q,
                                                 int32_t S, int32_t nt, double L, double* __restrict__ llr,
                                                 uint8_t* __restrict__ int_mask, int8_t* __restrict__ codes,
                                                 int32_t* __restrict__ overflow)
{
    const int32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t k = blockIdx.y;  // nucleotide -> bits 2k, 2k+1
    if (s >= S) return;
    const int kd = kind[s];
    const int64_t r0 = row_ptr[s], r1 = row_ptr[s + 1];
    const int last_bit = 2 * nt - 1;
    for (int h = 0; h < 2; h++) {
        const int b = 2 * k + h;
        int n = 0;  // the count difference: the entry is n * L (0 for an int-0 entry)
        bool is_int = true;
        if (kd == 1) {
            int c0 = 0, c1 = 0, q0 = 0, q1 = 0;
            for (int64_t r = r0; r < r1; r++) {
                const int q = row_q[r];
                if (b == last_bit && q < kQSkip) continue;
                if (bit_is_zero(rows[r * nt + k], h == 0)) { c0++; q0 += q; }
                else { c1++; q1 += q; }
            }
            if (b == last_bit && c0 == 1 && c1 == 1) {
                if (q0 < kQSkip && q1 >= kQHigh) { n = -2; is_int = false; }
                else if (q0 >= kQHigh && q1 < kQSkip) { n = 2; is_int = false; }
            } else {
                n = c0 - c1;
                is_int = false;
            }
        } else if (kd == 2 && b == last_bit && r1 > r0) {
            if (row_q[r0] > kQHigh) {
                n = bit_is_zero(rows[r0 * nt], false) ? 1 : -1;
                is_int = false;
            }
        } else if (kd == 3 && b == last_bit) {
            int c0 = 0, c1 = 0;
            for (int64_t r = r0; r < r1; r++) {
                if (row_q[r] <= kQHigh) continue;
                if (bit_is_zero(rows[r * nt], false)) c0++;
                else c1++;
            }
            n = c0 - c1;
            is_int = false;
        }
        // (double)n * L: the reference's (count_0 - count_1) * math.log(...),
        // and 2.0 * L, L, -L for the special cases -- the same doubles
        llr[(size_t)b * S + s] = is_int ? 0.0 : (double)n * L;
        if (int_mask) int_mask[(size_t)b * S + s] = is_int;
        if (codes) {
            codes[(size_t)b * S + s] = (int8_t)max(-127, min(127, n));
            if (n > 127 || n < -127) *overflow = 1;
        }
    }
}

// Levenshtein distance, one pair per lane, the DP row and string b staged
// in LDS lane-interleaved (element j of lane l at j*64 + l).  Same
// recurrence as def_func.edit_dist: equal characters take the diagonal,
// otherwise 1 + min(diagonal, up, left).
__global__ void __launch_bounds__(64) k_edit_distance(const uint8_t* __restrict__ seqs,
                                                      const int64_t* __restrict__ off,
                                                      const int32_t* __restrict__ len,
                                                      const int32_t* __restrict__ pa, const int32_t* __restrict__ pb,
                                                      int64_t n_pairs, int32_t max_len, int32_t* __restrict__ dist)
{
    extern __shared__ uint8_t smem[];
    const int lane = threadIdx.x;
    uint16_t* row = reinterpret_cast<uint16_t*>(smem);
    uint8_t* bs = smem + sizeof(uint16_t) * 64 * (size_t)(max_len + 1);
    const int64_t p = (int64_t)blockIdx.x * 64 + lane;
    if (p >= n_pairs) return;
    const uint8_t* a = seqs + off[pa[p]];
    const uint8_t* bg = seqs + off[pb[p]];
    const int la = len[pa[p]], lb = len[pb[p]];
    for (int j = 0; j < lb; j++) bs[j * 64 + lane] = bg[j];
    for (int j = 0; j <= lb; j++) row[j * 64 + lane] = (uint16_t)j;
    for (int i = 1; i <= la; i++) {
        const uint8_t ai = a[i - 1];
        uint16_t diag = row[lane];
        row[lane] = (uint16_t)i;
        uint16_t left = (uint16_t)i;
        for (int j = 1; j <= lb; j++) {
            const uint16_t up = row[j * 64 + lane];
            uint16_t v;
            if (ai == bs[(j - 1) * 64 + lane]) v = diag;
            else v = (uint16_t)(min(min(diag, up), left) + 1);
            row[j * 64 + lane] = v;
            diag = up;
            left = v;
        }
    }
    dist[p] = row[lb * 64 + lane];
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    template <class T> T* as() { return static_cast<T*>(p); }
};

int dev_copy_in(DevBuf& d, const void* src, size_t bytes)
{
    LDPC_HIP(hipMalloc(&d.p, std::max<size_t>(bytes, 16)));
    if (bytes) LDPC_HIP(hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice));
    return LDPC_OK;
}

}  // namespace
}  // namespace ldpc

using ldpc::set_error;

static int dna_llr(int32_t n_strands, const int32_t* kind, const int64_t* row_ptr, const uint8_t* rows,
                   const int32_t* row_q, int32_t payload_nt, double llr_unit, double* llr, uint8_t* int_mask,
                   int8_t* codes, int32_t* codes_exact, int32_t device)
{
    using namespace ldpc;
    if (n_strands < 0 || payload_nt < 1 || !kind || !row_ptr || !llr || (codes && !codes_exact)) {
        set_error("ldpc_dna_llr: bad arguments");
        return LDPC_ERR_ARG;
    }
    if (codes_exact) *codes_exact = 1;
    if (n_strands == 0) return LDPC_OK;
    const int64_t R = row_ptr[n_strands];
    if (R < 0 || R > INT64_MAX / payload_nt || row_ptr[0] != 0 || (R > 0 && (!rows || !row_q))) {
        set_error("ldpc_dna_llr: bad row_ptr / rows");
        return LDPC_ERR_ARG;
    }
    for (int32_t s = 0; s < n_strands; s++) {
        if (row_ptr[s + 1] < row_ptr[s] || kind[s] < 0 || kind[s] > 3) {
            set_error("ldpc_dna_llr: row_ptr not monotone or kind out of range");
            return LDPC_ERR_ARG;
        }
    }
    int ndev = 0;
    LDPC_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        set_error("ldpc_dna_llr: no such device");
        return LDPC_ERR_DEVICE;
    }
    LDPC_HIP(hipSetDevice(device));
    const size_t out_n = (size_t)2 * payload_nt * n_strands;
    DevBuf dk, dp, dr, dq, dl, dm, dc, dov;
    int rc;
    if ((rc = dev_copy_in(dk, kind, sizeof(int32_t) * n_strands))) return rc;
    if ((rc = dev_copy_in(dp, row_ptr, sizeof(int64_t) * ((size_t)n_strands + 1)))) return rc;
    if ((rc = dev_copy_in(dr, rows, (size_t)R * payload_nt))) return rc;
    if ((rc = dev_copy_in(dq, row_q, sizeof(int32_t) * (size_t)R))) return rc;
    LDPC_HIP(hipMalloc(&dl.p, sizeof(double) * out_n));
    if (int_mask) LDPC_HIP(hipMalloc(&dm.p, out_n));
    if (codes) {
        const int32_t zero = 0;
        LDPC_HIP(hipMalloc(&dc.p, out_n));
        if ((rc = dev_copy_in(dov, &zero, sizeof zero))) return rc;
    }
    dim3 grid((unsigned)((n_strands + 255) / 256), (unsigned)payload_nt);
    hipLaunchKernelGGL(k_dna_llr, grid, dim3(256), 0, 0, dk.as<int32_t>(), dp.as<int64_t>(), dr.as<uint8_t>(),
                       dq.as<int32_t>(), n_strands, payload_nt, llr_unit, dl.as<double>(),
                       int_mask ? dm.as<uint8_t>() : nullptr, codes ? dc.as<int8_t>() : nullptr,
                       codes ? dov.as<int32_t>() : nullptr);
    LDPC_HIP(hipGetLastError());
    LDPC_HIP(hipMemcpy(llr, dl.p, sizeof(double) * out_n, hipMemcpyDeviceToHost));
    if (int_mask) LDPC_HIP(hipMemcpy(int_mask, dm.p, out_n, hipMemcpyDeviceToHost));
    if (codes) {
        int32_t ov = 0;
        LDPC_HIP(hipMemcpy(codes, dc.p, out_n, hipMemcpyDeviceToHost));
        LDPC_HIP(hipMemcpy(&ov, dov.p, sizeof ov, hipMemcpyDeviceToHost));
        *codes_exact = ov ? 0 : 1;
    }
    return LDPC_OK;
}


extern "C" {

int ldpc_dna_llr(int32_t n_strands, const int32_t* kind, const int64_t* row_ptr, const uint8_t* rows,
                 const int32_t* row_q, int32_t payload_nt, double llr_unit, double* llr, uint8_t* int_mask,
                 int32_t device)
{
    return dna_llr(n_strands, kind, row_ptr, rows, row_q, payload_nt, llr_unit, llr, int_mask, nullptr, nullptr,
                   device);
}

int ldpc_dna_llr_codes(int32_t n_strands, const int32_t* kind, const int64_t* row_ptr, const uint8_t* rows,
                       const int32_t* row_q, int32_t payload_nt, double llr_unit, double* llr, uint8_t* int_mask,
                       int8_t* codes, int32_t* codes_exact, int32_t device)
{
    return dna_llr(n_strands, kind, row_ptr, rows, row_q, payload_nt, llr_unit, llr, int_mask, codes, codes_exact,
                   device);
}

int ldpc_dna_edit_distance(const uint8_t* seqs, const int64_t* offsets, const int32_t* lengths, int64_t n_seqs,
                           const int32_t* pair_a, const int32_t* pair_b, int64_t n_pairs, int32_t* dist,
                           int32_t device)
{
    using namespace ldpc;
    constexpr int32_t kMaxLen = 800;  // 64 lanes x (801 x 2 B + 800 B) of LDS
    if (n_seqs < 0 || n_pairs < 0 || (n_pairs > 0 && (!pair_a || !pair_b || !dist || !offsets || !lengths))) {
        set_error("ldpc_dna_edit_distance: bad arguments");
        return LDPC_ERR_ARG;
    }
    if (n_pairs == 0) return LDPC_OK;
    int64_t total = 0;
    int32_t max_len = 0;
    for (int64_t i = 0; i < n_seqs; i++) {
        if (lengths[i] < 0 || offsets[i] < 0 || offsets[i] > INT64_MAX - lengths[i]) {
            set_error("ldpc_dna_edit_distance: negative or overflowing length/offset");
            return LDPC_ERR_ARG;
        }
        total = std::max<int64_t>(total, offsets[i] + lengths[i]);
        max_len = std::max(max_len, lengths[i]);
    }
    for (int64_t p = 0; p < n_pairs; p++) {
        if (pair_a[p] < 0 || pair_a[p] >= n_seqs || pair_b[p] < 0 || pair_b[p] >= n_seqs) {
            set_error("ldpc_dna_edit_distance: pair index out of range");
            return LDPC_ERR_ARG;
        }
    }
    if (max_len > kMaxLen) {
        set_error("ldpc_dna_edit_distance: sequences longer than 800 are not supported");
        return LDPC_ERR_UNSUPPORTED;
    }
    if (total > 0 && !seqs) {
        set_error("ldpc_dna_edit_distance: null sequences");
        return LDPC_ERR_ARG;
    }
    int ndev = 0;
    LDPC_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        set_error("ldpc_dna_edit_distance: no such device");
        return LDPC_ERR_DEVICE;
    }
    LDPC_HIP(hipSetDevice(device));
    DevBuf ds, doff, dlen, da, db, dd;
    int rc;
    if ((rc = dev_copy_in(ds, seqs, (size_t)total))) return rc;
    if ((rc = dev_copy_in(doff, offsets, sizeof(int64_t) * (size_t)n_seqs))) return rc;
    if ((rc = dev_copy_in(dlen, lengths, sizeof(int32_t) * (size_t)n_seqs))) return rc;
    if ((rc = dev_copy_in(da, pair_a, sizeof(int32_t) * (size_t)n_pairs))) return rc;
    if ((rc = dev_copy_in(db, pair_b, sizeof(int32_t) * (size_t)n_pairs))) return rc;
    LDPC_HIP(hipMalloc(&dd.p, sizeof(int32_t) * (size_t)n_pairs));
    const size_t lds = (sizeof(uint16_t) * (size_t)(max_len + 1) + (size_t)max_len) * 64;
    const unsigned blocks = (unsigned)((n_pairs + 63) / 64);
    hipLaunchKernelGGL(k_edit_distance, dim3(blocks), dim3(64), lds, 0, ds.as<uint8_t>(), doff.as<int64_t>(),
                       dlen.as<int32_t>(), da.as<int32_t>(), db.as<int32_t>(), n_pairs, max_len, dd.as<int32_t>());
    LDPC_HIP(hipGetLastError());
    LDPC_HIP(hipMemcpy(dist, dd.p, sizeof(int32_t) * (size_t)n_pairs, hipMemcpyDeviceToHost));
    return LDPC_OK;
}

}  // extern "C"
