/*
 * ldpc_amd.h -- C ABI of the MI355X-native batched LDPC decoder.
 *
 * Drop-in boundary for the `ldpc.exe` step of the DNA-storage pipeline of
 * sjpark0905/DNA-LDPC-codes.  The reference crosses a process boundary once
 * per codeword (ex_decoder/decoder.py:553-562 -> def_func.py:47-51 ->
 * `ldpc 0 0 0 7 200 1 <codeword> <soft> <pchk> 0 0 0 0`), re-parses the .pchk
 * each time and decodes one frame on one CPU thread.  This ABI replaces that
 * with: load the .pchk once, decode a whole batch of LLR vectors per call on
 * one or more GPUs.
 *
 * Plain C types only: pointers + sizes, caller-owned buffers.  The library
 * owns device memory and the graph; a graph is immutable after load and may
 * be shared by threads; every call is reentrant per handle (no globals beyond
 * the thread-local error string).  Errors are negative return codes plus
 * ldpc_last_error() -- never exit(), unlike the reference (rcode.cpp:61-79,
 * mod2sparse.cpp:513-514).
 *
 * Arithmetic contract: IEEE fp64, reference operation order, bit-exact hard
 * decisions / iteration counts with LDPC_dec/ldpc/dec.cpp.
 */
#ifndef LDPC_AMD_H
#define LDPC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_AMD_ABI_VERSION 3

/* error codes */
enum {
    LDPC_OK = 0,
    LDPC_ERR_ARG = -1,      /* bad argument */
    LDPC_ERR_IO = -2,       /* cannot open / read a file */
    LDPC_ERR_FORMAT = -3,   /* not a parity-check file / malformed */
    LDPC_ERR_DEVICE = -4,   /* HIP runtime error, no device, out of memory */
    LDPC_ERR_UNSUPPORTED = -5 /* graph shape outside the compiled kernels */
};

/* decoder algorithms (reference decoder_type, DNA_main.cpp:49, 1565-1594) */
enum {
    LDPC_ALGO_BP = 0,  /* sum-product, LR domain: Run_Belief_Propagation_Decoder dec.cpp:583 */
    LDPC_ALGO_MSA = 1, /* float min-sum: Run_MSA_Decoder_INF dec.cpp:1216 (ldpc argv decoder_type 20) */
    /* integer-message decoders of dec.cpp (not used by the DNA flow; LLR input):
     * QMSA -- quantized min-sum Run_MSA_Decoder dec.cpp:1174 with q-bit messages,
     *         quantizer step and offset beta (decoder_type 20/21 with g_precision > 0);
     *         zero-posterior ties use a seeded counter hash instead of MKL rand_int(2)
     * GALLAGER_* -- Run_Gallager_Decoder dec.cpp:699 type 0/1/2 (decoder_type 1/2/3)
     *         on the hard decision of the input (LLR < 0 -> -1, else +1) */
    LDPC_ALGO_QMSA = 2,
    LDPC_ALGO_GALLAGER_A = 3,
    LDPC_ALGO_GALLAGER_B1 = 4,
    LDPC_ALGO_GALLAGER_B2 = 5
};

/* posterior output kinds (ldpc_opts.post_kind) */
enum {
    LDPC_POST_LLR = 0,   /* BP: log(P), P = LR*prod(lr) with NaN->1; MSA: L (already an LLR) */
    LDPC_POST_RATIO = 1  /* BP only: the raw fp64 posterior likelihood ratio P (bit-exact checks) */
};

/* input kinds for device-resident decode */
enum {
    LDPC_IN_LLR = 0, /* ln(P0/P1); BP converts with exp() (on device: ocml exp) */
    LDPC_IN_LR = 1   /* P0/P1 (BP only) -- what the reference feeds its BP (DNA_main.cpp:1344) */
};

typedef struct ldpc_graph ldpc_graph;

/* Decode schedule.  The schedule changes only which
 * codewords share a launch and where messages live between the phases, never
 * a codeword's arithmetic: every schedule is bit-exact.  A zeroed struct (or
 * a NULL pointer) selects the defaults, which were chosen by same-process A/B
 * measurements on MI355X.  The library reads no environment variable to pick
 * a schedule. */
enum {
    LDPC_SCHED_NONTEMPORAL = 1 << 0,    /* grouped schedule (and compressed min-sum): nontemporal
                                           variable->check stream (default on) */
    LDPC_SCHED_CONTINUOUS = 1 << 3,     /* continuous batching: a finished codeword's lane is refilled with
                                           the next one (fp64 decoders on graphs whose column degrees are all
                                           <= 32, or (8,72)-regular; default on; needs hard / iters / valid
                                           outputs) */
    LDPC_SCHED_MSA_COMPRESSED = 1 << 4, /* min-sum check->variable messages as per-row records (min1, min2,
                                           NaN planes) + one 16-bit meta word per row and codeword
                                           ((8,72)-regular graphs with E < 2^18; default on) */
    LDPC_SCHED_RESIDENT = 1 << 5,       /* continuous BP / fp64 min-sum on (8,72)-regular graphs with N % 32 == 0
                                           or graphs with rows <= 96 and columns <= 32: a pool of pool_tiles tiles
                                           iterated
                                           in place, its state sized to the 256 MB Infinity Cache, the
                                           syndrome fused into the check kernel (default on when the lane
                                           pool is chosen by the engine or is at most 4 tiles) */
    LDPC_SCHED_SPLIT_SYNDROME = 1 << 6, /* (ldpc_engine_info only) continuous grouped schedule: syndrome
                                           spread over syn_blocks blocks per tile */
    LDPC_SCHED_FIRST_FROM_PRIOR = 1 << 12, /* single-fill BP decodes: the first check derives its messages
                                              from the prior instead of E stored copies (default on) */
    LDPC_SCHED_LR_TABLE = 1 << 13,      /* ldpc_decode, BP (host exp) and min-sum: LLR batches on a k * unit
                                           lattice cross PCIe as one byte each and are decoded as codes with the
                                           table k * unit (BP: its host exp), as ldpc_engine_decode_codes
                                           (default on; off = fp64 input: host exp / copy of every value) */
    LDPC_SCHED_DEBUG_NO_DRAIN = 1 << 14, /* tests only: the host ignores a drained pool, so a decode runs
                                           into its step bound and returns LDPC_ERR_DEVICE (default off) */
    LDPC_SCHED_DEBUG_BAD_LANE = 1 << 15 /* tests only (continuous schedules): the lane that claims codeword 0
                                           records an out-of-range index instead; the kernels' bounds checks
                                           skip its output stores and input reads and the decode returns
                                           LDPC_ERR_DEVICE (default off) */
};

typedef struct ldpc_schedule {
    int32_t flags_set;   /* LDPC_SCHED_* bits whose value is taken from `flags`; the others keep the default */
    int32_t flags;
    int32_t group_tiles; /* grouped schedule: 64-codeword tiles per check/variable launch
                            (0 = default: 3, 8 for compressed min-sum; < 0 = the whole pass) */
    int32_t var_cpw;     /* columns per variable-phase wavefront: 1, 2, 4 or 8 (3: compressed min-sum only;
                            0 = default: 2 for coded input in the resident pool or the compressed
                            min-sum, else 4) */
    int32_t pool_tiles;  /* resident pool tiles when the engine chooses the pool (0 = default: 3 for the
                            (8,72)-regular kernels, else as many as fit ~226 MB of messages + priors) */
    int32_t poll_every;  /* resident pool: steps between occupancy polls (0 = default 8) */
    int32_t syn_blocks;  /* continuous grouped schedule: syndrome blocks per tile (0 = default 32) */
    int32_t reserved;    /* 0 */
} ldpc_schedule;

typedef struct ldpc_opts {
    int32_t n_devices;      /* <= 0: use device 0 only; at most 64 (else LDPC_ERR_ARG) */
    const int32_t *devices; /* device ordinals >= 0 (NULL: 0..n_devices-1) */
    int64_t chunk;          /* lane pool: codewords resident per device at once (0: auto --
                               all of a shard of <= 1024, else the engine's own pool);
                               codewords cross PCIe in double-buffered chunks of
                               max(4096, chunk) that overlap the decode */
    int32_t exp_on_host;    /* BP: compute LR = exp(LLR) with the host libm, exactly as
                               DNA_main.cpp:1344 does (default 1 when opts == NULL) */
    int32_t post_kind;      /* LDPC_POST_* */
    int32_t host_threads;   /* threads for host exp/packing (0: auto; clamped to 256) */
    int32_t msa_precision;  /* LDPC_ALGO_QMSA: message bits q, 2..16 (Set_MSA dec.cpp:1683) */
    int32_t msa_offset;     /* LDPC_ALGO_QMSA: offset beta (1 = offset min-sum, decoder_type 21) */
    int32_t reserved0;
    double msa_step;        /* LDPC_ALGO_QMSA: quantizer step (g_step_length), > 0 */
    uint64_t tie_seed;      /* LDPC_ALGO_QMSA: seed of the zero-posterior tie hash */
    const ldpc_schedule *schedule; /* NULL: the default schedule (ABI version 2) */
} ldpc_opts;

/* ------------------------------------------------------------------------ */
/* Graph                                                                     */
/* ------------------------------------------------------------------------ */

/* Largest M or N a graph may have (every constructor below returns
 * LDPC_ERR_UNSUPPORTED above it).  The reference allocates whatever a file's
 * header asks for (mod2sparse_allocate via mod2sparse_read,
 * mod2sparse.cpp:381-400); a 12-byte .pchk could otherwise make the host
 * allocate and clear 16 GB of row/column pointers. */
#define LDPC_MAX_DIM (1 << 26)

/* Load a Radford-Neal .pchk file.  Replaces read_pchk (rcode.cpp:54-85) +
 * mod2sparse_read (mod2sparse.cpp:381-427): same magic ('P'<<8)+0x80, same
 * record stream, same row/column ordering and duplicate rule
 * (mod2sparse_insert, mod2sparse.cpp:502-604).  *err gets LDPC_OK or a code. */
ldpc_graph *ldpc_graph_load(const char *pchk_path, int *err);

/* Build a graph from (row, col) pairs (0-based).  Same ordering/dedup rules. */
ldpc_graph *ldpc_graph_from_edges(int32_t M, int32_t N, const int32_t *rows, const int32_t *cols,
                                  int64_t n_edges, int *err);

/* Load an alist file with the rules of the reference's alist-to-pchk
 * (alist-to-pchk.cpp:36-160); transpose != 0 is its -t option. */
ldpc_graph *ldpc_graph_load_alist(const char *alist_path, int32_t transpose, int *err);

/* Write the graph as a .pchk (intio_write magic + mod2sparse_write,
 * mod2sparse.cpp:338-376) or as an alist file. */
int ldpc_graph_save_pchk(const ldpc_graph *g, const char *pchk_path);
int ldpc_graph_save_alist(const ldpc_graph *g, const char *alist_path);

/* Build the RS-based LDPC code of RS_LDPC.c (RS LDPC encode/RS_LDPC/
 * RS_LDPC.c:221-431): q = 2^s (2 <= s <= 10), M = gamma*q, N = rho*q,
 * 3 <= rho <= q, 1 <= gamma <= q.  Optional outputs: gen_poly[rho-1]
 * (generator polynomial exponents, -1 = zero) and coset[q*q] (coset number
 * of every RS codeword, -1 = none) -- the tables its H_pri = 0 mode prints.
 * The DNA code's decode_n18432_m2048_final.pchk is (8, 72, 8) with its
 * columns permuted (tests/golden/rs_8_72_8_colperm.npz). */
ldpc_graph *ldpc_graph_rs_ldpc(int32_t s, int32_t rho, int32_t gamma, int32_t *gen_poly,
                               int32_t *coset, int *err);

void ldpc_graph_free(ldpc_graph *g);

/* Dimensions and degrees (CheckRegular, dec.cpp:138-189). */
int ldpc_graph_info(const ldpc_graph *g, int32_t *M, int32_t *N, int64_t *E, int32_t *dv_max,
                    int32_t *regular_dv, int32_t *dc_max, int32_t *regular_dc);

/* Block structure of array codes (RS-LDPC, quasi-cyclic): H is row_blocks x
 * col_blocks permutation matrices of size Q, rows in contiguous blocks.  Q = 0
 * when H has no such structure (regular degrees, M = dv * Q, N = dc * Q).
 * col_block[N] (may be NULL) receives each column's block.  The column blocks
 * are found as contiguous runs of Q columns or, for RS-LDPC codes with
 * permuted columns (the DNA code), by matching the column row sets against
 * ldpc_graph_rs_ldpc(log2 Q, col_blocks, row_blocks).  Code-structure tooling;
 * the decoders do not depend on it. */
int ldpc_graph_blocks(const ldpc_graph *g, int32_t *Q, int32_t *row_blocks, int32_t *col_blocks,
                      int32_t *col_block);

/* Copy out the CSR/CSC edge arrays (row_ptr[M+1], col_idx[E], col_ptr[N+1],
 * col_edge[E]); any pointer may be NULL. */
int ldpc_graph_edges(const ldpc_graph *g, int32_t *row_ptr, int32_t *col_idx, int32_t *col_ptr,
                     int32_t *col_edge);

/* Syndrome on the host: returns the number of unsatisfied checks for hard
 * bits dblk[N] (check.cpp:28-45); pchk[M] (may be NULL) receives parities. */
int ldpc_graph_syndrome(const ldpc_graph *g, const uint8_t *dblk, uint8_t *pchk);

/* ------------------------------------------------------------------------ */
/* Batched decode, host buffers (the in-process replacement of ldpc.exe)     */
/* ------------------------------------------------------------------------ */

/* Decode B codewords.  llr: [B][N] row-major fp64 channel LLRs ln(P0/P1) --
 * what soft*.txt holds (decoder.py:314, 528-535).  Outputs (caller-owned,
 * any of post/iters/valid may be NULL):
 *   hard_out [B][N] u8  -- the reference's dblk / dec_*.txt bits
 *   post_out [B][N] f64 -- per opts->post_kind
 *   iters_out[B]    i32 -- return value of Run_*_Decoder (dec.cpp:604, 1249)
 *   valid_out[B]    u8  -- *bIsCodeword (syndrome zero at exit)
 * Replaces LDPC_Decode (DNA_main.cpp:1565-1594) for decoder_type 0 / 20. */
int ldpc_decode(const ldpc_graph *g, const double *llr, int64_t B, int32_t max_iter, int32_t algo,
                uint8_t *hard_out, double *post_out, int32_t *iters_out, uint8_t *valid_out,
                const ldpc_opts *opts);

/* The same decode for a channel output held as small integers -- the DNA
 * pipeline's per-bit read-count differences k = count_0 - count_1, whose LLR
 * is k * ln((1-eps)/eps) (decoder.py:314) -- so no [B][N] fp64 matrix is
 * built, scanned or sent: codes [B][N] int8 (host), table[256] the channel
 * value of code k at table[k + 128], of kind table_kind (LDPC_IN_LLR; for BP
 * also LDPC_IN_LR).  BP's LR is the host libm exp of an LLR table entry, as
 * DNA_main.cpp:1344 computes it per bit.  Identical results to ldpc_decode on
 * llr[b][j] = table[codes[b][j] + 128] (LDPC_IN_LLR); one byte per bit
 * crosses PCIe.  Outputs and opts as ldpc_decode. */
int ldpc_decode_codes(const ldpc_graph *g, const int8_t *codes, const double *table, int32_t table_kind,
                      int64_t B, int32_t max_iter, int32_t algo, uint8_t *hard_out, double *post_out,
                      int32_t *iters_out, uint8_t *valid_out, const ldpc_opts *opts);

/* ------------------------------------------------------------------------ */
/* Device-resident engine (benchmarks, pipelines that keep data in HBM)      */
/* ------------------------------------------------------------------------ */
typedef struct ldpc_engine ldpc_engine;

/* One engine = one device + one HIP stream + chunk-sized message buffers,
 * with the default schedule.  An engine serves one thread at a time (its
 * calls enqueue on its one stream); engines on one graph may run in
 * different threads at once. */
ldpc_engine *ldpc_engine_create(const ldpc_graph *g, int32_t device, int32_t algo, int64_t chunk, int *err);

/* Same with an explicit schedule (NULL = defaults). */
ldpc_engine *ldpc_engine_create_ex(const ldpc_graph *g, int32_t device, int32_t algo, int64_t chunk,
                                   const ldpc_schedule *schedule, int *err);
void ldpc_engine_free(ldpc_engine *e);

/* Decode B codewords whose input already lives in device memory (d_in:
 * [B][N] fp64, kind LDPC_IN_*).  Device outputs (NULL to skip): d_hard
 * [B][N] u8, d_post [B][N] f64 (post_kind), d_iters [B] i32, d_valid [B] u8.
 * Asynchronous on the engine's stream; ldpc_engine_sync() waits. */
int ldpc_engine_decode(ldpc_engine *e, const double *d_in, int32_t in_kind, int64_t B, int32_t max_iter,
                       uint8_t *d_hard, double *d_post, int32_t post_kind, int32_t *d_iters, uint8_t *d_valid);

/* The same decode for channel outputs given as small integers -- the DNA
 * pipeline's per-bit count differences k, whose LLR is k * ln((1-eps)/eps)
 * (decoder.py:314), or a BSC's +-1: d_codes [B][N] int8 on the device and
 * table[256] (host) the channel value of code k at table[k + 128], of kind
 * table_kind (LDPC_IN_LLR; LDPC_IN_LR for BP only).  BP takes LR = the host
 * libm exp of an LLR table entry, as DNA_main.cpp:1344 does per bit.  The
 * result equals ldpc_engine_decode on the fp64 input table[code + 128]
 * bit for bit; the continuous schedules keep each codeword's prior as its
 * one-byte code instead of an fp64 value. */
int ldpc_engine_decode_codes(ldpc_engine *e, const int8_t *d_codes, const double *table, int32_t table_kind,
                             int64_t B, int32_t max_iter, uint8_t *d_hard, double *d_post, int32_t post_kind,
                             int32_t *d_iters, uint8_t *d_valid);

int ldpc_engine_sync(ldpc_engine *e);

/* The engine's HIP stream (hipStream_t as void*). */
void *ldpc_engine_stream(ldpc_engine *e);

/* Synthetic BSC channel on device: for codeword
 * index b in [b0, b0+B) and bit j, the transmitted bit is
 * codewords[(b mod n_cw)][j] (d_codewords: [n_cw][N] u8 on device), flipped
 * when hash(seed, b, j) < p; output value = +-llr_mag (LDPC_IN_LLR) or
 * +-exp(+-llr_mag) with host-computed exp (LDPC_IN_LR), written to d_out
 * [B][N] fp64. */
int ldpc_engine_gen_bsc(ldpc_engine *e, double *d_out, int32_t out_kind, int64_t b0, int64_t B,
                        const uint8_t *d_codewords, int32_t n_cw, uint64_t seed, double p, double llr_mag);

/* The same channel as codes for ldpc_engine_decode_codes: d_out [B][N] int8,
 * +1 where the received bit is 0 and -1 where it is 1 (table[129] = llr_mag,
 * table[127] = -llr_mag gives ldpc_engine_gen_bsc's LLRs). */
int ldpc_engine_gen_bsc_codes(ldpc_engine *e, int8_t *d_out, int64_t b0, int64_t B, const uint8_t *d_codewords,
                              int32_t n_cw, uint64_t seed, double p);

/* Kernel timing: HIP events on the engine stream around every stride-th
 * launch of each kernel class (stride 1 = every launch, 0 = off).  Enabling
 * resets the counters; read them after ldpc_engine_sync(). */
typedef struct ldpc_kernel_stats {
    int64_t launches[6];    /* [0]=check [1]=variable [2]=syndrome [3]=init [4]=finalize [5]=other */
    int64_t sampled[6];     /* launches that carried events */
    double ms[6];           /* summed device time of the sampled launches */
} ldpc_kernel_stats;

int ldpc_engine_profile(ldpc_engine *e, int32_t stride);

/* Parameters of LDPC_ALGO_QMSA (ignored by the other algorithms); the
 * engine starts with q = 6, step = 0.5, beta = 0, seed = 0. */
int ldpc_engine_set_params(ldpc_engine *e, int32_t msa_precision, double msa_step, int32_t msa_offset,
                           uint64_t tie_seed);
/* The schedule an engine runs with: resident codewords per pass (the lane
 * pool in continuous mode), tiles per launch, and the LDPC_SCHED_* bits that
 * are in effect. */
int ldpc_engine_info(ldpc_engine *e, int64_t *cap, int64_t *group_tiles, int32_t *flags);
int ldpc_engine_stats(ldpc_engine *e, ldpc_kernel_stats *out);

/* Pinned (page-locked) host memory.  Host-buffer inputs that live in it cross
 * PCIe straight from the caller's array (ldpc_decode_codes: no staging
 * copy); any other host memory is staged through the library's own pinned
 * buffers. */
void *ldpc_host_alloc(size_t bytes);
int ldpc_host_free(void *p);

/* Device buffers for callers without their own HIP allocator (bench, tests). */
enum { LDPC_H2D = 0, LDPC_D2H = 1, LDPC_D2D = 2 };
void *ldpc_dev_malloc(int32_t device, size_t bytes);
int ldpc_dev_free(int32_t device, void *p);
int ldpc_dev_memcpy(int32_t device, void *dst, const void *src, size_t bytes, int32_t kind);

/* ------------------------------------------------------------------------ */
/* DNA soft-input construction (the step before the decoder)                 */
/* ------------------------------------------------------------------------ */
/* Per-strand LLRs from read candidates -- the arithmetic of decoder.py's
 * strand loop (ex_decoder/decoder.py:142-519; count rule :266-320,
 * :442-497).  The caller (dna_llr.py) classifies strand s into kind[s]:
 *   0 no LLRs, 1 count over its rows, 2 one short candidate, 3 alignment
 *   failed (count of the failed rows' last bases)
 * and lays the candidate rows of strand s at rows[row_ptr[s]..row_ptr[s+1])
 * (payload_nt bytes each, ASCII bases; for kinds 2 and 3 byte 0 of a row is
 * the candidate's last base) with per-row quality row_q.  Output, on the
 * host: llr[2*payload_nt][n_strands] (row i = soft file i+1, i.e. the
 * decoder's [codeword][bit] layout) and optionally int_mask of the same
 * shape (1 where the reference leaves an int 0, which str() prints as "0").
 * Runs on `device`. */
int ldpc_dna_llr(int32_t n_strands, const int32_t *kind, const int64_t *row_ptr, const uint8_t *rows,
                 const int32_t *row_q, int32_t payload_nt, double llr_unit, double *llr, uint8_t *int_mask,
                 int32_t device);

/* ldpc_dna_llr, plus each entry's count difference as an int8 code:
 * llr = codes * llr_unit exactly (decoder.py:297-314), codes
 * [2*payload_nt][n_strands].  *codes_exact = 1 when every |code| <= 127,
 * else 0 (the codes are then saturated and only llr is usable).  The codes
 * and the table k * llr_unit feed ldpc_decode_codes / the engine's coded
 * input without a host lattice pass over the fp64 matrix. */
int ldpc_dna_llr_codes(int32_t n_strands, const int32_t *kind, const int64_t *row_ptr, const uint8_t *rows,
                       const int32_t *row_q, int32_t payload_nt, double llr_unit, double *llr, uint8_t *int_mask,
                       int8_t *codes, int32_t *codes_exact, int32_t device);

/* Levenshtein distances of sequence pairs on `device`
 * (def_func.edit_dist, def_func.py:10-26).  Sequence i is
 * seqs[offsets[i] .. offsets[i]+lengths[i]); lengths <= 800. */
int ldpc_dna_edit_distance(const uint8_t *seqs, const int64_t *offsets, const int32_t *lengths, int64_t n_seqs,
                           const int32_t *pair_a, const int32_t *pair_b, int64_t n_pairs, int32_t *dist,
                           int32_t device);

/* Write soft<rs>_n18432_m1860_<i+1>.txt, i < n_files, into dir: row i of
 * llr as str(value)+' ' tokens (decoder.py:511-516, def_func.py:54-57);
 * int_mask (may be NULL) marks the int-0 entries.  Host only. */
int ldpc_write_soft_files(const char *dir, int32_t rs, const double *llr, const uint8_t *int_mask,
                          int32_t n_files, int32_t n_strands);

/* Python repr() of a double into out (NUL-terminated); returns its length. */
int ldpc_py_float_repr(double v, char *out, int32_t cap);

/* ------------------------------------------------------------------------ */
/* misc                                                                      */
/* ------------------------------------------------------------------------ */
const char *ldpc_last_error(void); /* thread-local message for the last failing call */
int ldpc_device_count(void);
int ldpc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_AMD_H */
