/* ldpc_oracle.h -- TEST INFRASTRUCTURE ONLY (see ldpc_oracle.c header). */
#ifndef LDPC_ORACLE_H
#define LDPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_ERR_OPEN = -1, ORACLE_ERR_MAGIC = -2, ORACLE_ERR_FORMAT = -3 };
enum { ORACLE_ALGO_BP = 0, ORACLE_ALGO_MSA = 1 };
enum { ORACLE_POST_LLR = 0, ORACLE_POST_RATIO = 1 };

typedef struct {
    int M, N;
    int64_t E;
    int *row_ptr;  /* [M+1] CSR: edges of row i are row_ptr[i]..row_ptr[i+1]-1, ascending column */
    int *col_idx;  /* [E]   column of CSR edge e */
    int *col_ptr;  /* [N+1] CSC */
    int *col_edge; /* [E]   CSR edge ids of column j in ascending row order */
} oracle_graph;

int oracle_graph_load(const char *path, oracle_graph *g);
void oracle_graph_free(oracle_graph *g);
void oracle_check_regular(const oracle_graph *g, int *dv, int *reg_dv, int *dc, int *reg_dc);
int oracle_check(const oracle_graph *g, const uint8_t *dblk, uint8_t *pchk);
int oracle_bp(const oracle_graph *g, const double *LR, int max_iter, uint8_t *dblk, double *post_ratio, int *valid);
int oracle_msa(const oracle_graph *g, const double *LLR, int max_iter, uint8_t *dblk, double *L, int *valid);
int oracle_decode_batch(const oracle_graph *g, const double *llr, int64_t B, int max_iter, int algo,
                        int post_mode, int nthreads, uint8_t *hard, double *post, int32_t *iters, uint8_t *valid);

/* Integer-message decoders of dec.cpp (test oracle for LDPC_ALGO_QMSA and
 * LDPC_ALGO_GALLAGER_*; algo 2 = quantized/offset min-sum Run_MSA_Decoder
 * dec.cpp:1174, 3/4/5 = Run_Gallager_Decoder dec.cpp:699 type 0/1/2).
 * Zero-posterior ties use the counter hash shared with the product
 * (kernels_int.hpp tie_bit) in place of MKL rand_int(2).  post: L_Q or the
 * decided +-1 (the prior at 0 iterations). */
int oracle_decode_int_batch(const oracle_graph *g, const double *llr, int64_t B, int max_iter, int algo,
                            int precision, double step, int beta, uint64_t seed, int nthreads,
                            uint8_t *hard, double *post, int32_t *iters, uint8_t *valid);

#ifdef __cplusplus
}
#endif


#endif
