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

#ifdef __cplusplus
}
#endif
#endif
