// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" wrapper (our own code) around the REFERENCE's unmodified
// graph loader and syndrome sources, compiled in place from
// /root/reference/LDPC_dec/ldpc by oracle/Makefile into oracle/_ref/libref.so:
//   rcode.cpp (read_pchk :54-85), mod2sparse.cpp (read :381-427, insert
//   :502-604, mulvec :855-881), check.cpp (check :28-45), intio.cpp, open.cpp,
//   alloc.cpp, mod2dense.cpp, mod2convert.cpp.
// None of those files needs Intel MKL or MSVC-only functions, so they build
// with plain g++ and no stand-ins.  dec.cpp (BP/MSA arithmetic) does need them
// (rand.h:8 mkl_vsl.h; dec.cpp:676,687 _isnan) and is NOT built.
//
// Used by tests/test_graph.py to pin the oracle's and the product's CSR/CSC
// edge ordering and syndrome against the reference's own linked lists.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#include "mod2sparse.h"
#include "rcode.h"
#include "check.h"
#include "intio.h"

extern "C" {

// read_pchk() exits the process on error (rcode.cpp:61-79); callers pass a
// known-good file.
int ref_load(const char *path, int *M_out, int *N_out)
{
    read_pchk((char *)path);
    *M_out = mod2sparse_rows(H);
    *N_out = mod2sparse_cols(H);
    return 0;
}

// read_pchk's own steps without its exit(): the magic word through intio_read,
// then mod2sparse_read (rcode.cpp:60-79).  0 = accepted (H replaced),
// -1 = cannot open, -2 = wrong magic, -3 = mod2sparse_read refused the
// records.  mod2sparse_read allocates whatever the header asks for and
// chk_alloc exits when that fails, so callers keep M and N small.
int ref_try_load(const char *path, int *M_out, int *N_out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    if (intio_read(f) != ('P' << 8) + 0x80) {
        fclose(f);
        return -2;
    }
    mod2sparse *h = mod2sparse_read(f);
    fclose(f);
    if (!h) return -3;
    if (H) mod2sparse_free(H);
    H = h;
    M = mod2sparse_rows(H);
    N = mod2sparse_cols(H);
    *M_out = M;
    *N_out = N;
    return 0;
}

// Walk every row list (first..last) and emit the column indices in list
// order; row_deg[i] receives the list length.  Returns the edge count.
int64_t ref_rows(int *row_deg, int *cols_out)
{
    int64_t k = 0;
    for (int i = 0; i < mod2sparse_rows(H); i++) {
        int d = 0;
        for (mod2entry *e = mod2sparse_first_in_row(H, i); !mod2sparse_at_end(e); e = mod2sparse_next_in_row(e)) {
            cols_out[k++] = mod2sparse_col(e);
            d++;
        }
        row_deg[i] = d;
    }
    return k;
}

// Walk every column list and emit row indices in list order.
int64_t ref_cols(int *col_deg, int *rows_out)
{
    int64_t k = 0;
    for (int j = 0; j < mod2sparse_cols(H); j++) {
        int d = 0;
        for (mod2entry *e = mod2sparse_first_in_col(H, j); !mod2sparse_at_end(e); e = mod2sparse_next_in_col(e)) {
            rows_out[k++] = mod2sparse_row(e);
            d++;
        }
        col_deg[j] = d;
    }
    return k;
}

// The reference syndrome: c = sum(H * dblk mod 2), pchk receives the parities.
int ref_check(const uint8_t *dblk, uint8_t *pchk)
{
    return check(H, (char *)dblk, (char *)pchk);
}

}  // extern "C"
