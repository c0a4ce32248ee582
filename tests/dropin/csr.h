// tests/dropin/csr.h — TEST INFRASTRUCTURE: the caller-side CSR header a main.cpp-shaped program
// brings with it (the role of the reference's src/csr.h:1-45). The drop-in test compiles against
// the library with THIS layout and a class-typed IndexType (util.h here), so the field order and
// widths below are the ABI being tested: include/spmv_types.h declares the same three structs
// with uint32_t, and tests/test_abi.py + tests/test_run_elf.py check that both views agree.
// The functions are the csr.cpp entry points main.cpp calls; csr_host.cpp implements them for
// the test over the CPU oracle (never part of the product library).
#ifndef DROPIN_TEST_CSR_H
#define DROPIN_TEST_CSR_H
#include "util.h"
#include <math.h>

/* header line of a matrix file: three counts, then the column-block count the reader derives */
typedef struct csr_header {
    IndexType nr_rows, nr_cols, nr_nzeros;  /* 4 bytes each (ap_uint<32>-sized class here) */
    int blocks;                             /* column blocks (the library reports 1) */
} csr_header;

/* host CSR: row_ptr[nr_rows + 1], col_ind / values[nr_nzeros]; Filename is only carried along */
typedef struct csr_matrix {
    IndexType *row_ptr;   /* offset 0  */
    IndexType *col_ind;   /* offset 8  */
    ValueType *values;    /* offset 16 */
    IndexType nr_nzeros, nr_rows, nr_cols;  /* offsets 24, 28, 32 */
    char *Filename;       /* offset 40 */
} csr_matrix;

/* dense host vector (x, y_gold, y_fpga in main.cpp) */
typedef struct csr_vector {
    ValueType *values;
    IndexType nr_values;
} csr_vector;

/* reader pair (the library's fast reader can stand behind them) */
int read_csr_header(csr_header *hdr, char *Filename);
int read_csr_matrix(csr_matrix *matrix, char *Filename);
/* allocation helpers of the caller (main.cpp frees what these return) */
csr_matrix *create_csr_matrix(csr_header hdr);
void delete_csr_matrix(csr_matrix *matrix);
csr_vector *create_csr_vector(IndexType nr_values);
void delete_csr_vector(csr_vector *vector);
/* the caller's input vector and the software SpMV that verification compares against */
void init_vector_rand(csr_vector *vector, ValueType max);
void spmv_gold(csr_matrix *matrix, ValueType *x, ValueType *y);
#endif
