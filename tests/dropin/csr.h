// tests/dropin/csr.h — TEST INFRASTRUCTURE: restatement of the caller-side src/csr.h (csr.h:1-45):
// the CSR structs main.cpp uses and the csr.cpp functions it calls (implemented for the test in
// csr_host.cpp over the CPU oracle).
#ifndef DROPIN_TEST_CSR_H
#define DROPIN_TEST_CSR_H
#include "util.h"
#include <math.h>

typedef struct csr_header {
    IndexType nr_rows, nr_cols, nr_nzeros;
    int blocks;
} csr_header;

typedef struct csr_matrix {
    IndexType *row_ptr;
    IndexType *col_ind;
    ValueType *values;
    IndexType nr_nzeros, nr_rows, nr_cols;
    char *Filename;
} csr_matrix;

typedef struct csr_vector {
    ValueType *values;
    IndexType nr_values;
} csr_vector;

int read_csr_header(csr_header *hdr, char *Filename);
csr_matrix *create_csr_matrix(csr_header hdr);
void delete_csr_matrix(csr_matrix *matrix);
int read_csr_matrix(csr_matrix *matrix, char *Filename);
csr_vector *create_csr_vector(IndexType nr_values);
void delete_csr_vector(csr_vector *vector);
void init_vector_rand(csr_vector *vector, ValueType max);
void spmv_gold(csr_matrix *matrix, ValueType *x, ValueType *y);
#endif
