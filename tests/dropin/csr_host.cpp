// tests/dropin/csr_host.cpp — TEST INFRASTRUCTURE: the csr.cpp functions main.cpp calls
// (csr.cpp:10-194), implemented over the CPU oracle (oracle/csr_ref.c) for the drop-in build
// test. It plays the part of the reference's csr.cpp, which stays on the caller's side.
#include <cstdlib>

#include "csr.h"

extern "C" {
int oracle_read_csr_header(const char *, uint32_t *, uint32_t *, uint32_t *, uint32_t, int *);
int oracle_read_csr_matrix(const char *, uint32_t, uint32_t, uint32_t *, uint32_t *, ValueType *);
void oracle_init_vector_rand(ValueType *, uint32_t, ValueType);
void oracle_spmv_gold(uint32_t, const uint32_t *, const uint32_t *, const ValueType *, const ValueType *, ValueType *);
}

double getTimestamp()
{
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_usec + tv.tv_sec * 1e6;
}

int read_csr_header(csr_header *hdr, char *Filename)
{
    uint32_t r, c, z;
    const int rc = oracle_read_csr_header(Filename, &r, &c, &z, 32768, &hdr->blocks);
    hdr->nr_rows = r;
    hdr->nr_cols = c;
    hdr->nr_nzeros = z;
    return rc;
}

csr_matrix *create_csr_matrix(csr_header hdr)
{
    csr_matrix *m = (csr_matrix *)std::malloc(sizeof(csr_matrix));
    m->nr_rows = hdr.nr_rows;
    m->nr_cols = hdr.nr_cols;
    m->nr_nzeros = hdr.nr_nzeros;
    m->row_ptr = (IndexType *)std::calloc(uint32_t(hdr.nr_rows) + 1, sizeof(IndexType));
    m->col_ind = (IndexType *)std::calloc(uint32_t(hdr.nr_nzeros) + 1, sizeof(IndexType));
    m->values = (ValueType *)std::calloc(uint32_t(hdr.nr_nzeros) + 1, sizeof(ValueType));
    m->Filename = nullptr;
    return m;
}

void delete_csr_matrix(csr_matrix *m)
{
    std::free(m->row_ptr);
    std::free(m->col_ind);
    std::free(m->values);
    std::free(m);
}

int read_csr_matrix(csr_matrix *m, char *Filename)
{
    m->Filename = Filename;
    return oracle_read_csr_matrix(Filename, m->nr_rows, m->nr_nzeros, reinterpret_cast<uint32_t *>(m->row_ptr),
                                  reinterpret_cast<uint32_t *>(m->col_ind), m->values);
}

csr_vector *create_csr_vector(IndexType n)
{
    csr_vector *v = (csr_vector *)std::malloc(sizeof(csr_vector));
    v->values = (ValueType *)std::calloc(uint32_t(n) + 1, sizeof(ValueType));
    v->nr_values = n;
    return v;
}

void delete_csr_vector(csr_vector *v)
{
    std::free(v->values);
    std::free(v);
}

void init_vector_rand(csr_vector *v, ValueType max) { oracle_init_vector_rand(v->values, v->nr_values, max); }

void spmv_gold(csr_matrix *m, ValueType *x, ValueType *y)
{
    oracle_spmv_gold(m->nr_rows, reinterpret_cast<const uint32_t *>(m->row_ptr),
                     reinterpret_cast<const uint32_t *>(m->col_ind), m->values, x, y);
}
