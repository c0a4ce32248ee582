/*
 * spmv_types.h — the data types of the csr_hw_wrapper drop-in boundary.
 *
 * Restates (does not copy) the reference's type header set:
 *   util.h:9-26      IndexType = ap_uint<32>  -> uint32_t (same 4-byte layout; the reference
 *                    passes it to fscanf("%u"), csr.cpp:21), ValueType = float|double by DOUBLE
 *   util.h:61-69     128-bit bus word BusDataType -> opaque 16-byte struct (only ever a device
 *                    pointer on MI355X; host code never dereferences it)
 *   csr.h:7-29       csr_header / csr_matrix / csr_vector (field names and order kept)
 *   csr_hw.h:8-33    csr_hw_header / csr_hw_matrix / csr_hw_vector (field names and order kept,
 *                    because main.cpp:69,86-87 reads hw_matrix[0]->blocks, ->nr_cols and passes
 *                    hw_matrix[i] to storage_overhead)
 *
 * Build knob: DOUBLE=1 (default) -> ValueType double, DOUBLE=0 -> float, exactly as the
 * reference's Makefile:17,71 passes -DDOUBLE. One shared library is built per precision.
 *
 * Drop-in use from the reference's own sources: include the reference's util.h and csr.h first
 * and define SPMV_USE_CALLER_CSR_TYPES; the caller's IndexType/ValueType/csr_* types and its
 * ap_uint<128> BusDataType are then used (same sizes and field order), see INTEGRATION.md §1.
 */
#ifndef SPMV_TYPES_H
#define SPMV_TYPES_H

#include <stdint.h>
#include <stdbool.h>

#ifndef DOUBLE
#define DOUBLE 1
#endif

#ifndef SPMV_USE_CALLER_CSR_TYPES
typedef uint32_t IndexType;               /* util.h:9  (ap_uint<32>) */
#if DOUBLE == 0
typedef float ValueType;                  /* util.h:19 */
#else
typedef double ValueType;                 /* util.h:23 */
#endif
/* util.h:61-69: the reference moves 128-bit words over the AXI bus. On MI355X the hw
 * representation lives in HBM; a BusDataType* in the structs below is an opaque device
 * address of a 16-byte-aligned buffer. */
typedef struct BusDataType {
    uint64_t lo, hi;
} BusDataType;
#endif

#ifndef INDEX_TYPE_BIT_WIDTH
#define INDEX_TYPE_BIT_WIDTH 32
#endif
#ifndef VALUE_TYPE_BIT_WIDTH
#if DOUBLE == 0
#define VALUE_TYPE_BIT_WIDTH 32
#else
#define VALUE_TYPE_BIT_WIDTH 64
#endif
#endif
#ifndef BUS_BIT_WIDTH
#define BUS_BIT_WIDTH 128
#endif

#ifndef SPMV_USE_CALLER_CSR_TYPES
/* csr.h:7-13 */
typedef struct csr_header {
    IndexType nr_rows;
    IndexType nr_cols;
    IndexType nr_nzeros;
    int blocks;
} csr_header;

/* csr.h:15-24 */
typedef struct csr_matrix {
    IndexType *row_ptr;
    IndexType *col_ind;
    ValueType *values;
    IndexType nr_nzeros;
    IndexType nr_rows;
    IndexType nr_cols;
    char *Filename;
} csr_matrix;

/* csr.h:26-29 */
typedef struct csr_vector {
    ValueType *values;
    IndexType nr_values;
} csr_vector;
#endif /* SPMV_USE_CALLER_CSR_TYPES */

/* csr_hw.h:8-14 */
typedef struct csr_hw_header {
    IndexType expanded_nr_rows;
    IndexType expanded_nr_cols;
    IndexType expanded_nr_nzeros;
    int blocks;
} csr_hw_header;

/* csr_hw.h:16-26. One handle per "Compute Unit"; on MI355X a unit is a GPU (or a virtual unit
 * on a GPU). Arrays are indexed by column block. submatrix[b] is a device
 * address. The library allocates a larger private object whose first member is this struct. */
typedef struct csr_hw_matrix {
    BusDataType **submatrix;
    IndexType *nr_rows;
    IndexType *nr_cols;
    IndexType *nr_nzeros;
    IndexType *nr_ci;
    IndexType *nr_val;
    int blocks;
} csr_hw_matrix;

/* csr_hw.h:28-33. values[b] is a device address (x block b on unit 0's GPU). */
typedef struct csr_hw_vector {
    BusDataType **values;
    IndexType *nr_values;
    int blocks;
} csr_hw_vector;

#endif /* SPMV_TYPES_H */
