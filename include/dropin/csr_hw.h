/*
 * include/dropin/csr_hw.h — forward that replaces the reference's src/csr_hw.h (csr_hw.h:1-150).
 * The structs csr_hw_header / csr_hw_matrix / csr_hw_vector and the two functions main.cpp uses
 * from it (storage_overhead, csr_hw.h:140; verification, csr_hw.h:148) are declared by the
 * library's C-ABI header; the per-CU-count builders (csr_hw.h:49-135) are internal to the FPGA
 * path and have no counterpart.
 */
#ifndef SPMV_DROPIN_CSR_HW_H
#define SPMV_DROPIN_CSR_HW_H
#include "csr_hw_wrapper.h" /* include/dropin/csr_hw_wrapper.h */
#endif /* SPMV_DROPIN_CSR_HW_H */
