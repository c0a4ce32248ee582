/*
 * include/dropin/csr_hw_wrapper.h — forward that replaces the reference's src/csr_hw_wrapper.h
 * (csr_hw_wrapper.h:1-19) in an unchanged src/main.cpp build.
 *
 * The caller's own util.h (IndexType, ValueType, ComputeUnits from -DCU) and csr.h (csr_matrix,
 * csr_vector) stay; the MI355X library's C-ABI is declared over those types. Compile with
 * -I<repo>/include/dropin -I<repo>/include after deleting src/csr_hw_wrapper.h, src/csr_hw.h and
 * src/spmv.h (so that main.cpp's quoted includes find these forwards).
 *
 * ComputeUnits: main.cpp sizes its loops with the compile-time CU (main.cpp:86-87, util.h:41-59).
 * This forward hands that count to the library before main() runs (spmv_hw_set_units), so the
 * library builds exactly ComputeUnits unit slices (units map to GPUs round-robin; more units than
 * GPUs share one). Without a CU define (or with SPMV_DROPIN_NO_CU_HINT) the count comes from env
 * SPMV_NGPUS; hw_matrix still has >= 12 + 1 slots, the unused ones NULL.
 */
#ifndef SPMV_DROPIN_CSR_HW_WRAPPER_H
#define SPMV_DROPIN_CSR_HW_WRAPPER_H

#include "util.h" /* the caller's: IndexType, ValueType, BusDataType, ComputeUnits */
#include "csr.h"  /* the caller's: csr_header, csr_matrix, csr_vector */
#ifndef SPMV_USE_CALLER_CSR_TYPES
#define SPMV_USE_CALLER_CSR_TYPES
#endif
#include "spmv_mi355x.h" /* include/csr_hw_wrapper.h of this repository */

#if defined(__cplusplus) && defined(ComputeUnits) && !defined(SPMV_DROPIN_NO_CU_HINT)
namespace spmv_dropin_detail {
/* runs during static initialisation of every translation unit that includes this header */
static const int compute_units_registered = (spmv_hw_set_units(ComputeUnits), ComputeUnits);
}  // namespace spmv_dropin_detail
#endif

#endif /* SPMV_DROPIN_CSR_HW_WRAPPER_H */
