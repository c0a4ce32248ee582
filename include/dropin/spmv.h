/*
 * include/dropin/spmv.h — forward that replaces the reference's src/spmv.h (spmv.h:1-200+), the
 * declaration of the FPGA device entry spmv() (spmv.cpp:169-205) and its SDSoC data pragmas.
 * On MI355X that entry is the library's HIP kernels behind spmv_hw(); main.cpp includes this
 * header (main.cpp:14) but calls nothing from it.
 */
#ifndef SPMV_DROPIN_SPMV_H
#define SPMV_DROPIN_SPMV_H
#include "csr_hw_wrapper.h" /* include/dropin/csr_hw_wrapper.h */
#endif /* SPMV_DROPIN_SPMV_H */
