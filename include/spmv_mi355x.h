/*
 * spmv_mi355x.h — include alias for the MI355X drop-in.
 *
 * The reference's own src/csr_hw_wrapper.h is replaced by a forward that includes THIS file, so
 * that the forward does not have to include a header with its own name.
 */
#ifndef SPMV_MI355X_H
#define SPMV_MI355X_H
#include "csr_hw_wrapper.h"
#endif
