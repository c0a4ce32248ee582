/*
 * include/dropin/sds_lib.h — the SDSoC runtime header that main.cpp:8 and csr_hw.h:5 include.
 * The MI355X build has no SDSoC runtime: main.cpp and csr.cpp call none of its functions, and the
 * FPGA buffers it allocated (sds_alloc_non_cacheable, csr_hw.cpp:180) are HBM allocations inside
 * the library. For any other caller code that still allocates through it, the calls map to
 * page-aligned host memory.
 */
#ifndef SPMV_DROPIN_SDS_LIB_H
#define SPMV_DROPIN_SDS_LIB_H
#include <stdlib.h>

static inline void *sds_alloc(size_t size)
{
    void *p = NULL;
    return posix_memalign(&p, 4096, size ? size : 1) == 0 ? p : NULL;
}
static inline void *sds_alloc_non_cacheable(size_t size) { return sds_alloc(size); }
static inline void *sds_alloc_cacheable(size_t size) { return sds_alloc(size); }
static inline void sds_free(void *p) { free(p); }

#endif /* SPMV_DROPIN_SDS_LIB_H */
