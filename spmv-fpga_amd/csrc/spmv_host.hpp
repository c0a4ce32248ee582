// Host-only internals of libspmv_hw (no HIP): what host.cpp and reader.cpp share with the rest of
// the library. tests/sanitize/Makefile compiles these two sources with g++ -fsanitize=... into a
// host-only check program, so nothing here may need the HIP headers.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "csr_hw_wrapper.h"

namespace spmvhw {

void set_error(const std::string &msg);
const char *get_error();

// Environment switches of the measurement-only tools build (make ablations, -DSPMV_ABLATIONS:
// layouts and schedules that were measured and not kept, or that tests force). The product
// library reads only the caller-facing knobs INTEGRATION.md §1.4 documents; there this is null.
inline const char *ablation_env(const char *name)
{
#ifdef SPMV_ABLATIONS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// wall clock in microseconds (util.cpp:3-8)
double timestamp_us();

// One piece of accum_results' '+=' (csr_hw.cpp:1531-1565): dst[i] += src[i] for i < count, once
// the copy that fills src has landed. `ready` is opaque here (the library passes a hipEvent_t):
// host_accumulate hands it to the caller's wait function before reading src.
struct add_part {
    ValueType *dst;
    const ValueType *src;
    uint64_t count;
    void *ready;
};

struct accum_options {
    bool prefault = true;  // map each thread's ranges of dst writable while the copies run
    bool split = true;     // thread t adds the t-th 1/T of every part (false: whole parts t, t+T, ..)
    int threads = 16;      // at most this many threads (1 below 2^18 values in all)
};

// Adds the parts in on up to opts.threads host threads, in part order; wait(ready) returns 0 once
// a part's source is complete (nonzero: error, message in *err; the adds of that thread stop).
// Returns the timestamp_us at which the last part was seen complete; *failed is set when any
// wait failed.
double host_accumulate(const add_part *parts, size_t nparts, int (*wait)(void *ready, std::string *err),
                       const accum_options &opts, bool *failed, std::string *err);

// maps [p, p + count) writable keeping its contents (madvise(MADV_POPULATE_WRITE), else a
// touch per page)
void prefault(ValueType *p, uint64_t count);

}  // namespace spmvhw
