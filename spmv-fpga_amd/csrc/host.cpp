// Host-only parts of libspmv_hw (no HIP calls): the error channel, the nnz-balanced row
// partition, the exchange schedule of the multi-GPU merge, the threaded accum_results '+=',
// verification and storage_overhead. Besides the product library, tests/sanitize/Makefile builds
// this file and reader.cpp with g++ under AddressSanitizer + UBSan and under ThreadSanitizer
// (SURVEY §5 "sanitizers").
#include <sys/mman.h>
#include <sys/time.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <iomanip>
#include <iostream>
#include <thread>
#include <vector>

#include "spmv_host.hpp"

namespace spmvhw {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
const char *get_error() { return g_err.c_str(); }

double timestamp_us()
{
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_usec + tv.tv_sec * 1e6;
}

// Maps the caller's y pages writable while the DMA runs, keeping their contents: a fresh
// calloc'd y_fpga (main.cpp:74) otherwise takes one page fault per 4 KiB inside the adds
void prefault(ValueType *p, uint64_t count)
{
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif
    const uintptr_t pg = 4096;
    const uintptr_t b = ((uintptr_t)p + pg - 1) & ~(pg - 1), e = (uintptr_t)(p + count) & ~(pg - 1);
    if (e <= b || madvise((void *)b, e - b, MADV_POPULATE_WRITE) == 0)
        return;
    for (uintptr_t a = b; a < e; a += pg) {  // older kernels: touch each page
        volatile ValueType *q = (volatile ValueType *)a;
        *q = *q;
    }
}

// Thread t of T adds its range of every part in part (= copy landing) order as soon as that
// part's copy has landed, so the adds run behind the DMA and the last piece to land leaves 1/T of
// a piece per thread (split = false: thread t adds whole parts t, t + T, ... instead). Each thread
// first maps its ranges of the caller's y writable, while the DMA runs.
double host_accumulate(const add_part *parts, size_t nparts, int (*wait)(void *ready, std::string *err),
                       const accum_options &o, bool *failed, std::string *err)
{
    uint64_t total = 0;
    for (size_t k = 0; k < nparts; ++k)
        total += parts[k].count;
    const size_t T = nparts == 0          ? 0
                     : total < (1u << 18) ? 1
                                          : std::min<size_t>(std::max(1, o.threads), o.split ? size_t(64) : nparts);
    auto range = [&](size_t t, size_t k, uint64_t &b, uint64_t &e) {
        const uint64_t n = parts[k].count;
        if (o.split)
            b = n * t / T, e = n * (t + 1) / T;
        else
            b = 0, e = k % T == t ? n : 0;
    };
    std::vector<double> landed(T, 0.0);
    std::vector<std::string> errs(T);
    std::atomic<bool> bad{false};
    auto work = [&](size_t t) {
        uint64_t b, e;
        if (o.prefault)
            for (size_t k = 0; k < nparts; ++k) {
                range(t, k, b, e);
                if (e > b)
                    prefault(parts[k].dst + b, e - b);
            }
        for (size_t k = 0; k < nparts; ++k) {
            range(t, k, b, e);
            if (e <= b)
                continue;
            const add_part &q = parts[k];
            if (wait(q.ready, &errs[t])) {
                bad.store(true);
                return;
            }
            landed[t] = timestamp_us();
            for (uint64_t i = b; i < e; ++i)
                q.dst[i] += q.src[i];
        }
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; ++t)
        th.emplace_back(work, t);
    if (T)
        work(0);
    for (auto &t : th)
        t.join();
    *failed = bad.load();
    if (*failed && err)
        for (const std::string &s : errs)
            if (!s.empty()) {
                *err = s;
                break;
            }
    return T ? *std::max_element(landed.begin(), landed.end()) : timestamp_us();
}

}  // namespace spmvhw

using namespace spmvhw;

extern "C" {

const char *spmv_hw_last_error(void) { return get_error(); }
int spmv_hw_value_bytes(void) { return (int)sizeof(ValueType); }

// the S1 rule of prepare_balanced_hw_matrix (csr_hw.cpp:459-468): unit u's slice starts at the
// first row whose start reaches u/units of the non-zeros
int spmv_partition_rows(const IndexType *row_ptr, IndexType nr_rows, int units, IndexType *bounds)
{
    if (!row_ptr || !bounds || units < 1) {
        set_error("spmv_partition_rows: bad arguments");
        return 1;
    }
    const uint64_t nnz = uint64_t(row_ptr[nr_rows]) - row_ptr[0];
    bounds[0] = 0;
    for (int u = 1; u < units; ++u) {
        const uint64_t target = row_ptr[0] + nnz * uint64_t(u) / uint64_t(units);
        // first row whose start is >= target
        const IndexType *it = std::lower_bound(row_ptr, row_ptr + nr_rows, (IndexType)target);
        IndexType b = (IndexType)(it - row_ptr);
        bounds[u] = std::max(b, bounds[u - 1]);
    }
    bounds[units] = nr_rows;
    return 0;
}

// accum_results (csr_hw.cpp:1531-1565) loops the CUs and adds each CU's compact y slice into the
// host y. Here the slices meet on the devices; this is the list of what one rank does for one
// step (include/csr_hw_wrapper.h, spmv_xop):
//   gather     rank 0 computes into its rows of y and receives every other non-empty slice at
//              that slice's offset; rank r > 0 computes into its slice buffer and sends it
//   reduce     every rank zeroes its full-length partial, computes into its rows of it, and the
//              partials are summed into rank 0's y (also at one rank: RCCL copies the partial)
//   all-gather every rank computes into its rows of the next x, then every non-empty slice is
//              broadcast from its owner into every rank's next x (all-gather, unequal counts)
// Empty slices neither compute nor communicate.
int spmv_mgpu_schedule(int exchange, int rank, int nranks, const IndexType *bounds, spmv_xop *ops, int cap)
{
    if (exchange < SPMV_MGPU_GATHER || exchange > SPMV_MGPU_ALLGATHER || nranks < 1 || rank < 0 || rank >= nranks ||
        !bounds || cap < 0 || (cap > 0 && !ops)) {
        set_error("spmv_mgpu_schedule: bad arguments");
        return -1;
    }
    if (bounds[0] != 0) {
        set_error("spmv_mgpu_schedule: bounds must start at 0");
        return -1;
    }
    for (int r = 0; r < nranks; ++r)
        if (bounds[r + 1] < bounds[r]) {
            set_error("spmv_mgpu_schedule: bounds must be non-decreasing");
            return -1;
        }
    int n = 0;
    auto emit = [&](int kind, int buf, int peer, int out, IndexType offset, IndexType count) {
        if (n < cap)
            ops[n] = spmv_xop{kind, buf, peer, out, offset, count};
        ++n;
    };
    const IndexType nr_rows = bounds[nranks];
    const IndexType b0 = bounds[rank], rows = bounds[rank + 1] - bounds[rank];
    auto rows_of = [&](int r) { return bounds[r + 1] - bounds[r]; };
    if (exchange == SPMV_MGPU_GATHER) {
        if (rank == 0) {
            if (rows)
                emit(SPMV_XOP_COMPUTE, SPMV_XBUF_Y, -1, -1, b0, rows);
            for (int p = 1; p < nranks; ++p)
                if (rows_of(p))
                    emit(SPMV_XOP_RECV, SPMV_XBUF_Y, p, -1, bounds[p], rows_of(p));
        } else if (rows) {
            emit(SPMV_XOP_COMPUTE, SPMV_XBUF_SLICE, -1, -1, 0, rows);
            emit(SPMV_XOP_SEND, SPMV_XBUF_SLICE, 0, -1, 0, rows);
        }
    } else if (exchange == SPMV_MGPU_REDUCE) {
        if (nr_rows) {
            emit(SPMV_XOP_ZERO, SPMV_XBUF_PART, -1, -1, 0, nr_rows);
            if (rows)
                emit(SPMV_XOP_COMPUTE, SPMV_XBUF_PART, -1, -1, b0, rows);
            emit(SPMV_XOP_REDUCE, SPMV_XBUF_PART, 0, rank == 0 ? SPMV_XBUF_Y : -1, 0, nr_rows);
        }
    } else {
        if (rows)
            emit(SPMV_XOP_COMPUTE, SPMV_XBUF_XNEXT, -1, -1, b0, rows);
        if (nranks > 1)
            for (int r = 0; r < nranks; ++r)
                if (rows_of(r))
                    emit(SPMV_XOP_BCAST, SPMV_XBUF_XNEXT, r, -1, bounds[r], rows_of(r));
    }
    return n;
}

// csr_hw.cpp:1401-1409: MB of one unit's representation (computed in 64 bits)
ValueType storage_overhead(csr_hw_matrix *matrix)
{
    if (!matrix)
        return 0;
    uint64_t bits = uint64_t(matrix->blocks) * 5 * INDEX_TYPE_BIT_WIDTH;
    for (int b = 0; b < matrix->blocks; ++b)
        bits += (uint64_t(matrix->nr_ci[b]) + matrix->nr_val[b]) * BUS_BIT_WIDTH;
    return (ValueType)(bits / (8.0 * 1024 * 1024));
}

// csr_hw.cpp:1571-1590
int verification(uint32_t nr_values, ValueType *sw_values, ValueType *hw_values, int verbose)
{
    const ValueType diff_thres = (ValueType)1e-5;
    int status = 0;
    IndexType err_cnt = 0;
    for (IndexType i = 0; i < nr_values; ++i) {
        const ValueType diff = std::fabs(sw_values[i] - hw_values[i]);
        if (verbose == 2)
            std::cout << std::setprecision(14) << i << " : y_gold = " << sw_values[i]
                      << "\ty_hw = " << hw_values[i] << "\n";
        if (diff >= diff_thres || diff != diff) {
            status = 1;
            ++err_cnt;
            if (verbose == 1 || verbose == 2)
                std::cout << std::setprecision(14) << "\tError occurs at " << i << " : y_gold = "
                          << sw_values[i] << ", y_hw = " << hw_values[i]
                          << ". Relative difference is " << std::fabs(diff / sw_values[i]) << "\n";
        }
    }
    if (status)
        std::cout << "Total errors : " << err_cnt << "\n";
    std::cout.flush();
    return status;
}

}  // extern "C"
