// Host-only check program for the sanitizer builds (tests/sanitize/Makefile): drives the host
// code of libspmv_hw -- the multi-threaded reader (reader.cpp), the row partition, the exchange
// schedule, the threaded accum_results '+=' (host.cpp), verification and storage_overhead --
// compiled with g++ under AddressSanitizer + UBSan and under ThreadSanitizer. No HIP.
//
//   host_check read <file.mtx> <out.bin>   spmv_read_csr -> binary dump (n, m, nnz, row_ptr, col, val)
//                                          and the header/matrix pair of calls, compared
//   host_check partition                   random row_ptr, 1..16 units, against a restated S1 rule
//   host_check schedule                    every exchange at 1..8 ranks, rows covered once
//   host_check accumulate                  producer threads land parts while 16 threads add them
//   host_check verify                      verification / storage_overhead semantics
// Prints "OK <what>" and exits 0; any failed check prints "FAIL ..." and exits 1.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "spmv_host.hpp"

using namespace spmvhw;

#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

static int cmd_read(const char *path, const char *out)
{
    csr_matrix m;
    const int rc = spmv_read_csr(path, &m);
    if (rc) {
        std::printf("READ_ERROR %d %s\n", rc, spmv_hw_last_error());
        return 0;  // an error code is a result too (the caller compares it)
    }
    // the two-call form (csr.cpp's read_csr_header + read_csr_matrix) gives the same arrays
    csr_header h;
    CHECK(spmv_read_csr_header(&h, path) == 0);
    CHECK(h.nr_rows == m.nr_rows && h.nr_cols == m.nr_cols && h.nr_nzeros == m.nr_nzeros);
    csr_matrix m2;
    std::memset(&m2, 0, sizeof(m2));
    m2.nr_rows = h.nr_rows;
    m2.nr_cols = h.nr_cols;
    m2.nr_nzeros = h.nr_nzeros;
    std::vector<IndexType> rp(size_t(h.nr_rows) + 1), ci(std::max<size_t>(h.nr_nzeros, 1));
    std::vector<ValueType> va(std::max<size_t>(h.nr_nzeros, 1));
    m2.row_ptr = rp.data();
    m2.col_ind = ci.data();
    m2.values = va.data();
    CHECK(spmv_read_csr_matrix(&m2, path) == 0);
    CHECK(std::memcmp(rp.data(), m.row_ptr, rp.size() * sizeof(IndexType)) == 0);
    CHECK(std::memcmp(ci.data(), m.col_ind, size_t(h.nr_nzeros) * sizeof(IndexType)) == 0);
    CHECK(std::memcmp(va.data(), m.values, size_t(h.nr_nzeros) * sizeof(ValueType)) == 0);
    FILE *f = std::fopen(out, "wb");
    CHECK(f);
    const uint64_t head[4] = {m.nr_rows, m.nr_cols, m.nr_nzeros, sizeof(ValueType)};
    CHECK(std::fwrite(head, sizeof(head), 1, f) == 1);
    CHECK(std::fwrite(m.row_ptr, sizeof(IndexType), size_t(m.nr_rows) + 1, f) == size_t(m.nr_rows) + 1);
    if (m.nr_nzeros) {
        CHECK(std::fwrite(m.col_ind, sizeof(IndexType), m.nr_nzeros, f) == m.nr_nzeros);
        CHECK(std::fwrite(m.values, sizeof(ValueType), m.nr_nzeros, f) == m.nr_nzeros);
    }
    std::fclose(f);
    spmv_free_csr(&m);
    std::printf("OK read %s\n", path);
    return 0;
}

static int cmd_partition()
{
    std::mt19937_64 g(5);
    for (int it = 0; it < 300; ++it) {
        const uint32_t n = it % 10 == 0 ? 0 : uint32_t(g() % 5000);
        std::vector<IndexType> rp(size_t(n) + 1, 0);
        const uint64_t base = it % 3 == 0 ? 1000 : 0;  // a slice of a larger matrix starts past 0
        rp[0] = (IndexType)base;
        for (uint32_t i = 0; i < n; ++i)
            rp[i + 1] = rp[i] + (IndexType)(g() % 7 == 0 ? g() % 400 : g() % 6);
        for (int units = 1; units <= 16; ++units) {
            std::vector<IndexType> b(units + 1, 0xdeadbeef);
            CHECK(spmv_partition_rows(rp.data(), n, units, b.data()) == 0);
            CHECK(b[0] == 0 && b[units] == n);
            const uint64_t nnz = rp[n] - rp[0];
            for (int u = 1; u < units; ++u) {
                CHECK(b[u] >= b[u - 1]);
                // restated S1 rule: the first row whose start reaches u/units of the non-zeros
                const uint64_t target = rp[0] + nnz * uint64_t(u) / uint64_t(units);
                uint32_t want = 0;
                while (want < n && rp[want] < target)
                    ++want;
                CHECK(b[u] == std::max<IndexType>(want, b[u - 1]));
            }
        }
    }
    IndexType one[2];
    CHECK(spmv_partition_rows(nullptr, 0, 1, one) == 1);
    CHECK(std::strlen(spmv_hw_last_error()) > 0);
    std::printf("OK partition\n");
    return 0;
}

static int cmd_schedule()
{
    std::mt19937_64 g(9);
    for (int it = 0; it < 400; ++it) {
        const int nr = 1 + int(g() % 8);
        const uint32_t n = it % 17 == 0 ? 0 : uint32_t(g() % 3000);
        std::vector<IndexType> b(nr + 1, 0);
        for (int r = 1; r < nr; ++r)
            b[r] = (IndexType)(g() % (size_t(n) + 1));
        b[nr] = n;
        std::sort(b.begin(), b.end());
        for (int ex = SPMV_MGPU_GATHER; ex <= SPMV_MGPU_ALLGATHER; ++ex) {
            std::vector<int> cover(n, 0);
            std::vector<std::vector<spmv_xop>> all(nr);
            for (int r = 0; r < nr; ++r) {
                const int cnt = spmv_mgpu_schedule(ex, r, nr, b.data(), nullptr, 0);
                CHECK(cnt >= 0 && cnt <= 2 + 2 * nr);
                all[r].resize(cnt + 1);
                CHECK(spmv_mgpu_schedule(ex, r, nr, b.data(), all[r].data(), cnt) == cnt);
                all[r].resize(cnt);
                for (const spmv_xop &o : all[r]) {
                    CHECK(o.count > 0);
                    const uint64_t len = o.buf == SPMV_XBUF_SLICE ? b[r + 1] - b[r] : n;
                    CHECK(uint64_t(o.offset) + o.count <= len);
                    if (ex == SPMV_MGPU_GATHER && r == 0)
                        for (uint32_t i = o.offset; i < o.offset + o.count; ++i)
                            ++cover[i];
                }
            }
            if (ex == SPMV_MGPU_GATHER)
                for (uint32_t i = 0; i < n; ++i)
                    CHECK(cover[i] == 1);
            if (ex == SPMV_MGPU_ALLGATHER)  // every rank lists the same broadcasts
                for (int r = 1; r < nr; ++r) {
                    std::vector<spmv_xop> a, c;
                    for (const spmv_xop &o : all[0])
                        if (o.kind == SPMV_XOP_BCAST)
                            a.push_back(o);
                    for (const spmv_xop &o : all[r])
                        if (o.kind == SPMV_XOP_BCAST)
                            c.push_back(o);
                    CHECK(a.size() == c.size());
                    for (size_t k = 0; k < a.size(); ++k)
                        CHECK(std::memcmp(&a[k], &c[k], sizeof(spmv_xop)) == 0);
                }
        }
    }
    spmv_xop o;
    CHECK(spmv_mgpu_schedule(5, 0, 1, nullptr, &o, 1) == -1);
    std::printf("OK schedule\n");
    return 0;
}

// a part "lands" when its flag is set (release) by a producer thread: the stand-in for the DMA
// copy and its event; the wait spins with acquire, as hipEventSynchronize orders the host reads
struct Landing {
    std::atomic<int> done{0};
};

static int wait_flag(void *ready, std::string *err)
{
    Landing *l = static_cast<Landing *>(ready);
    for (int spin = 0; !l->done.load(std::memory_order_acquire); ++spin) {
        if (spin > 200000000) {
            *err = "part never landed";
            return 1;
        }
        std::this_thread::yield();
    }
    return 0;
}

static int cmd_accumulate()
{
    std::mt19937_64 g(3);
    for (int round = 0; round < 12; ++round) {
        const size_t units = 1 + round % 4, pieces = 1 + g() % 9;
        const uint64_t rows = round % 3 == 0 ? 1000 : 300000 + g() % 100000;  // below / above 2^18
        std::vector<ValueType> y(rows * units), want(rows * units);
        for (size_t i = 0; i < y.size(); ++i)
            y[i] = want[i] = ValueType(int(g() % 100)) / 4;
        std::vector<std::vector<ValueType>> stage(units, std::vector<ValueType>(rows));
        std::vector<ValueType> src(rows * units);
        for (size_t i = 0; i < src.size(); ++i) {
            src[i] = ValueType(int(g() % 100)) / 8;
            want[i] += src[i];
        }
        std::vector<Landing> land(units * pieces);
        std::vector<add_part> parts;
        for (size_t j = 0; j < pieces; ++j)  // landing order: piece j of every unit
            for (size_t u = 0; u < units; ++u) {
                const uint64_t b = rows * j / pieces, e = rows * (j + 1) / pieces;
                parts.push_back({y.data() + u * rows + b, stage[u].data() + b, e - b, &land[u * pieces + j]});
            }
        // one producer per unit copies its pieces into the staging buffer, in order
        std::vector<std::thread> prod;
        for (size_t u = 0; u < units; ++u)
            prod.emplace_back([&, u] {
                for (size_t j = 0; j < pieces; ++j) {
                    const uint64_t b = rows * j / pieces, e = rows * (j + 1) / pieces;
                    std::memcpy(stage[u].data() + b, src.data() + u * rows + b, (e - b) * sizeof(ValueType));
                    land[u * pieces + j].done.store(1, std::memory_order_release);
                    std::this_thread::sleep_for(std::chrono::microseconds(50 * (j % 3)));
                }
            });
        accum_options o;
        o.split = round % 2 == 0;
        o.prefault = round % 4 != 1;
        o.threads = 16;
        bool failed = true;
        std::string err;
        const double t = host_accumulate(parts.data(), parts.size(), wait_flag, o, &failed, &err);
        for (auto &p : prod)
            p.join();
        CHECK(!failed && t > 0);
        for (size_t i = 0; i < y.size(); ++i)
            CHECK(y[i] == want[i]);
    }
    // nothing to add: returns at once
    bool failed = true;
    accum_options o;
    host_accumulate(nullptr, 0, wait_flag, o, &failed, nullptr);
    CHECK(!failed);
    std::printf("OK accumulate\n");
    return 0;
}

static int cmd_verify()
{
    std::vector<ValueType> a(100), b(100);
    for (int i = 0; i < 100; ++i)
        a[i] = b[i] = ValueType(i) / 7;
    CHECK(verification(100, a.data(), b.data(), 0) == 0);
    b[17] += ValueType(1e-3);
    b[42] = std::nan("");
    CHECK(verification(100, a.data(), b.data(), 1) == 1);
    CHECK(verification(0, nullptr, nullptr, 0) == 0);
    IndexType ci[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, vl[2] = {0xFFFFFFFFu, 1};
    csr_hw_matrix m;
    std::memset(&m, 0, sizeof(m));
    m.nr_ci = ci;
    m.nr_val = vl;
    m.blocks = 2;
    const double mb = (double)storage_overhead(&m);
    const double want = (2.0 * 5 * 32 + (3.0 * 4294967295.0 + 1.0) * 128) / (8.0 * 1024 * 1024);
    CHECK(std::fabs(mb - want) <= want * 1e-6);
    CHECK(storage_overhead(nullptr) == 0);
    std::printf("OK verify\n");
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 4 && !std::strcmp(argv[1], "read"))
        return cmd_read(argv[2], argv[3]);
    if (argc >= 2 && !std::strcmp(argv[1], "partition"))
        return cmd_partition();
    if (argc >= 2 && !std::strcmp(argv[1], "schedule"))
        return cmd_schedule();
    if (argc >= 2 && !std::strcmp(argv[1], "accumulate"))
        return cmd_accumulate();
    if (argc >= 2 && !std::strcmp(argv[1], "verify"))
        return cmd_verify();
    std::fprintf(stderr, "usage: host_check read <mtx> <out> | partition | schedule | accumulate | verify\n");
    return 2;
}
