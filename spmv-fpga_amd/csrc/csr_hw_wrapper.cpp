// The reference API (csr_hw_wrapper.h:9-17, csr_hw.h:140,148) as a thin C-ABI shim over the
// MI355X plans. One handle per unit ("Compute Unit" -> GPU, util.h:41-59); units own
// contiguous nnz-balanced row slices (the role of prepare_balanced_hw_matrix's S1 split,
// csr_hw.cpp:459). x is replicated on every GPU in use (the reference copies x into every CU's
// BRAM, spmv.cpp:280-294). spmv_hw runs every unit's kernels, then adds each unit's y slice
// into the caller's y_fpga (the role of accum_results, csr_hw.cpp:1531-1565, and the loop
// csr_hw_wrapper.cpp:276-281), printing the reference's timing lines. By default every GPU's
// slice comes back over its own PCIe link (SPMV_HW_MERGE=auto|host); with SPMV_HW_MERGE=gather
// (or reduce) the slices first meet on GPU 0 over xGMI (an RCCL gather of the disjoint slices,
// or the literal ncclReduce(sum) of full-length partials) and one D2H copy brings y to the host.
#include <sys/mman.h>
#include <sys/time.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <atomic>
#include <mutex>
#include <functional>
#include <thread>

#include "spmv_internal.hpp"

using namespace spmvhw;

namespace {

[[noreturn]] void die(const std::string &what)
{
    std::fprintf(stderr, "spmv_hw: %s\n", what.c_str());
    std::fflush(stderr);
    std::exit(1);
}

void check(hipError_t e, const char *what)
{
    if (e != hipSuccess)
        die(std::string(what) + ": " + hipGetErrorString(e));
}

int device_count()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1)
        die("no HIP device available (the MI355X path has no CPU fallback)");
    return n;
}

int unit_device(int unit) { return unit % device_count(); }

// how spmv_hw merges the unit slices (env SPMV_HW_MERGE, read by create_csr_hw_matrix)
enum { kMergeHost = 0, kMergeGather = 1, kMergeReduce = 2 };

// completion events of the pieces of one y copy (device-to-host), created on first use on the
// device whose stream records them
struct d2h_events {
    int device = 0;
    std::vector<hipEvent_t> ev;
    hipEvent_t get(size_t k)
    {
        while (ev.size() <= k) {
            hipEvent_t e = nullptr;
            check(hipSetDevice(device), "hipSetDevice");
            const char *bs = ablation_env("SPMV_HW_BLOCKING_SYNC");
            check(hipEventCreateWithFlags(&e, hipEventDisableTiming | (bs && bs[0] == '1' ? hipEventBlockingSync : 0)),
                  "hipEventCreate");
            ev.push_back(e);
        }
        return ev[k];
    }
    ~d2h_events()
    {
        for (hipEvent_t e : ev)
            (void)hipEventDestroy(e);
    }
};

// the RCCL clique of a matrix whose units sit on distinct GPUs (owned by unit 0's handle)
struct hw_clique {
    spmv_mgpu *mg = nullptr;
    int mode = kMergeGather;
    std::vector<int> devices;       // of units 0..n-1
    ValueType *h_full = nullptr;    // pinned staging of the whole y
    uint64_t rows = 0;
    d2h_events done;                // of the y copy's pieces (device 0)
    ~hw_clique()
    {
        if (mg)
            spmv_mgpu_destroy(mg);
        if (h_full)
            (void)hipHostFree(h_full);
    }
};

struct hw_matrix_impl {
    csr_hw_matrix pub;  // must stay the first member: callers see a csr_hw_matrix*
    spmv_plan *plan = nullptr;
    hw_clique *clique = nullptr;  // unit 0 only
    int unit = 0, device = 0;
    IndexType row_begin = 0, row_end = 0;
    // spmv_hw scratch, kept across calls: the unit's y slice on its GPU and a pinned host
    // staging copy (the reference allocates its y per call, csr_hw_wrapper.cpp:198,287)
    ValueType *d_y = nullptr;
    ValueType *h_stage = nullptr;
    d2h_events done;  // of the y copy's pieces
    // streamed copy-back (plans whose sweep flags each panel's y, sweep_can_flag_panels): the
    // panel flags in pinned host memory, the call's epoch, the panels' row bounds and the stream
    // the pieces' copies run on while the kernel still sweeps
    uint32_t *h_flags = nullptr;
    uint32_t *d_flags = nullptr;
    ValueType *h_direct = nullptr;  // (tools build, SPMV_HW_DIRECT=1) y stored by the sweep over PCIe
    ValueType *d_direct = nullptr;
    uint32_t epoch = 0;
    std::vector<uint32_t> panel_rows;
    hipStream_t copy_stream = nullptr;
    BusDataType *sub[1] = {nullptr};
    IndexType nr_rows[1] = {0}, nr_cols[1] = {0}, nr_nzeros[1] = {0}, nr_ci[1] = {0}, nr_val[1] = {0};
};

struct hw_vector_impl {
    csr_hw_vector pub;  // first member
    BusDataType *vals[1] = {nullptr};
    IndexType nr_values[1] = {0};
    std::vector<ValueType *> per_device;  // x: a copy on every device in use; y: one buffer
    int device = 0;
};

hw_matrix_impl *impl(csr_hw_matrix *m) { return reinterpret_cast<hw_matrix_impl *>(m); }

// The unit arrays (hw_matrix, hw_y) carry one extra null entry, so every call knows the unit
// count of the matrix it was given (several matrices with different SPMV_NGPUS may coexist).
template <typename T>
int units_of(T **arr)
{
    int u = 0;
    while (arr[u])
        ++u;
    return u;
}
hw_vector_impl *impl(csr_hw_vector *v) { return reinterpret_cast<hw_vector_impl *>(v); }

std::mutex g_mu;
int g_units_max = 0;                    // most units of any create_csr_hw_matrix so far (x upload)
std::vector<hipStream_t> g_streams;     // one stream per unit

hipStream_t unit_stream(int unit)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_streams.size() <= unit)
        g_streams.resize(unit + 1, nullptr);
    if (!g_streams[unit]) {
        check(hipSetDevice(unit_device(unit)), "hipSetDevice");
        check(hipStreamCreateWithFlags(&g_streams[unit], hipStreamNonBlocking), "hipStreamCreate");
    }
    return g_streams[unit];
}

// device y and pinned staging of unit m (once per matrix)
void alloc_y_scratch(hw_matrix_impl *m)
{
    const uint64_t rows = m->row_end - m->row_begin;
    check(hipSetDevice(m->device), "hipSetDevice");
    if (!m->d_y)  // (create_csr_hw_matrix makes both while the plan builds)
        check(hipMalloc((void **)&m->d_y, rows * sizeof(ValueType)), "hipMalloc(y)");
    if (!m->h_stage)
        check(hipHostMalloc((void **)&m->h_stage, rows * sizeof(ValueType), hipHostMallocDefault),
              "hipHostMalloc(y stage)");
}

uint64_t ceil16(uint64_t bytes) { return (bytes + 15) / 16; }

// auto (default) and host: the host merge (y_fpga is host memory: G slices come back over G PCIe
// links at once); gather | reduce: the RCCL forms (one unit per GPU; they fail
// fast when RCCL cannot form the clique)
int merge_mode(int units)
{
    const char *e = std::getenv("SPMV_HW_MERGE");
    const int ndev = device_count();
    if (!e || !*e || !std::strcmp(e, "auto") || !std::strcmp(e, "host"))
        return kMergeHost;
    const int m = !std::strcmp(e, "gather") ? kMergeGather : !std::strcmp(e, "reduce") ? kMergeReduce : -1;
    if (m < 0)
        die(std::string("SPMV_HW_MERGE=") + e + ": expected auto, host, gather or reduce");
    if (units > ndev)
        die(std::string("SPMV_HW_MERGE=") + e + " needs one unit per GPU (" + std::to_string(units) + " units, " +
            std::to_string(ndev) + " devices)");
    return m;
}

// spmv_hw copies a unit's y back while its sweep still runs (SPMV_HW_STREAM, default on; 0 off)
bool stream_enabled()
{
    const char *e = std::getenv("SPMV_HW_STREAM");
    return !(e && e[0] == '0');
}

// The copy pattern of spmv_hw's unstreamed host merge (`pieces` copies of y into the pinned
// staging, each followed by its event), run three times on the unit's stream at create time for
// plans that do not stream their copy-back. One whole-y warm copy alone left the second
// spmv_hw call's enqueue of the pieces stalling for ~10 ms (and a later one for a few ms) in most
// processes measured (profiles/r06zu_*, r06zv_*): the runtime's first uses of that many copies
// and events on a stream happen here instead. Streamed plans (copies on their own stream) never
// showed it and skip this (it adds ~25 ms to create_csr_hw_matrix at 10M rows).
void warm_copies(ValueType *stage, const ValueType *d_src, uint64_t rows, uint64_t pieces, hipStream_t s,
                 d2h_events &done)
{
    for (int rep = 0; rep < 3 && rows; ++rep) {
        for (uint64_t t = 0; t < pieces; ++t) {
            const uint64_t b = rows * t / pieces, e = rows * (t + 1) / pieces;
            check(hipMemcpyAsync(stage + b, d_src + b, (e - b) * sizeof(ValueType), hipMemcpyDeviceToHost, s),
                  "warm D2H");
            check(hipEventRecord(done.get(t), s), "warm D2H");
        }
        check(hipStreamSynchronize(s), "warm D2H");
    }
}

// streamed copy-back of unit m (host merge): pinned panel flags the sweep kernel writes, the
// panels' row bounds on the host and a copy stream (its first large copy run here, like the
// unit stream's)
void setup_streaming(hw_matrix_impl *m)
{
    const spmv_plan &pl = *m->plan;
    if (!sweep_can_flag_panels(pl) || m->row_end == m->row_begin) {
        if (m->copy_stream) {  // (created ahead by create_csr_hw_matrix; not needed)
            check(hipSetDevice(m->device), "hipSetDevice");
            (void)hipStreamDestroy(m->copy_stream);
            m->copy_stream = nullptr;
        }
        return;
    }
    check(hipSetDevice(m->device), "hipSetDevice");
    m->panel_rows.resize(pl.npanels + 1);
    check(hipMemcpy(m->panel_rows.data(), pl.d_panel_row, (pl.npanels + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost),
          "panel rows");
    check(hipHostMalloc((void **)&m->h_flags, pl.npanels * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped),
          "hipHostMalloc(panel flags)");
    std::memset(m->h_flags, 0, pl.npanels * sizeof(uint32_t));
    check(hipHostGetDevicePointer((void **)&m->d_flags, m->h_flags, 0), "hipHostGetDevicePointer(panel flags)");
    if (!m->copy_stream)  // (else made by create_csr_hw_matrix while the plan built)
        check(hipStreamCreateWithFlags(&m->copy_stream, hipStreamNonBlocking), "hipStreamCreate");
    const uint64_t rows = m->row_end - m->row_begin;
    if (ablation_env("SPMV_HW_DIRECT") && pl.kernel == kKernelSweep) {  // the measurement form: y straight
                                                                         // into host memory (sweep only)
        check(hipHostMalloc((void **)&m->h_direct, rows * sizeof(ValueType), hipHostMallocCoherent | hipHostMallocMapped),
              "hipHostMalloc(direct y)");
        check(hipHostGetDevicePointer((void **)&m->d_direct, m->h_direct, 0), "hipHostGetDevicePointer(direct y)");
    }
    check(hipMemcpyAsync(m->h_stage, m->d_y, rows * sizeof(ValueType), hipMemcpyDeviceToHost, m->copy_stream),
          "warm D2H");
    check(hipStreamSynchronize(m->copy_stream), "warm D2H");
}

int env_pieces(int dflt)
{
    const char *e = ablation_env("SPMV_HW_PIECES");
    return e ? std::max(1, std::atoi(e)) : dflt;
}


// Panel bounds of a streamed copy-back's k pieces over P panels. The copy engine runs the pieces
// back to back, so what is left when the last copy lands is that piece's host add: the pieces
// taper (weights 16, 16, ..., 8, 4, 2, 1, 1 -- the last two 1/64 of y each at k = 8) instead of
// k equal parts. The tools build's SPMV_HW_PIECE_SHAPE=equal gives the equal parts.
std::vector<uint32_t> piece_bounds(uint32_t P, uint32_t k)
{
    std::vector<uint32_t> q(k + 1, 0);
    const char *sh = ablation_env("SPMV_HW_PIECE_SHAPE");
    const bool equal = k < 4 || (sh && std::strcmp(sh, "equal") == 0);
    std::vector<uint64_t> w(k, 1);
    if (!equal)
        for (int j = (int)k - 3; j >= 0; --j)
            w[j] = std::min<uint64_t>(16, 2 * w[j + 1]);
    uint64_t W = 0;
    for (uint64_t v : w)
        W += v;
    uint64_t c = 0;
    for (uint32_t j = 1; j <= k; ++j) {
        c += w[j - 1];
        // at least one panel per piece (k <= P)
        const uint64_t b = uint64_t(P) * c / W;
        q[j] = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(b, q[j - 1] + 1), P - (k - j));
    }
    return q;
}

// Copies rows [0, rows) of a device y slice into pinned staging on stream s as `pieces` copies,
// each followed by an event, and appends one add_part per piece (dst = the caller's y). The
// host adds of a piece then start while later pieces are still crossing PCIe. 8 pieces of y in
// all by default (env SPMV_HW_PIECES); SPMV_HW_PIPELINE=0: one copy and one event for the whole
// slice (every add waits for all of it). Measured on 10M fp64 rows, one GPU
// (profiles/r03aq_spmv_hw_merge.jsonl): accumulation 1.86-1.91 ms pieced vs 2.71-2.93 ms whole,
// against 1.43 ms for the bare copy.
void enqueue_d2h(ValueType *y_dst, ValueType *stage, const ValueType *d_src, uint64_t rows, uint64_t pieces,
                 hipStream_t s, d2h_events &done, std::vector<add_part> &parts)
{
    const char *pe = std::getenv("SPMV_HW_PIPELINE");
    const bool pipe = !(pe && pe[0] == '0');
    if (!pipe) {
        check(hipMemcpyAsync(stage, d_src, rows * sizeof(ValueType), hipMemcpyDeviceToHost, s), "hipMemcpyAsync(y)");
        check(hipEventRecord(done.get(0), s), "hipEventRecord");
    }
    for (uint64_t t = 0; t < pieces; ++t) {
        const uint64_t b = rows * t / pieces, e = rows * (t + 1) / pieces;
        if (pipe) {
            check(hipMemcpyAsync(stage + b, d_src + b, (e - b) * sizeof(ValueType), hipMemcpyDeviceToHost, s),
                  "hipMemcpyAsync(y)");
            check(hipEventRecord(done.get(t), s), "hipEventRecord");
        }
        parts.push_back({y_dst + b, stage + b, e - b, static_cast<void *>(done.get(pipe ? t : 0))});
    }
}

int wait_event(void *ready, std::string *err)
{
    const hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(ready));
    if (e != hipSuccess)
        *err = std::string("y copy: ") + hipGetErrorString(e);
    return e != hipSuccess;
}

// One piece of a streamed copy-back: rows [b, e) of unit m's slice = its panels [q0, q1). The
// calling thread records `ev` after the piece's copy once every panel of it is flagged; until
// then an adding thread waits on `state` (0 pending, 1 copy enqueued, -1 failed).
struct streamed_piece {
    hw_matrix_impl *m = nullptr;
    uint32_t q0 = 0, q1 = 0;
    uint64_t b = 0, e = 0;
    hipEvent_t ev = nullptr;
    std::atomic<int> state{0};
    std::string err;
    double t_ready = 0.0, t_enq = 0.0;  // (SPMV_HW_TRACE) flags all seen / copy enqueued, timestamp_us
    std::atomic<int64_t> t_landed{0};   // (SPMV_HW_TRACE) first adding thread to see the copy done, us
    hipEvent_t t_copied = nullptr;      // (SPMV_HW_TRACE) timing event after the copy, device clock
    bool by_flags = false;              // the flags, not the end of the kernels, released the piece
};

int wait_streamed(void *ready, std::string *err)
{
    auto *pc = static_cast<streamed_piece *>(ready);
    int st;
    while ((st = pc->state.load(std::memory_order_acquire)) == 0)
        std::this_thread::yield();
    if (st < 0) {
        *err = pc->err;
        return 1;
    }
    if (pc->ev && wait_event(pc->ev, err))
        return 1;  // (direct form: the flags were the landing)
    int64_t none = 0;
    pc->t_landed.compare_exchange_strong(none, (int64_t)timestamp_us(), std::memory_order_relaxed);
    return 0;
}

// Copy each piece as soon as its panels are flagged, in landing order, on the calling thread --
// the only thread that asks about the units' kernel streams (a runtime call on a stream another
// thread is synchronising on waits for that synchronisation: the flags would be seen at the end
// of the kernel only). A piece whose flags do not all arrive is copied once its unit's kernels
// have ended (y is final then), so this returns whatever the kernel did; a failed kernel or copy
// marks the rest of the pieces failed. Returns when every piece's copy is enqueued and every
// unit's kernels have ended, and when (timestamp_us) the last of them was seen to end.
double feed_pieces(std::vector<streamed_piece> &pcs, const std::vector<hw_matrix_impl *> &us,
                   std::vector<double> *seen)
{
    std::string fail;
    std::vector<double> ended(us.size(), 0.0);
    auto poll_units = [&]() {  // has each unit's launch ended? (first time seen, timestamp_us)
        bool all = true;
        for (size_t k = 0; k < us.size(); ++k) {
            if (ended[k] > 0.0)
                continue;
            const hipError_t q = hipStreamQuery(unit_stream(us[k]->unit));
            if (q == hipSuccess) {
                ended[k] = timestamp_us();
            } else {
                all = false;
                if (q != hipErrorNotReady && fail.empty())
                    fail = std::string("spmv kernels: ") + hipGetErrorString(q);
            }
        }
        return all;
    };
    auto unit_ended = [&](const hw_matrix_impl *m) {
        for (size_t k = 0; k < us.size(); ++k)
            if (us[k] == m)
                return ended[k] > 0.0;
        return true;
    };
    for (streamed_piece &pc : pcs) {
        hw_matrix_impl *m = pc.m;
        for (uint32_t spin = 0; fail.empty(); ++spin) {
            if (seen && pc.m == pcs[0].m) {  // (SPMV_HW_TRACE) when each panel's flag was first seen
                const uint32_t P = (uint32_t)seen->size();
                for (uint32_t q = 0; q < P; ++q)
                    if ((*seen)[q] == 0.0 && __atomic_load_n(&m->h_flags[q], __ATOMIC_ACQUIRE) == m->epoch)
                        (*seen)[q] = timestamp_us();
            }
            bool all = true;
            for (uint32_t q = pc.q0; q < pc.q1 && all; ++q)
                all = __atomic_load_n(&m->h_flags[q], __ATOMIC_ACQUIRE) == m->epoch;
            if (all) {
                pc.by_flags = true;
                break;
            }
            if (spin % 16 == 15) {
                poll_units();
                if (unit_ended(m))
                    break;
            }
        }
        pc.t_ready = timestamp_us();
        if (fail.empty() && m->plan->y_host) {
            // direct form: the rows are in host memory already (a piece released by the kernel's
            // end is too: the end of the kernel publishes every store at system scope)
            pc.ev = nullptr;
        } else if (fail.empty()) {
            hipError_t e = hipSetDevice(m->device);
            if (e == hipSuccess)
                e = hipMemcpyAsync(m->h_stage + pc.b, m->d_y + pc.b, (pc.e - pc.b) * sizeof(ValueType),
                                   hipMemcpyDeviceToHost, m->copy_stream);
            if (e == hipSuccess)
                e = hipEventRecord(pc.ev, m->copy_stream);
            if (e == hipSuccess && pc.t_copied)
                e = hipEventRecord(pc.t_copied, m->copy_stream);
            if (e != hipSuccess)
                fail = std::string("y copy: ") + hipGetErrorString(e);
            pc.t_enq = timestamp_us();
        }
        if (!fail.empty()) {
            pc.err = fail;
            pc.state.store(-1, std::memory_order_release);
        } else {
            pc.state.store(1, std::memory_order_release);
        }
    }
    while (fail.empty() && !poll_units())
        std::this_thread::yield();
    if (!fail.empty())
        die(fail);
    return *std::max_element(ended.begin(), ended.end());
}

// accum_results' '+=' of the landed pieces into the caller's y (spmv_host.hpp, host.cpp) on up
// to 16 host threads; returns when (timestamp_us) the last copy was seen complete. The
// documented knob SPMV_HW_PREFAULT=0 lets the adds take the page faults; the split and thread
// count are switches of the tools build.
double accumulate(const std::vector<add_part> &parts, int (*wait)(void *, std::string *) = wait_event,
                  int threads = accum_options().threads)
{
    accum_options o;
    o.threads = threads;
    const char *pf = std::getenv("SPMV_HW_PREFAULT");
    o.prefault = !(pf && pf[0] == '0');
    const char *se = ablation_env("SPMV_HW_ADD_SPLIT");
    o.split = !(se && se[0] == '0');
    if (const char *te = ablation_env("SPMV_HW_ADD_THREADS"))
        o.threads = std::max(1, std::atoi(te));
    bool failed = false;
    std::string err;
    const double landed = host_accumulate(parts.data(), parts.size(), wait, o, &failed, &err);
    if (failed)
        die(err);
    return landed;
}

// spmv_hw with the host merge on plans whose sweep flags each panel (csr_hw_wrapper.cpp:193-288):
// every unit's kernel is launched with this call's epoch; the calling thread copies each piece
// of y (8 pieces in all, whole panels each) as soon as its panels are flagged, and the adding
// threads add every piece as soon as it landed -- so the PCIe copy-back and the host '+=' run
// while the SpMV still sweeps, instead of after it. The printed times keep the reference's
// meaning: "Hardware execution" ends when every unit's kernels have ended, "Result accumulation"
// when the last add is done (what of it was overlapped is no longer counted there).
void spmv_hw_streamed(csr_hw_matrix **hw_matrix, int units, hw_vector_impl *x, csr_vector *y_fpga, bool trace)
{
    auto tr = [&](const char *what, double since) {
        if (trace)
            std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", what, (timestamp_us() - since) / 1000);
    };
    // pieces: piece j of every unit, then j + 1 (landing order); each piece whole panels
    std::vector<std::pair<hw_matrix_impl *, uint32_t>> cuts;  // (unit, pieces)
    size_t n = 0;
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        if (m->row_end == m->row_begin)
            continue;
        const uint64_t rows = m->row_end - m->row_begin;
        const uint32_t P = (uint32_t)m->panel_rows.size() - 1;
        const uint32_t k = std::min<uint32_t>(P, rows < (1u << 18) ? 1u : (uint32_t)std::max(2, env_pieces(8) / units));
        cuts.push_back({m, k});
        n += k;
    }
    std::vector<streamed_piece> pcs(n);
    std::vector<std::vector<uint32_t>> qb;
    for (auto &c : cuts)
        qb.push_back(piece_bounds((uint32_t)c.first->panel_rows.size() - 1, c.second));
    size_t i = 0;
    for (uint32_t j = 0, more = 1; more; ++j) {
        more = 0;
        for (size_t ci = 0; ci < cuts.size(); ++ci) {
            auto &c = cuts[ci];
            if (j >= c.second)
                continue;
            more = 1;
            hw_matrix_impl *m = c.first;
            streamed_piece &pc = pcs[i++];
            pc.m = m;
            pc.q0 = qb[ci][j];
            pc.q1 = qb[ci][j + 1];
            pc.b = m->panel_rows[pc.q0];
            pc.e = m->panel_rows[pc.q1];
            m->done.device = m->device;
            pc.ev = m->done.get(j);
        }
    }
    // (tools build) SPMV_HW_DIRECT=1: every unit's sweep stores y straight into host memory
    const char *de = ablation_env("SPMV_HW_DIRECT");
    bool direct = de && de[0] == '1';
    for (auto &c : cuts)
        direct = direct && c.first->d_direct;
    std::vector<add_part> parts(n);
    for (size_t k = 0; k < n; ++k)
        parts[k] = {y_fpga->values + pcs[k].m->row_begin + pcs[k].b,
                    (direct ? pcs[k].m->h_direct : pcs[k].m->h_stage) + pcs[k].b, pcs[k].e - pcs[k].b,
                    static_cast<void *>(&pcs[k])};

    // (SPMV_HW_TRACE) device-clock times of each piece's copy, from its unit's kernel launch
    std::vector<hipEvent_t> t_launch(units, nullptr);
    if (trace) {
        for (int u = 0; u < units; ++u) {
            check(hipSetDevice(impl(hw_matrix[u])->device), "hipSetDevice");
            check(hipEventCreate(&t_launch[u]), "hipEventCreate");
        }
        for (streamed_piece &pc : pcs) {
            check(hipSetDevice(pc.m->device), "hipSetDevice");
            check(hipEventCreate(&pc.t_copied), "hipEventCreate");
        }
    }
    const double hw_s = timestamp_us();
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        if (m->row_end == m->row_begin)
            continue;
        if (t_launch[u])
            check(hipEventRecord(t_launch[u], unit_stream(u)), "hipEventRecord");
        if (++m->epoch == 0)  // (0 is the flags' initial value)
            m->epoch = 1;
        m->plan->y_flag = m->d_flags;
        m->plan->y_epoch = m->epoch;
        m->plan->y_host = direct ? m->d_direct : nullptr;
        const int rc = spmv_plan_run(m->plan, x->per_device[m->device], m->d_y, unit_stream(u));
        m->plan->y_flag = nullptr;
        if (rc)
            die(std::string("spmv_hw: ") + spmv_hw_last_error());
    }
    tr("spmv_hw: launches", hw_s);
    std::vector<double> seen(trace && !cuts.empty() ? cuts[0].first->panel_rows.size() - 1 : 0, 0.0);
    std::vector<hw_matrix_impl *> us;
    for (auto &c : cuts)
        us.push_back(c.first);
    double landed = 0.0;
    // 8 adding threads: the streamed adds keep pace with the copy engine's ~52 GB/s on 8, and
    // fewer threads leave the feeding thread its core (interleaved A/B on the 10M/160M plan,
    // profiles/r06zg_spmv_hw_pieces_threads_ab.jsonl: Total 2.09 / 2.15 / 2.20 ms on 8 / 12 / 16
    // threads; the unstreamed merge, whose adds start after the kernel, keeps 16)
    std::thread adder([&] { landed = accumulate(parts, wait_streamed, 8); });
    const double hw_f = us.empty() ? timestamp_us() : feed_pieces(pcs, us, trace ? &seen : nullptr);
    for (hw_matrix_impl *m : us)
        m->plan->y_host = nullptr;
    const double hw_exec = (hw_f - hw_s) / 1000.0;
    std::printf("Hardware execution time : %.6f ms elapsed\n", hw_exec);
    adder.join();  // (accumulate exits the process on a failed piece)
    if (trace) {
        std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", "spmv_hw: D2H landed (streamed)", (landed - hw_f) / 1000);
        std::vector<double> t;
        for (double v : seen)
            if (v > 0.0)
                t.push_back((v - hw_s) / 1000);
        std::sort(t.begin(), t.end());
        if (!t.empty())
            std::fprintf(stderr, "spmv_hw trace:   unit 0: %zu of %zu panel flags seen while the pieces were fed; "
                                 "first %.3f, median %.3f, last %.3f ms after the launch\n",
                         t.size(), seen.size(), t.front(), t[t.size() / 2], t.back());
        for (const streamed_piece &pc : pcs) {
            // when each piece was released, its copy enqueued, the copy done (device clock, from
            // the unit's kernel launch) and first seen done by an adding thread (host clock)
            float copied = -1.0f;  // (the direct form records no copy; a failed query would stay
                                   // behind as the thread's last error for the next launch check)
            if (pc.ev && pc.t_copied && hipEventElapsedTime(&copied, t_launch[pc.m->unit], pc.t_copied) != hipSuccess) {
                copied = -1.0f;
                (void)hipGetLastError();
            }
            std::fprintf(stderr,
                         "spmv_hw trace:   piece unit %d panels [%u, %u) ready %.3f ms (%s), enqueued %.3f ms, "
                         "copied %.3f ms (device), landed %.3f ms\n",
                         pc.m->unit, pc.q0, pc.q1, (pc.t_ready - hw_s) / 1000, pc.by_flags ? "flags" : "kernel end",
                         (pc.t_enq - hw_s) / 1000, copied, (double(pc.t_landed.load()) - hw_s) / 1000);
        }
    }
    for (streamed_piece &pc : pcs)
        if (pc.t_copied)
            (void)hipEventDestroy(pc.t_copied);
    for (hipEvent_t e : t_launch)
        if (e)
            (void)hipEventDestroy(e);
    tr("spmv_hw: accumulation after the kernels", hw_f);
    const double ra_exec = std::max(0.0, (timestamp_us() - hw_f) / 1000.0);
    std::printf("Result accumulation time : %.6f ms elapsed\n", ra_exec);
    std::printf("Total time  : %.6f ms elapsed\n", hw_exec + ra_exec);
    std::fflush(stdout);
}

}  // namespace

extern "C" {

namespace {
std::atomic<int> g_units_hint{0};  // spmv_hw_set_units (the caller's compile-time ComputeUnits)
// the reference's largest build (CU=12, util.h:41-59): hw_matrix always has at least this many
// slots, so a caller that loops its compile-time ComputeUnits (main.cpp:86-87) over fewer units
// reads null handles (storage_overhead(NULL) = 0), never past the array
constexpr int kMaxReferenceUnits = 12;
}  // namespace

int spmv_hw_set_units(int units)
{
    const int prev = g_units_hint.exchange(units > 0 ? units : 0);
    return prev;
}

int spmv_hw_units(void)
{
    const int hint = g_units_hint.load();
    if (hint > 0)
        return hint;
    const char *s = std::getenv("SPMV_NGPUS");
    int u = s ? std::atoi(s) : 1;
    return u < 1 ? 1 : u;
}

// csr_hw_wrapper.cpp:3-80 (+ csr_hw.cpp:377-429 per CU count)
void create_csr_hw_matrix(csr_matrix *matrix, csr_hw_matrix ***hw_matrix, bool ***empty_rows_bitmap)
{
    if (!matrix || !hw_matrix || !empty_rows_bitmap)
        die("create_csr_hw_matrix: null argument");
    const int units = spmv_hw_units();
    const IndexType n = matrix->nr_rows;
    const bool trace = std::getenv("SPMV_HW_TRACE") != nullptr;
    const double t0 = timestamp_us();
    (void)device_count();  // the first HIP call of the process initialises the runtime
    if (trace)
        std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", "HIP runtime init", (timestamp_us() - t0) / 1000);
    std::vector<IndexType> bounds(units + 1, 0);
    if (spmv_partition_rows(matrix->row_ptr, n, units, bounds.data()))
        die(spmv_hw_last_error());

    const int merge = merge_mode(units);
    // null-terminated, and never shorter than the reference's largest CU count (+1)
    *hw_matrix = (csr_hw_matrix **)std::calloc(std::max(units, kMaxReferenceUnits) + 1, sizeof(csr_hw_matrix *));
    uint64_t in_bytes = 0, nnz_total = 0;
    for (int u = 0; u < units; ++u) {
        auto *h = new hw_matrix_impl();
        h->unit = u;
        h->device = unit_device(u);
        h->row_begin = bounds[u];
        h->row_end = bounds[u + 1];
        const double tp = timestamp_us();
        // the host merge's y scratch (device y, pinned staging) and its copy stream are made on a
        // helper thread while the plan builds (at 10M fp64 rows: ~27 ms against the plan's ~95;
        // the first large D2H copies stay after the build, where they do not slow its upload)
        hipError_t prep_err = hipSuccess;
        std::thread prep;
        if (h->row_end > h->row_begin && merge == kMergeHost) {
            prep = std::thread([h, &prep_err] {
                const size_t bytes = size_t(h->row_end - h->row_begin) * sizeof(ValueType);
                hipError_t e = hipSetDevice(h->device);
                if (e == hipSuccess)
                    e = hipMalloc((void **)&h->d_y, bytes);
                if (e == hipSuccess)
                    e = hipHostMalloc((void **)&h->h_stage, bytes, hipHostMallocDefault);
                if (e == hipSuccess)
                    e = hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking);
                prep_err = e;
            });
        }
        const int plan_rc = spmv_plan_create_host(&h->plan, h->device, matrix, h->row_begin, h->row_end);
        if (prep.joinable())
            prep.join();
        if (plan_rc)
            die(std::string("create_csr_hw_matrix: ") + spmv_hw_last_error());
        check(prep_err, "create_csr_hw_matrix: y staging");
        if (trace)
            std::fprintf(stderr, "spmv_hw trace: unit %d %-21s %9.3f ms\n", u, "plan", (timestamp_us() - tp) / 1000);
        const double ts = timestamp_us();
        // the streamed copy-back's panel flags, or an unstreamed plan's piece warm-up, here (the y
        // buffers and the first D2H copies were made while the plan built): none of it inside
        // spmv_hw's timed region
        const hipStream_t us = unit_stream(u);
        const IndexType rows = h->row_end - h->row_begin;
        if (rows && merge == kMergeHost) {  // the RCCL merge stages the whole y instead (below)
            alloc_y_scratch(h);  // (made by the helper above)
            // full size first (large copies take a different path whose first use costs ~20 ms)
            check(hipMemcpyAsync(h->h_stage, h->d_y, size_t(rows) * sizeof(ValueType), hipMemcpyDeviceToHost, us),
                  "warm D2H");
            check(hipStreamSynchronize(us), "warm D2H");
            setup_streaming(h);
            if (!h->h_flags) {  // a plan whose copy-back waits for the kernel: its own pieces too
                h->done.device = h->device;
                warm_copies(h->h_stage, h->d_y, rows, rows < (1u << 18) ? 1 : std::max(2, env_pieces(8) / units), us,
                            h->done);
            }
        }
        if (trace)
            std::fprintf(stderr, "spmv_hw trace: unit %d %-21s %9.3f ms\n", u, "y staging + copy warm-up",
                         (timestamp_us() - ts) / 1000);
        spmv_plan_stats st;
        spmv_plan_get_stats(h->plan, &st);
        const spmv_plan &pl = *h->plan;
        const bool sweep = pl.kernel == kKernelSweep || pl.kernel == kKernelBinned;
        const bool slices = pl.kernel == kKernelSlices;
        // stored entries of the representation (padded for tiles, sweep and slices, plain for
        // gold / FPGA order / blocked)
        const uint64_t stored = sweep    ? pl.ent_pad
                                : slices ? pl.slice_slots * kWave
                                : pl.kernel != kKernelTiles ? pl.nnz
                                                            : pl.nnz_pad;
        const uint64_t val_bytes = stored * sizeof(ValueType);
        // the index stream of the unit's representation (opaque device address)
        h->sub[0] = pl.kernel == kKernelBinned ? reinterpret_cast<BusDataType *>(pl.d_b_colw)
                    : sweep ? (pl.d_s_col ? reinterpret_cast<BusDataType *>(pl.d_s_col)
                                          : reinterpret_cast<BusDataType *>(pl.d_s_row16))
                    : (slices || pl.kernel == kKernelBlocked || pl.tile_col_bytes < 4)
                        ? reinterpret_cast<BusDataType *>(pl.d_colnar)
                        : reinterpret_cast<BusDataType *>(pl.d_col);
        h->nr_rows[0] = (IndexType)st.nr_nonempty_rows;
        h->nr_cols[0] = matrix->nr_cols;
        h->nr_nzeros[0] = (IndexType)stored;
        h->nr_ci[0] = (IndexType)ceil16(st.device_bytes - val_bytes);
        h->nr_val[0] = (IndexType)ceil16(val_bytes);
        h->pub.submatrix = h->sub;
        h->pub.nr_rows = h->nr_rows;
        h->pub.nr_cols = h->nr_cols;
        h->pub.nr_nzeros = h->nr_nzeros;
        h->pub.nr_ci = h->nr_ci;
        h->pub.nr_val = h->nr_val;
        h->pub.blocks = 1;
        (*hw_matrix)[u] = &h->pub;
        in_bytes += st.device_bytes;
        nnz_total += st.nr_nzeros;
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_units_max = std::max(g_units_max, units);
    }
    if (merge != kMergeHost) {
        // the clique is formed here (ncclCommInitAll), outside spmv_hw's timed region
        auto *c = new hw_clique();
        c->mode = merge;
        std::vector<const spmv_plan *> plans(units);
        for (int u = 0; u < units; ++u) {
            c->devices.push_back(impl((*hw_matrix)[u])->device);
            plans[u] = impl((*hw_matrix)[u])->plan;
        }
        c->rows = n;
        if (mgpu_create_borrowed(&c->mg, units, c->devices.data(), bounds.data(), matrix->nr_cols, plans.data()))
            die(std::string("create_csr_hw_matrix: RCCL merge: ") + spmv_hw_last_error());
        check(hipSetDevice(c->devices[0]), "hipSetDevice");
        check(hipHostMalloc((void **)&c->h_full, std::max<uint64_t>(n, 1) * sizeof(ValueType), hipHostMallocDefault),
              "hipHostMalloc(y stage)");
        if (n) {  // first large D2H copy here, not in the first spmv_hw (as for the host merge)
            check(hipMemcpyAsync(c->h_full, mgpu_root_y(c->mg), size_t(n) * sizeof(ValueType), hipMemcpyDeviceToHost,
                                 unit_stream(0)),
                  "warm D2H");
            check(hipStreamSynchronize(unit_stream(0)), "warm D2H");
        }
        impl((*hw_matrix)[0])->clique = c;
    }
    // empty_rows_bitmap[block][row] (csr_hw.cpp:391-393, :340-347): inner rows live inside the
    // outer allocation, so the caller's free(outer) (main.cpp:95) releases all of it.
    const int blocks = 1;
    bool **bm = (bool **)std::malloc(blocks * sizeof(bool *) + size_t(blocks) * n * sizeof(bool) + 1);
    bool *rows = reinterpret_cast<bool *>(bm + blocks);
    for (IndexType r = 0; r < n; ++r)
        rows[r] = matrix->row_ptr[r + 1] == matrix->row_ptr[r];
    bm[0] = rows;
    *empty_rows_bitmap = bm;

    // csr_hw.cpp:420-421
    const double mb = 8.0 * 1024 * 1024;
    const double in_mb = in_bytes * 8.0 / mb, out_mb = double(n) * VALUE_TYPE_BIT_WIDTH / mb;
    std::cout << "Total non-zeros : " << nnz_total << ". Total " << in_mb + out_mb
              << " MB transferred ( in : " << in_mb << ", out : " << out_mb << ")\n";
}

// csr_hw_wrapper.cpp:82-185: one y vector per unit (its row slice), on that unit's device
void create_csr_hw_y_vector(csr_hw_matrix **hw_matrix, csr_hw_vector ***hw_vector)
{
    if (!hw_matrix || !hw_vector)
        die("create_csr_hw_y_vector: null argument");
    const int units = units_of(hw_matrix);
    *hw_vector = (csr_hw_vector **)std::calloc(std::max(units, kMaxReferenceUnits) + 1, sizeof(csr_hw_vector *));
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        auto *v = new hw_vector_impl();
        v->device = m->device;
        const IndexType rows = m->row_end - m->row_begin;
        ValueType *d = nullptr;
        check(hipSetDevice(v->device), "hipSetDevice");
        if (rows)
            check(hipMalloc((void **)&d, size_t(rows) * sizeof(ValueType)), "hipMalloc(y)");
        v->per_device.assign(1, d);
        v->vals[0] = reinterpret_cast<BusDataType *>(d);
        v->nr_values[0] = rows;
        v->pub.values = v->vals;
        v->pub.nr_values = v->nr_values;
        v->pub.blocks = 1;
        (*hw_vector)[u] = &v->pub;
    }
}

// csr_hw_wrapper.cpp:187-191 (+ write_csr_hw_vector, csr_hw.cpp:1470-1488): x is uploaded
// once to every device that hosts a unit.
void create_csr_hw_x_vector(csr_hw_vector **hw_x, csr_vector *x, int blocks, IndexType *nr_cols)
{
    if (!hw_x || !x || !nr_cols)
        die("create_csr_hw_x_vector: null argument");
    if (blocks != 1)
        die("create_csr_hw_x_vector: blocks must be hw_matrix[0]->blocks (1)");
    if (x->nr_values > nr_cols[0])
        die("create_csr_hw_x_vector: x is longer than the matrix has columns");
    const double tx = timestamp_us();
    const int units = std::max(g_units_max, spmv_hw_units());
    const int ndev = std::min(units, device_count());
    auto *v = new hw_vector_impl();
    v->per_device.assign(ndev, nullptr);
    const size_t cols = nr_cols[0];
    for (int d = 0; d < ndev; ++d) {
        check(hipSetDevice(d), "hipSetDevice");
        ValueType *p = nullptr;
        check(hipMalloc((void **)&p, std::max<size_t>(cols, 1) * sizeof(ValueType)), "hipMalloc(x)");
        check(hipMemset(p, 0, std::max<size_t>(cols, 1) * sizeof(ValueType)), "hipMemset(x)");
        if (x->nr_values && upload_staged(p, x->values, size_t(x->nr_values) * sizeof(ValueType), nullptr))
            die(std::string("create_csr_hw_x_vector: ") + spmv_hw_last_error());
        v->per_device[d] = p;
    }
    v->vals[0] = reinterpret_cast<BusDataType *>(v->per_device[0]);
    v->nr_values[0] = (IndexType)cols;
    v->pub.values = v->vals;
    v->pub.nr_values = v->nr_values;
    v->pub.blocks = 1;
    *hw_x = &v->pub;
    if (std::getenv("SPMV_HW_TRACE"))
        std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", "x upload", (timestamp_us() - tx) / 1000);
}

// csr_hw_wrapper.cpp:193-288
void spmv_hw(csr_hw_matrix **hw_matrix, csr_hw_vector *hw_x, csr_vector *y_fpga, bool **empty_rows_bitmap)
{
    (void)empty_rows_bitmap;  // the device representation carries its own row map
    if (!hw_matrix || !hw_x || !y_fpga)
        die("spmv_hw: null argument");
    const int units = units_of(hw_matrix);
    hw_vector_impl *x = impl(hw_x);
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        const IndexType rows = m->row_end - m->row_begin;
        if (m->row_end > y_fpga->nr_values)
            die("spmv_hw: y_fpga is shorter than the matrix has rows");
        if ((size_t)m->device >= x->per_device.size())
            die("spmv_hw: x vector was not uploaded to device " + std::to_string(m->device));
        if (rows && !m->d_y && !impl(hw_matrix[0])->clique)
            alloc_y_scratch(m);
    }

    const bool trace = std::getenv("SPMV_HW_TRACE") != nullptr;
    auto tr = [&](const char *what, double since) {
        if (trace)
            std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", what, (timestamp_us() - since) / 1000);
    };
    if (hw_clique *c = units ? impl(hw_matrix[0])->clique : nullptr) {
        // kernels on every GPU, then the slices meet on GPU 0 over xGMI (RCCL gather, or the
        // ncclReduce of full-length partials = accum_results' +=); "hardware" time covers both
        std::vector<const ValueType *> xs(units);
        for (int u = 0; u < units; ++u)
            xs[u] = x->per_device[c->devices[u]];
        const double hw_s = timestamp_us();
        if (mgpu_run_on(c->mg, c->mode == kMergeReduce ? 1 : 0, xs.data()))
            die(std::string("spmv_hw: ") + spmv_hw_last_error());
        const double hw_exec = (timestamp_us() - hw_s) / 1000.0;
        std::printf("Hardware execution time : %.6f ms elapsed\n", hw_exec);
        if (trace) {
            double cms = 0, ems = 0;
            spmv_mgpu_get_timing(c->mg, &cms, &ems);
            std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms (kernels %.3f, exchange %.3f, %d RCCL calls)\n",
                         "spmv_hw: RCCL merge", hw_exec, cms, ems, mgpu_rccl_calls(c->mg));
        }
        // one D2H copy of the whole y from GPU 0, then the host += (accum_results into y_fpga)
        const double ra_s = timestamp_us();
        check(hipSetDevice(c->devices[0]), "hipSetDevice");
        std::vector<add_part> parts;
        c->done.device = c->devices[0];
        if (c->rows)
            enqueue_d2h(y_fpga->values, c->h_full, mgpu_root_y(c->mg), c->rows, c->rows < (1u << 18) ? 1 : env_pieces(8),
                        unit_stream(0), c->done, parts);
        const double landed = accumulate(parts);
        if (trace)
            std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", "spmv_hw: D2H landed", (landed - ra_s) / 1000);
        tr("spmv_hw: D2H + host accumulation", ra_s);
        const double ra_exec = (timestamp_us() - ra_s) / 1000.0;
        std::printf("Result accumulation time : %.6f ms elapsed\n", ra_exec);
        std::printf("Total time  : %.6f ms elapsed\n", hw_exec + ra_exec);
        std::fflush(stdout);
        return;
    }
    bool streamed = units > 0 && stream_enabled();  // (read per call, like SPMV_HW_PIPELINE)
    for (int u = 0; u < units && streamed; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        streamed = m->row_end == m->row_begin || (m->h_flags && sweep_can_flag_panels(*m->plan));
    }
    if (streamed)
        return spmv_hw_streamed(hw_matrix, units, x, y_fpga, trace);
    // kernels of every unit (one stream per unit; units on different GPUs run concurrently)
    const double hw_s = timestamp_us();
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        if (m->row_end == m->row_begin)
            continue;
        if (spmv_plan_run(m->plan, x->per_device[m->device], m->d_y, unit_stream(u)))
            die(std::string("spmv_hw: ") + spmv_hw_last_error());
    }
    tr("spmv_hw: launches", hw_s);
    for (int u = 0; u < units; ++u) {
        check(hipSetDevice(impl(hw_matrix[u])->device), "hipSetDevice");
        check(hipStreamSynchronize(unit_stream(u)), "spmv kernels");
    }
    const double hw_exec = (timestamp_us() - hw_s) / 1000.0;
    std::printf("Hardware execution time : %.6f ms elapsed\n", hw_exec);

    // accum_results: every unit's slice comes back over its own PCIe link into pinned memory
    // (all copies in flight together, each cut into pieces); host threads map their part of
    // y_fpga while the DMA runs and add each piece in as soon as its copy has landed
    const double ra_s = timestamp_us();
    // pieces in landing order: piece j of every unit (their copies run in parallel), then j + 1
    std::vector<std::vector<add_part>> per_unit(units);
    for (int u = 0; u < units; ++u) {
        hw_matrix_impl *m = impl(hw_matrix[u]);
        const uint64_t rows = m->row_end - m->row_begin;
        if (!rows)
            continue;
        check(hipSetDevice(m->device), "hipSetDevice");
        m->done.device = m->device;
        enqueue_d2h(y_fpga->values + m->row_begin, m->h_stage, m->d_y, rows,
                    rows < (1u << 18) ? 1 : std::max(2, env_pieces(8) / units), unit_stream(u), m->done,
                    per_unit[u]);
    }
    std::vector<add_part> parts;
    for (size_t j = 0, more = 1; more; ++j) {
        more = 0;
        for (int u = 0; u < units; ++u)
            if (j < per_unit[u].size()) {
                parts.push_back(per_unit[u][j]);
                more = 1;
            }
    }
    tr("spmv_hw: D2H enqueue", ra_s);
    const double landed = accumulate(parts);
    if (trace)
        std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms\n", "spmv_hw: D2H landed", (landed - ra_s) / 1000);
    tr("spmv_hw: host accumulation", ra_s);
    const double ra_exec = (timestamp_us() - ra_s) / 1000.0;
    std::printf("Result accumulation time : %.6f ms elapsed\n", ra_exec);
    std::printf("Total time  : %.6f ms elapsed\n", hw_exec + ra_exec);
    std::fflush(stdout);
}

// csr_hw_wrapper.cpp:291-296
void delete_csr_hw_matrix(csr_hw_matrix **hw_matrix)
{
    if (!hw_matrix)
        return;
    const int units = units_of(hw_matrix);
    for (int u = 0; u < units; ++u) {
        if (!hw_matrix[u])
            continue;
        hw_matrix_impl *m = impl(hw_matrix[u]);
        delete m->clique;  // before the plans it borrows
        spmv_plan_destroy(m->plan);
        if (m->copy_stream || m->h_flags) {
            (void)hipSetDevice(m->device);
            if (m->copy_stream)
                (void)hipStreamDestroy(m->copy_stream);
            if (m->h_flags)
                (void)hipHostFree(m->h_flags);
            if (m->h_direct)
                (void)hipHostFree(m->h_direct);
        }
        if (m->d_y || m->h_stage) {
            (void)hipSetDevice(m->device);
            if (m->d_y)
                (void)hipFree(m->d_y);
            if (m->h_stage)
                (void)hipHostFree(m->h_stage);
        }

        delete m;
    }
    std::free(hw_matrix);
}

static void delete_vector(csr_hw_vector *v)
{
    if (!v)
        return;
    hw_vector_impl *h = impl(v);
    for (size_t d = 0; d < h->per_device.size(); ++d) {
        if (h->per_device[d]) {
            (void)hipSetDevice(h->per_device.size() == 1 ? h->device : (int)d);
            (void)hipFree(h->per_device[d]);
        }
    }
    delete h;
}

// csr_hw_wrapper.cpp:298-303
void delete_csr_hw_y_vector(csr_hw_vector **hw_vector)
{
    if (!hw_vector)
        return;
    const int units = units_of(hw_vector);
    for (int u = 0; u < units; ++u)
        delete_vector(hw_vector[u]);
    std::free(hw_vector);
}

// csr_hw_wrapper.cpp:305-308
void delete_csr_hw_x_vector(csr_hw_vector *hw_vector) { delete_vector(hw_vector); }

}  // extern "C"
