// Part 4 of the C-ABI: one host process driving several MI355X with an RCCL exchange over xGMI
// (SURVEY.md §5 "one process driving 8 GPUs (ncclCommInitAll)", §8(e)).
//
// The reference splits every column block's rows into nnz-balanced slices, one per Compute Unit
// (prepare_balanced_hw_matrix, csr_hw.cpp:459-468), copies x into every CU (spmv.cpp:280-294),
// and the host merges the CUs' compact y slices (accum_results, csr_hw.cpp:1531-1565, looped in
// csr_hw_wrapper.cpp:276-281). Here a unit is a GPU: each device holds a plan for its row slice
// (spmv_plan_create_host) and a replicated x; the slices are exchanged on the devices with RCCL
// instead of over PCIe through the host:
//   SPMV_MGPU_GATHER    ncclSend/ncclRecv of the disjoint slices into the root's y (each GPU
//                       sends its (r1-r0) rows over its own xGMI link: bandwidth-optimal)
//   SPMV_MGPU_REDUCE    ncclReduce(sum) of full-length zero-filled partials into the root: the
//                       literal `+=` of accum_results
//   SPMV_MGPU_ALLGATHER every device broadcasts its slice into every device's next x (grouped
//                       ncclBroadcast = all-gather with unequal counts); the next run computes
//                       A * y (iterative solvers)
// Two ways to form the communicator: one process driving every GPU (spmv_mgpu_create,
// ncclCommInitAll), or one process per GPU (spmv_mgpu_create_rank, ncclCommInitRank with an id
// made by spmv_mgpu_unique_id on rank 0 and shared by the caller), which is how bench.py's ranks
// exchange y natively. The exchange code is the same: it loops over the devices this process
// drives, each with its rank in the clique.
// RCCL is loaded at run time (dlopen), so the library itself does not depend on it; a process
// that already loaded RCCL (e.g. PyTorch's) shares that copy.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "spmv_internal.hpp"

using namespace spmvhw;

namespace {

struct Rccl {
    void *h = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclBroadcast) Broadcast = nullptr;
    decltype(&ncclReduce) Reduce = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclCommCount) CommCount = nullptr;
};

// first RCCL already in the process, else the ROCm one
const Rccl *rccl()
{
    static Rccl r;
    static bool tried = false;
    if (tried)
        return r.h ? &r : nullptr;
    tried = true;
    for (const char *name : {"librccl.so.1", "librccl.so"}) {
        r.h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        if (r.h)
            break;
    }
    for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
        if (r.h)
            break;
        r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    }
    if (!r.h)
        return nullptr;
#define SYM(f) r.f = reinterpret_cast<decltype(r.f)>(dlsym(r.h, "nccl" #f))
    SYM(CommInitAll);
    SYM(CommInitRank);
    SYM(GetUniqueId);
    SYM(CommDestroy);
    SYM(GetErrorString);
    SYM(GroupStart);
    SYM(GroupEnd);
    SYM(Broadcast);
    SYM(Reduce);
    SYM(Send);
    SYM(Recv);
    SYM(CommCount);
#undef SYM
    if (!r.CommInitAll || !r.CommInitRank || !r.GetUniqueId || !r.CommDestroy || !r.GetErrorString || !r.GroupStart || !r.GroupEnd || !r.Broadcast ||
        !r.Reduce || !r.Send || !r.Recv || !r.CommCount) {
        r.h = nullptr;
        return nullptr;
    }
    return &r;
}

constexpr ncclDataType_t kNcclValue = sizeof(ValueType) == 8 ? ncclFloat64 : ncclFloat32;

}  // namespace

struct spmv_mgpu {
    const Rccl *nc = nullptr;
    int nloc = 0;                       // devices driven by this process
    int nranks = 0;                     // ranks of the clique (= slices)
    IndexType nr_rows = 0, nr_cols = 0;
    bool owns_plans = true;
    bool own_x = true;                  // false: every run takes the caller's x per device
    std::vector<int> dev, rank;         // per local device: HIP device and rank
    std::vector<IndexType> bounds;      // row slice of rank r: [bounds[r], bounds[r+1])
    std::vector<const spmv_plan *> plan;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<ValueType *> x, xnext;  // full-length x on every device; next x (all-gather)
    std::vector<ValueType *> yslice;    // rank > 0: its rows (rank 0 computes into y)
    std::vector<ValueType *> ypart;     // reduce mode: full-length partials, zero outside the slice
    std::vector<ValueType *> y;         // rank 0 only: the full y
    std::vector<hipEvent_t> ev;         // per device: start, kernels done, exchange done
    double compute_ms = 0, exchange_ms = 0;
    int rccl_calls = 0;                 // RCCL calls per step of the last run, all local devices
                                        // (the schedule's exchange ops; run, _pipelined and _graph)
    // spmv_mgpu_run_pipelined: per device a second stream for the exchange, a second y buffer
    // (and reduce partial), and the events that hand each buffer between the two streams
    struct Pipe {
        hipStream_t cs = nullptr;
        ValueType *buf2 = nullptr;   // second y: the root's full y / a rank's slice / reduce output
        ValueType *part2 = nullptr;  // reduce: second full-length partial
        hipEvent_t comp[2] = {nullptr, nullptr}, exch[2] = {nullptr, nullptr}, t0 = nullptr, t1 = nullptr;
    };
    std::vector<Pipe> pipe;
    // spmv_mgpu_run_graph (one device per handle): `g_iters` steps of kernels + exchange captured
    // into one hipGraph, re-captured when the exchange, the step count or the x buffer changes
    hipGraphExec_t gexec = nullptr;
    int g_exchange = -1, g_iters = 0;
    const ValueType *g_x = nullptr;

    void init(int n)
    {
        nloc = n;
        dev.assign(n, 0);
        rank.assign(n, 0);
        plan.assign(n, nullptr);
        comm.assign(n, nullptr);
        stream.assign(n, nullptr);
        x.assign(n, nullptr);
        xnext.assign(n, nullptr);
        yslice.assign(n, nullptr);
        ypart.assign(n, nullptr);
        y.assign(n, nullptr);
        ev.assign(3 * n, nullptr);
    }
    ~spmv_mgpu()
    {
        for (int d = 0; d < nloc; ++d) {
            (void)hipSetDevice(dev[d]);
            if (owns_plans && plan[d])
                spmv_plan_destroy(const_cast<spmv_plan *>(plan[d]));
            for (void *p : {(void *)x[d], (void *)xnext[d], (void *)yslice[d], (void *)ypart[d], (void *)y[d]})
                if (p)
                    (void)hipFree(p);
            if (comm[d] && nc)
                nc->CommDestroy(comm[d]);
            if (stream[d])
                (void)hipStreamDestroy(stream[d]);
            for (int k = 0; k < 3; ++k)
                if (ev[3 * d + k])
                    (void)hipEventDestroy(ev[3 * d + k]);
            if (d == 0 && gexec)
                (void)hipGraphExecDestroy(gexec);
            if (d < (int)pipe.size()) {
                Pipe &q = pipe[d];
                for (void *p : {(void *)q.buf2, (void *)q.part2})
                    if (p)
                        (void)hipFree(p);
                for (hipEvent_t e : {q.comp[0], q.comp[1], q.exch[0], q.exch[1], q.t0, q.t1})
                    if (e)
                        (void)hipEventDestroy(e);
                if (q.cs)
                    (void)hipStreamDestroy(q.cs);
            }
        }
    }
    IndexType rows_of(int r) const { return bounds[r + 1] - bounds[r]; }
    IndexType rows(int d) const { return rows_of(rank[d]); }
    // buffers every local device needs (stream, events, x, its y slice or the root's y)
    int alloc_device(int d)
    {
        SPMV_TRY(hipSetDevice(dev[d]));
        SPMV_TRY(hipStreamCreateWithFlags(&stream[d], hipStreamNonBlocking));
        for (int k = 0; k < 3; ++k)
            SPMV_TRY(hipEventCreate(&ev[3 * d + k]));
        const size_t xb = std::max<size_t>(nr_cols, 1) * sizeof(ValueType);
        if (own_x) {
            SPMV_TRY(hipMalloc((void **)&x[d], xb));
            SPMV_TRY(hipMemset(x[d], 0, xb));
        }
        if (rank[d] == 0)
            SPMV_TRY(hipMalloc((void **)&y[d], std::max<size_t>(nr_rows, 1) * sizeof(ValueType)));
        else
            SPMV_TRY(hipMalloc((void **)&yslice[d], std::max<size_t>(rows(d), 1) * sizeof(ValueType)));
        return 0;
    }
    int root_local() const  // local index of rank 0, or -1
    {
        for (int d = 0; d < nloc; ++d)
            if (rank[d] == 0)
                return d;
        return -1;
    }
};

#define MG_NCCL(expr)                                                                          \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess) {                                                               \
            set_error(std::string(#expr) + ": " + mg->nc->GetErrorString(r_));               \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

// The buffers a schedule (spmv_mgpu_schedule, host.cpp) names, resolved for one device (and one
// slot of the pipelined double buffer)
struct XBufs {
    ValueType *y, *slice, *part, *xnext;
    ValueType *at(int buf) const
    {
        return buf == SPMV_XBUF_Y ? y : buf == SPMV_XBUF_SLICE ? slice : buf == SPMV_XBUF_PART ? part : xnext;
    }
};

// the schedule of local device d's rank for one step (1: the handle's bounds were refused)
static int schedule_of(const spmv_mgpu *mg, int d, int exchange, std::vector<spmv_xop> &ops)
{
    ops.resize(2 + 2 * size_t(mg->nranks));
    const int n = spmv_mgpu_schedule(exchange, mg->rank[d], mg->nranks, mg->bounds.data(), ops.data(), (int)ops.size());
    if (n < 0 || size_t(n) > ops.size()) {
        set_error("spmv_mgpu: no exchange schedule for this handle's slices");
        return 1;
    }
    ops.resize(n);
    return 0;
}

static int exchange_ops(const std::vector<spmv_xop> &ops)
{
    int n = 0;
    for (const spmv_xop &o : ops)
        n += o.kind >= SPMV_XOP_SEND;
    return n;
}

static bool has_exchange(const std::vector<spmv_xop> &ops) { return exchange_ops(ops) > 0; }

// the local ops (ZERO, COMPUTE) of device d on its compute stream s
static int issue_local(spmv_mgpu *mg, int d, const std::vector<spmv_xop> &ops, const XBufs &b, const ValueType *x,
                       hipStream_t s)
{
    for (const spmv_xop &o : ops) {
        if (o.kind == SPMV_XOP_ZERO)
            SPMV_TRY(hipMemsetAsync(b.at(o.buf) + o.offset, 0, size_t(o.count) * sizeof(ValueType), s));
        else if (o.kind == SPMV_XOP_COMPUTE && spmv_plan_run(mg->plan[d], x, b.at(o.buf) + o.offset, s))
            return 1;
    }
    return 0;
}

// the exchange ops of device d on stream s; the caller brackets every local device's calls with
// one ncclGroupStart / ncclGroupEnd
static int issue_exchange(spmv_mgpu *mg, int d, const std::vector<spmv_xop> &ops, const XBufs &b, hipStream_t s)
{
    for (const spmv_xop &o : ops) {
        ValueType *p = b.at(o.buf) + o.offset;
        switch (o.kind) {
        case SPMV_XOP_SEND:
            MG_NCCL(mg->nc->Send(p, o.count, kNcclValue, o.peer, mg->comm[d], s));
            break;
        case SPMV_XOP_RECV:
            MG_NCCL(mg->nc->Recv(p, o.count, kNcclValue, o.peer, mg->comm[d], s));
            break;
        case SPMV_XOP_REDUCE:
            MG_NCCL(mg->nc->Reduce(p, o.out >= 0 ? b.at(o.out) + o.offset : nullptr, o.count, kNcclValue, ncclSum, o.peer,
                                   mg->comm[d], s));
            break;
        case SPMV_XOP_BCAST:
            MG_NCCL(mg->nc->Broadcast(p, p, o.count, kNcclValue, o.peer, mg->comm[d], s));
            break;
        default:
            break;
        }
    }
    return 0;
}

extern "C" {

int spmv_mgpu_create(spmv_mgpu **out, int ndev, const int *devices, const csr_matrix *m)
{
    if (!out || ndev < 1 || !m) {
        set_error("spmv_mgpu_create: bad arguments");
        return 1;
    }
    *out = nullptr;
    int count = 0;
    SPMV_TRY(hipGetDeviceCount(&count));
    std::vector<int> dl(ndev);
    for (int d = 0; d < ndev; ++d) {
        dl[d] = devices ? devices[d] : d;
        if (dl[d] < 0 || dl[d] >= count) {
            set_error("spmv_mgpu_create: device " + std::to_string(dl[d]) + " does not exist");
            return 1;
        }
        for (int e = 0; e < d; ++e)
            if (dl[e] == dl[d]) {
                set_error("spmv_mgpu_create: a device appears twice (one RCCL rank per GPU)");
                return 1;
            }
    }
    const Rccl *nc = rccl();
    if (!nc) {
        set_error("spmv_mgpu_create: RCCL (librccl.so.1) could not be loaded");
        return 1;
    }
    std::unique_ptr<spmv_mgpu> mg(new spmv_mgpu());
    mg->nc = nc;
    mg->init(ndev);
    mg->nranks = ndev;
    mg->nr_rows = m->nr_rows;
    mg->nr_cols = m->nr_cols;
    mg->bounds.assign(ndev + 1, 0);
    if (spmv_partition_rows(m->row_ptr, m->nr_rows, ndev, mg->bounds.data()))
        return 1;
    for (int d = 0; d < ndev; ++d) {
        mg->dev[d] = dl[d];
        mg->rank[d] = d;
        spmv_plan *pl = nullptr;
        if (spmv_plan_create_host(&pl, dl[d], m, mg->bounds[d], mg->bounds[d + 1]))
            return 1;
        mg->plan[d] = pl;
        if (mg->alloc_device(d))
            return 1;
    }
    {
        ncclResult_t r = nc->CommInitAll(mg->comm.data(), ndev, dl.data());
        if (r != ncclSuccess) {
            mg->comm.assign(ndev, nullptr);
            set_error(std::string("spmv_mgpu_create: ncclCommInitAll: ") + nc->GetErrorString(r));
            return 1;
        }
    }
    *out = mg.release();
    return 0;
}

int spmv_mgpu_unique_id(unsigned char *id)
{
    if (!id) {
        set_error("spmv_mgpu_unique_id: null argument");
        return 1;
    }
    const Rccl *nc = rccl();
    if (!nc) {
        set_error("spmv_mgpu_unique_id: RCCL (librccl.so.1) could not be loaded");
        return 1;
    }
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    const ncclResult_t r = nc->GetUniqueId(&u);
    if (r != ncclSuccess) {
        set_error(std::string("spmv_mgpu_unique_id: ") + nc->GetErrorString(r));
        return 1;
    }
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

int spmv_mgpu_create_rank(spmv_mgpu **out, int rank, int nranks, const unsigned char *id, int device,
                          const IndexType *bounds, IndexType nr_cols, const spmv_plan *plan)
{
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || !id || !bounds || !plan) {
        set_error("spmv_mgpu_create_rank: bad arguments");
        return 1;
    }
    *out = nullptr;
    for (int r = 0; r < nranks; ++r)
        if (bounds[r + 1] < bounds[r] || bounds[0] != 0) {
            set_error("spmv_mgpu_create_rank: bounds must start at 0 and be non-decreasing");
            return 1;
        }
    if (plan->nr_rows != bounds[rank + 1] - bounds[rank] || plan->nr_cols != nr_cols || plan->device != device) {
        set_error("spmv_mgpu_create_rank: the plan is not this rank's slice on `device`");
        return 1;
    }
    const Rccl *nc = rccl();
    if (!nc) {
        set_error("spmv_mgpu_create_rank: RCCL (librccl.so.1) could not be loaded");
        return 1;
    }
    std::unique_ptr<spmv_mgpu> mg(new spmv_mgpu());
    mg->nc = nc;
    mg->init(1);
    mg->owns_plans = false;
    mg->nranks = nranks;
    mg->bounds.assign(bounds, bounds + nranks + 1);
    mg->nr_rows = bounds[nranks];
    mg->nr_cols = nr_cols;
    mg->dev[0] = device;
    mg->rank[0] = rank;
    mg->plan[0] = plan;
    // join the clique first: a rank that failed before ncclCommInitRank would leave the others
    // waiting in it; failures after it are reported to the caller, who agrees with the other
    // ranks before the first collective
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    SPMV_TRY(hipSetDevice(device));
    const ncclResult_t r = nc->CommInitRank(&mg->comm[0], nranks, u, rank);
    if (r != ncclSuccess) {
        mg->comm[0] = nullptr;
        set_error(std::string("spmv_mgpu_create_rank: ncclCommInitRank: ") + nc->GetErrorString(r));
        return 1;
    }
    if (mg->alloc_device(0))
        return 1;
    *out = mg.release();
    return 0;
}

// RCCL broadcast of rank 0's x to every device's x, then wait
static int broadcast_x(spmv_mgpu *mg)
{
    if (mg->nranks == 1 || mg->nr_cols == 0)
        return 0;
    MG_NCCL(mg->nc->GroupStart());
    for (int d = 0; d < mg->nloc; ++d)
        MG_NCCL(mg->nc->Broadcast(mg->x[d], mg->x[d], mg->nr_cols, kNcclValue, 0, mg->comm[d], mg->stream[d]));
    MG_NCCL(mg->nc->GroupEnd());
    for (int d = 0; d < mg->nloc; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipStreamSynchronize(mg->stream[d]));
    }
    return 0;
}

// x (nr_cols values, host) -> rank 0's device, then one RCCL broadcast to every device. In the
// one-process-per-GPU form every rank calls it (h_x is read on rank 0 only).
int spmv_mgpu_set_x(spmv_mgpu *mg, const ValueType *h_x)
{
    if (!mg) {
        set_error("spmv_mgpu_set_x: bad arguments");
        return 1;
    }
    const int r0 = mg->root_local();
    if (r0 >= 0) {
        if (!h_x) {
            set_error("spmv_mgpu_set_x: rank 0 needs x");
            return 1;
        }
        SPMV_TRY(hipSetDevice(mg->dev[r0]));
        if (mg->nr_cols && upload_staged(mg->x[r0], h_x, size_t(mg->nr_cols) * sizeof(ValueType), mg->stream[r0]))
            return 1;
    }
    return broadcast_x(mg);
}

// the same from a device-resident x on rank 0's device. The handle's streams are non-blocking,
// so nothing would order the copy after the work that produced d_x: spmv_mgpu_set_x_device waits
// for everything this process queued on rank 0's device (hipDeviceSynchronize), the _on form only
// for the producer's `stream` (an event, no host wait; NULL = the legacy default stream).
static int set_x_device_impl(spmv_mgpu *mg, const ValueType *d_x, bool whole_device, hipStream_t producer)
{
    const int r0 = mg->root_local();
    if (r0 >= 0) {
        if (!d_x) {
            set_error("spmv_mgpu_set_x_device: rank 0 needs x");
            return 1;
        }
        SPMV_TRY(hipSetDevice(mg->dev[r0]));
        if (whole_device) {
            SPMV_TRY(hipDeviceSynchronize());
        } else {
            hipEvent_t e;
            SPMV_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            hipError_t rc = hipEventRecord(e, producer);
            if (rc == hipSuccess)
                rc = hipStreamWaitEvent(mg->stream[r0], e, 0);
            (void)hipEventDestroy(e);  // released once the wait has been satisfied
            SPMV_TRY(rc);
        }
        if (mg->nr_cols)
            SPMV_TRY(hipMemcpyAsync(mg->x[r0], d_x, size_t(mg->nr_cols) * sizeof(ValueType), hipMemcpyDeviceToDevice,
                                    mg->stream[r0]));
    }
    return broadcast_x(mg);
}

int spmv_mgpu_set_x_device(spmv_mgpu *mg, const ValueType *d_x)
{
    if (!mg) {
        set_error("spmv_mgpu_set_x_device: bad arguments");
        return 1;
    }
    return set_x_device_impl(mg, d_x, true, nullptr);
}

int spmv_mgpu_set_x_device_on(spmv_mgpu *mg, const ValueType *d_x, void *stream)
{
    if (!mg) {
        set_error("spmv_mgpu_set_x_device_on: bad arguments");
        return 1;
    }
    return set_x_device_impl(mg, d_x, false, (hipStream_t)stream);
}

}  // extern "C"

namespace spmvhw {

int mgpu_create_borrowed(spmv_mgpu **out, int n, const int *devices, const IndexType *bounds, IndexType nr_cols,
                         const spmv_plan *const *plans)
{
    *out = nullptr;
    const Rccl *nc = rccl();
    if (!nc) {
        set_error("RCCL (librccl.so.1) could not be loaded");
        return 1;
    }
    std::unique_ptr<spmv_mgpu> mg(new spmv_mgpu());
    mg->nc = nc;
    mg->init(n);
    mg->owns_plans = false;
    mg->own_x = false;
    mg->nranks = n;
    mg->bounds.assign(bounds, bounds + n + 1);
    mg->nr_rows = bounds[n];
    mg->nr_cols = nr_cols;
    for (int d = 0; d < n; ++d) {
        for (int e = 0; e < d; ++e)
            if (devices[e] == devices[d]) {
                set_error("a device appears twice (one RCCL rank per GPU)");
                return 1;
            }
        mg->dev[d] = devices[d];
        mg->rank[d] = d;
        mg->plan[d] = plans[d];
        if (mg->alloc_device(d))
            return 1;
    }
    const ncclResult_t r = nc->CommInitAll(mg->comm.data(), n, devices);
    if (r != ncclSuccess) {
        mg->comm.assign(n, nullptr);
        set_error(std::string("ncclCommInitAll: ") + nc->GetErrorString(r));
        return 1;
    }
    *out = mg.release();
    return 0;
}

int mgpu_rccl_calls(const spmv_mgpu *mg) { return mg->rccl_calls; }

const ValueType *mgpu_root_y(const spmv_mgpu *mg)
{
    const int r0 = mg->root_local();
    return r0 < 0 ? nullptr : mg->y[r0];
}

// the SpMV on every local device with x_dev[d] (NULL: the handle's own x), then the exchange
int mgpu_run_on(spmv_mgpu *mg, int exchange, const ValueType *const *x_dev)
{
    if (exchange < 0 || exchange > 2 || (!x_dev && !mg->own_x) || (exchange == 2 && !mg->own_x)) {
        set_error("spmv_mgpu_run: bad arguments");
        return 1;
    }
    if (exchange == 2 && mg->nr_rows != mg->nr_cols) {
        set_error("spmv_mgpu_run: the all-gather exchange makes y the next x (needs a square matrix)");
        return 1;
    }
    const int nl = mg->nloc;
    const size_t nb = size_t(mg->nr_rows) * sizeof(ValueType);
    // buffers of the exchange form, allocated on first use
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        if (exchange == 1 && !mg->ypart[d])
            SPMV_TRY(hipMalloc((void **)&mg->ypart[d], std::max<size_t>(nb, sizeof(ValueType))));
        if (exchange == 2 && !mg->xnext[d])
            SPMV_TRY(hipMalloc((void **)&mg->xnext[d], std::max<size_t>(nb, sizeof(ValueType))));
    }
    std::vector<std::vector<spmv_xop>> sch(nl);
    bool any = false;
    for (int d = 0; d < nl; ++d) {
        if (schedule_of(mg, d, exchange, sch[d]))
            return 1;
        any = any || has_exchange(sch[d]);
    }
    auto bufs = [&](int d) { return XBufs{mg->y[d], mg->yslice[d], mg->ypart[d], mg->xnext[d]}; };
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        hipStream_t s = mg->stream[d];
        SPMV_TRY(hipEventRecord(mg->ev[3 * d], s));
        if (issue_local(mg, d, sch[d], bufs(d), x_dev ? x_dev[d] : mg->x[d], s))
            return 1;
        SPMV_TRY(hipEventRecord(mg->ev[3 * d + 1], s));
    }
    mg->rccl_calls = 0;
    for (int d = 0; d < nl; ++d)
        mg->rccl_calls += exchange_ops(sch[d]);
    if (any) {
        MG_NCCL(mg->nc->GroupStart());
        for (int d = 0; d < nl; ++d)
            if (issue_exchange(mg, d, sch[d], bufs(d), mg->stream[d]))
                return 1;
        MG_NCCL(mg->nc->GroupEnd());
    }
    double cmax = 0, tmax = 0;
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipEventRecord(mg->ev[3 * d + 2], mg->stream[d]));
    }
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipEventSynchronize(mg->ev[3 * d + 2]));
        float c = 0, t = 0;
        SPMV_TRY(hipEventElapsedTime(&c, mg->ev[3 * d], mg->ev[3 * d + 1]));
        SPMV_TRY(hipEventElapsedTime(&t, mg->ev[3 * d], mg->ev[3 * d + 2]));
        cmax = std::max(cmax, (double)c);
        tmax = std::max(tmax, (double)t);
    }
    mg->compute_ms = cmax;
    mg->exchange_ms = std::max(0.0, tmax - cmax);
    if (exchange == 2)
        for (int d = 0; d < nl; ++d)
            std::swap(mg->x[d], mg->xnext[d]);  // y becomes the next x on every device
    return 0;
}

}  // namespace spmvhw

extern "C" {

int spmv_mgpu_run(spmv_mgpu *mg, int exchange)
{
    if (!mg || exchange < 0 || exchange > 2 || !mg->own_x) {
        set_error("spmv_mgpu_run: bad arguments");
        return 1;
    }
    return mgpu_run_on(mg, exchange, nullptr);
}

// `steps` SpMVs of the handle's x with the exchange of step k overlapping the kernels of step
// k + 1: the kernels run on each device's stream into one of two y buffers,
// the exchange (gather or reduce) on a second stream after an event, and a buffer is reused only
// once its exchange completed. One SpMV's own exchange cannot overlap its kernels: a slice of the
// strong-scaling matrix runs as one round of workgroups whose rows all finish at the end
// (DESIGN.md §6). Afterwards rank 0's y holds the last step's result (spmv_mgpu_get_y /
// spmv_mgpu_y_device with the same exchange). *ms_per_step: first kernel to last exchange, max
// over this process's devices, / steps.
int spmv_mgpu_run_pipelined(spmv_mgpu *mg, int exchange, int steps, double *ms_per_step)
{
    if (!mg || !mg->own_x || steps < 1 || (exchange != SPMV_MGPU_GATHER && exchange != SPMV_MGPU_REDUCE)) {
        set_error("spmv_mgpu_run_pipelined: bad arguments (gather or reduce, steps >= 1)");
        return 1;
    }
    const int nl = mg->nloc;
    const bool red = exchange == SPMV_MGPU_REDUCE;
    const size_t nb = size_t(mg->nr_rows) * sizeof(ValueType);
    if (mg->pipe.empty())
        mg->pipe.resize(nl);
    for (int d = 0; d < nl; ++d) {  // resources on first use
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        spmv_mgpu::Pipe &q = mg->pipe[d];
        if (!q.cs) {
            SPMV_TRY(hipStreamCreateWithFlags(&q.cs, hipStreamNonBlocking));
            for (int b = 0; b < 2; ++b) {
                SPMV_TRY(hipEventCreateWithFlags(&q.comp[b], hipEventDisableTiming));
                SPMV_TRY(hipEventCreateWithFlags(&q.exch[b], hipEventDisableTiming));
            }
            SPMV_TRY(hipEventCreate(&q.t0));
            SPMV_TRY(hipEventCreate(&q.t1));
        }
        const size_t yb = mg->rank[d] == 0 ? nb : size_t(mg->rows(d)) * sizeof(ValueType);
        if (!q.buf2)
            SPMV_TRY(hipMalloc((void **)&q.buf2, std::max<size_t>(std::max(yb, nb), sizeof(ValueType))));
        if (red && !mg->ypart[d])
            SPMV_TRY(hipMalloc((void **)&mg->ypart[d], std::max<size_t>(nb, sizeof(ValueType))));
        if (red && !q.part2)
            SPMV_TRY(hipMalloc((void **)&q.part2, std::max<size_t>(nb, sizeof(ValueType))));
    }
    // buffer set b of device d: the handle's own buffers (b = 0) or the pipeline's second ones
    auto bufs = [&](int d, int b) {
        spmv_mgpu::Pipe &q = mg->pipe[d];
        return b == 0 ? XBufs{mg->y[d], mg->yslice[d], mg->ypart[d], nullptr} : XBufs{q.buf2, q.buf2, q.part2, nullptr};
    };
    std::vector<std::vector<spmv_xop>> sch(nl);
    bool any = false;
    for (int d = 0; d < nl; ++d) {
        if (schedule_of(mg, d, exchange, sch[d]))
            return 1;
        any = any || has_exchange(sch[d]);
    }
    mg->rccl_calls = 0;
    for (int d = 0; d < nl; ++d)
        mg->rccl_calls += exchange_ops(sch[d]);
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipEventRecord(mg->pipe[d].t0, mg->stream[d]));
    }
    for (int k = 0; k < steps; ++k) {
        const int b = k & 1;
        for (int d = 0; d < nl; ++d) {
            SPMV_TRY(hipSetDevice(mg->dev[d]));
            spmv_mgpu::Pipe &q = mg->pipe[d];
            hipStream_t s = mg->stream[d];
            if (k >= 2)  // buffer b is free once the exchange of step k - 2 completed
                SPMV_TRY(hipStreamWaitEvent(s, q.exch[b], 0));
            if (issue_local(mg, d, sch[d], bufs(d, b), mg->x[d], s))
                return 1;
            SPMV_TRY(hipEventRecord(q.comp[b], s));
            SPMV_TRY(hipStreamWaitEvent(q.cs, q.comp[b], 0));
        }
        if (any) {
            MG_NCCL(mg->nc->GroupStart());
            for (int d = 0; d < nl; ++d)
                if (issue_exchange(mg, d, sch[d], bufs(d, b), mg->pipe[d].cs))
                    return 1;
            MG_NCCL(mg->nc->GroupEnd());
        }
        for (int d = 0; d < nl; ++d) {
            SPMV_TRY(hipSetDevice(mg->dev[d]));
            SPMV_TRY(hipEventRecord(mg->pipe[d].exch[b], mg->pipe[d].cs));
        }
    }
    double tmax = 0;
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        spmv_mgpu::Pipe &q = mg->pipe[d];
        SPMV_TRY(hipStreamWaitEvent(q.cs, mg->pipe[d].comp[(steps - 1) & 1], 0));
        SPMV_TRY(hipEventRecord(q.t1, q.cs));
    }
    for (int d = 0; d < nl; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipEventSynchronize(mg->pipe[d].t1));
        float t = 0;
        SPMV_TRY(hipEventElapsedTime(&t, mg->pipe[d].t0, mg->pipe[d].t1));
        tmax = std::max(tmax, (double)t);
        SPMV_TRY(hipStreamSynchronize(mg->stream[d]));
    }
    // the last result sits in the second buffers: copy it into rank 0's y, so y keeps its address
    // (pointers from spmv_mgpu_y_device and graphs captured by spmv_mgpu_run_graph stay valid)
    if ((steps - 1) & 1)
        for (int d = 0; d < nl; ++d)
            if (mg->rank[d] == 0 && mg->nr_rows) {
                SPMV_TRY(hipSetDevice(mg->dev[d]));
                SPMV_TRY(hipMemcpyAsync(mg->y[d], mg->pipe[d].buf2, nb, hipMemcpyDeviceToDevice, mg->stream[d]));
                SPMV_TRY(hipStreamSynchronize(mg->stream[d]));
            }
    if (ms_per_step)
        *ms_per_step = tmax / steps;
    return 0;
}

// one step of a one-device handle on stream s: the kernels on x_in, then the exchange; the
// all-gather writes every slice of the next x into x_out (capturable: kernels, a memset and
// RCCL calls only)
static int enqueue_step(spmv_mgpu *mg, int exchange, const ValueType *x_in, ValueType *x_out, hipStream_t s)
{
    std::vector<spmv_xop> ops;
    if (schedule_of(mg, 0, exchange, ops))
        return 1;
    const XBufs b{mg->y[0], mg->yslice[0], mg->ypart[0], x_out};
    if (issue_local(mg, 0, ops, b, x_in, s))
        return 1;
    if (has_exchange(ops)) {
        MG_NCCL(mg->nc->GroupStart());
        if (issue_exchange(mg, 0, ops, b, s))
            return 1;
        MG_NCCL(mg->nc->GroupEnd());
    }
    return 0;
}

// `iters` steps (SpMV + exchange) replayed from one hipGraph, for a handle that drives one
// device (one process per GPU, or a one-device clique): no host launch between the kernels and
// the RCCL exchange or between steps. The all-gather form iterates x <- A x (the iterative use
// of SURVEY §8f rank 3) and leaves A^iters x as this handle's x; gather / reduce repeat y = A x.
// *ms_per_step: the graph's duration / iters (HIP events on the handle's stream).
int spmv_mgpu_run_graph(spmv_mgpu *mg, int exchange, int iters, double *ms_per_step)
{
    if (!mg || !mg->own_x || iters < 1 || exchange < 0 || exchange > 2) {
        set_error("spmv_mgpu_run_graph: bad arguments");
        return 1;
    }
    if (mg->nloc != 1) {
        set_error("spmv_mgpu_run_graph: graph capture needs a handle that drives one device");
        return 1;
    }
    if (exchange == 2 && mg->nr_rows != mg->nr_cols) {
        set_error("spmv_mgpu_run_graph: the all-gather exchange makes y the next x (needs a square matrix)");
        return 1;
    }
    const size_t nb = std::max<size_t>(size_t(mg->nr_rows) * sizeof(ValueType), sizeof(ValueType));
    SPMV_TRY(hipSetDevice(mg->dev[0]));
    if (exchange == 1 && !mg->ypart[0])
        SPMV_TRY(hipMalloc((void **)&mg->ypart[0], nb));
    if (exchange == 2 && !mg->xnext[0])
        SPMV_TRY(hipMalloc((void **)&mg->xnext[0], nb));
    hipStream_t s = mg->stream[0];
    {
        std::vector<spmv_xop> ops;
        if (schedule_of(mg, 0, exchange, ops))
            return 1;
        mg->rccl_calls = exchange_ops(ops);  // per step; the graph replays them every step
    }
    if (!mg->gexec || mg->g_exchange != exchange || mg->g_iters != iters || mg->g_x != mg->x[0]) {
        if (mg->gexec) {
            SPMV_TRY(hipGraphExecDestroy(mg->gexec));
            mg->gexec = nullptr;
        }
        SPMV_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        int rc = 0;
        for (int i = 0; i < iters && !rc; ++i) {
            const bool odd = exchange == 2 && (i & 1);
            rc = enqueue_step(mg, exchange, odd ? mg->xnext[0] : mg->x[0], odd ? mg->x[0] : mg->xnext[0], s);
        }
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(s, &g);
        if (rc) {
            if (g)
                (void)hipGraphDestroy(g);
            return rc;
        }
        SPMV_TRY(ec);
        const hipError_t ei = hipGraphInstantiate(&mg->gexec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        SPMV_TRY(ei);
        mg->g_exchange = exchange;
        mg->g_iters = iters;
        mg->g_x = mg->x[0];
    }
    SPMV_TRY(hipEventRecord(mg->ev[0], s));
    SPMV_TRY(hipGraphLaunch(mg->gexec, s));
    SPMV_TRY(hipEventRecord(mg->ev[2], s));
    SPMV_TRY(hipEventSynchronize(mg->ev[2]));
    float t = 0;
    SPMV_TRY(hipEventElapsedTime(&t, mg->ev[0], mg->ev[2]));
    if (ms_per_step)
        *ms_per_step = double(t) / iters;
    if (exchange == 2 && (iters & 1))  // the last y sits in the other buffer: make it x
        std::swap(mg->x[0], mg->xnext[0]);
    return 0;
}

// y (nr_rows values) to the host: rank 0's y after a gather / reduce, any rank's x after an
// all-gather (that run's y)
int spmv_mgpu_get_y(spmv_mgpu *mg, ValueType *h_y, int exchange)
{
    if (!mg || !h_y || exchange < 0 || exchange > 2) {
        set_error("spmv_mgpu_get_y: bad arguments");
        return 1;
    }
    const int d = exchange == 2 ? 0 : mg->root_local();
    if (d < 0) {
        set_error("spmv_mgpu_get_y: y of a gather / reduce is on rank 0 only");
        return 1;
    }
    SPMV_TRY(hipSetDevice(mg->dev[d]));
    const ValueType *src = exchange == 2 ? mg->x[d] : mg->y[d];
    if (mg->nr_rows)
        SPMV_TRY(hipMemcpy(h_y, src, size_t(mg->nr_rows) * sizeof(ValueType), hipMemcpyDeviceToHost));
    return 0;
}

// device address of this process's y: rank 0's full y (gather / reduce), else the local device's
// x (all-gather: that run's y) -- for callers that keep y on the GPU
int spmv_mgpu_y_device(spmv_mgpu *mg, int exchange, ValueType **d_y)
{
    if (!mg || !d_y || exchange < 0 || exchange > 2) {
        set_error("spmv_mgpu_y_device: bad arguments");
        return 1;
    }
    const int d = exchange == 2 ? 0 : mg->root_local();
    if (d < 0) {
        set_error("spmv_mgpu_y_device: y of a gather / reduce is on rank 0 only");
        return 1;
    }
    *d_y = exchange == 2 ? mg->x[d] : mg->y[d];
    return 0;
}

int spmv_mgpu_get_timing(const spmv_mgpu *mg, double *compute_ms, double *exchange_ms)
{
    if (!mg) {
        set_error("spmv_mgpu_get_timing: null handle");
        return 1;
    }
    if (compute_ms)
        *compute_ms = mg->compute_ms;
    if (exchange_ms)
        *exchange_ms = mg->exchange_ms;
    return 0;
}

// row slice and HIP device of rank r (device -1 when rank r lives in another process)
int spmv_mgpu_slice(const spmv_mgpu *mg, int r, IndexType *row_begin, IndexType *row_end, int *device)
{
    if (!mg || r < 0 || r >= mg->nranks) {
        set_error("spmv_mgpu_slice: bad arguments");
        return 1;
    }
    if (row_begin)
        *row_begin = mg->bounds[r];
    if (row_end)
        *row_end = mg->bounds[r + 1];
    if (device) {
        *device = -1;
        for (int d = 0; d < mg->nloc; ++d)
            if (mg->rank[d] == r)
                *device = mg->dev[d];
    }
    return 0;
}

int spmv_mgpu_comm_count(const spmv_mgpu *mg, int *count)
{
    if (!mg || !count || !mg->comm[0]) {
        set_error("spmv_mgpu_comm_count: bad arguments");
        return 1;
    }
    MG_NCCL(mg->nc->CommCount(mg->comm[0], count));
    return 0;
}

void spmv_mgpu_destroy(spmv_mgpu *mg) { delete mg; }

}  // extern "C"
