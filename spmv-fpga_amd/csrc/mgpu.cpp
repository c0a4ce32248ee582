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
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclBroadcast) Broadcast = nullptr;
    decltype(&ncclReduce) Reduce = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
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
    SYM(CommDestroy);
    SYM(GetErrorString);
    SYM(GroupStart);
    SYM(GroupEnd);
    SYM(Broadcast);
    SYM(Reduce);
    SYM(Send);
    SYM(Recv);
#undef SYM
    if (!r.CommInitAll || !r.CommDestroy || !r.GetErrorString || !r.GroupStart || !r.GroupEnd || !r.Broadcast ||
        !r.Reduce || !r.Send || !r.Recv) {
        r.h = nullptr;
        return nullptr;
    }
    return &r;
}

constexpr ncclDataType_t kNcclValue = sizeof(ValueType) == 8 ? ncclFloat64 : ncclFloat32;

}  // namespace

struct spmv_mgpu {
    const Rccl *nc = nullptr;
    int ndev = 0;
    IndexType nr_rows = 0, nr_cols = 0;
    std::vector<int> dev;
    std::vector<IndexType> bounds;      // row slice of device d: [bounds[d], bounds[d+1])
    std::vector<spmv_plan *> plan;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<ValueType *> x, xnext;  // full-length x on every device; next x (all-gather)
    std::vector<ValueType *> yslice;    // device d's rows (d > 0; the root computes into y)
    std::vector<ValueType *> ypart;     // reduce mode: full-length partials, zero outside the slice
    ValueType *y = nullptr;             // root's full y
    std::vector<hipEvent_t> ev;         // per device: start, kernels done, exchange done
    double compute_ms = 0, exchange_ms = 0;

    ~spmv_mgpu()
    {
        for (int d = 0; d < ndev; ++d) {
            (void)hipSetDevice(dev[d]);
            if (d < (int)plan.size() && plan[d])
                spmv_plan_destroy(plan[d]);
            for (void *p : {(void *)x[d], (void *)xnext[d], (void *)yslice[d], (void *)ypart[d]})
                if (p)
                    (void)hipFree(p);
            if (d < (int)comm.size() && comm[d] && nc)
                nc->CommDestroy(comm[d]);
            if (stream[d])
                (void)hipStreamDestroy(stream[d]);
            for (int k = 0; k < 3; ++k)
                if (ev[3 * d + k])
                    (void)hipEventDestroy(ev[3 * d + k]);
        }
        if (y) {
            (void)hipSetDevice(dev[0]);
            (void)hipFree(y);
        }
    }
    IndexType rows(int d) const { return bounds[d + 1] - bounds[d]; }
};

#define MG_NCCL(expr)                                                                          \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess) {                                                               \
            set_error(std::string(#expr) + ": " + mg->nc->GetErrorString(r_));               \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

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
    mg->ndev = ndev;
    mg->dev = dl;
    mg->nr_rows = m->nr_rows;
    mg->nr_cols = m->nr_cols;
    mg->plan.assign(ndev, nullptr);
    mg->stream.assign(ndev, nullptr);
    mg->x.assign(ndev, nullptr);
    mg->xnext.assign(ndev, nullptr);
    mg->yslice.assign(ndev, nullptr);
    mg->ypart.assign(ndev, nullptr);
    mg->ev.assign(3 * ndev, nullptr);
    mg->bounds.assign(ndev + 1, 0);
    if (spmv_partition_rows(m->row_ptr, m->nr_rows, ndev, mg->bounds.data()))
        return 1;
    const size_t xb = std::max<size_t>(m->nr_cols, 1) * sizeof(ValueType);
    const size_t nb = std::max<size_t>(m->nr_rows, 1) * sizeof(ValueType);
    for (int d = 0; d < ndev; ++d) {
        SPMV_TRY(hipSetDevice(dl[d]));
        SPMV_TRY(hipStreamCreateWithFlags(&mg->stream[d], hipStreamNonBlocking));
        for (int k = 0; k < 3; ++k)
            SPMV_TRY(hipEventCreate(&mg->ev[3 * d + k]));
        if (spmv_plan_create_host(&mg->plan[d], dl[d], m, mg->bounds[d], mg->bounds[d + 1]))
            return 1;
        SPMV_TRY(hipMalloc((void **)&mg->x[d], xb));
        SPMV_TRY(hipMemset(mg->x[d], 0, xb));
        if (d > 0)
            SPMV_TRY(hipMalloc((void **)&mg->yslice[d], std::max<size_t>(mg->rows(d), 1) * sizeof(ValueType)));
        else
            SPMV_TRY(hipMalloc((void **)&mg->y, nb));
    }
    mg->comm.assign(ndev, nullptr);
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

// x (nr_cols values, host) -> the root device, then one RCCL broadcast to every device
int spmv_mgpu_set_x(spmv_mgpu *mg, const ValueType *h_x)
{
    if (!mg || !h_x) {
        set_error("spmv_mgpu_set_x: bad arguments");
        return 1;
    }
    SPMV_TRY(hipSetDevice(mg->dev[0]));
    if (mg->nr_cols && upload_staged(mg->x[0], h_x, size_t(mg->nr_cols) * sizeof(ValueType), mg->stream[0]))
        return 1;
    if (mg->ndev == 1 || mg->nr_cols == 0)
        return 0;
    MG_NCCL(mg->nc->GroupStart());
    for (int d = 0; d < mg->ndev; ++d)
        MG_NCCL(mg->nc->Broadcast(mg->x[0], mg->x[d], mg->nr_cols, kNcclValue, 0, mg->comm[d], mg->stream[d]));
    MG_NCCL(mg->nc->GroupEnd());
    for (int d = 0; d < mg->ndev; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipStreamSynchronize(mg->stream[d]));
    }
    return 0;
}

int spmv_mgpu_run(spmv_mgpu *mg, int exchange)
{
    if (!mg || exchange < 0 || exchange > 2) {
        set_error("spmv_mgpu_run: bad arguments");
        return 1;
    }
    if (exchange == 2 && mg->nr_rows != mg->nr_cols) {
        set_error("spmv_mgpu_run: the all-gather exchange makes y the next x (needs a square matrix)");
        return 1;
    }
    const int nd = mg->ndev;
    const size_t nb = size_t(mg->nr_rows) * sizeof(ValueType);
    // buffers of the exchange form, allocated on first use
    for (int d = 0; d < nd; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        if (exchange == 1 && nd > 1 && !mg->ypart[d])
            SPMV_TRY(hipMalloc((void **)&mg->ypart[d], std::max<size_t>(nb, sizeof(ValueType))));
        if (exchange == 2 && !mg->xnext[d])
            SPMV_TRY(hipMalloc((void **)&mg->xnext[d], std::max<size_t>(nb, sizeof(ValueType))));
    }
    // where device d's kernels write its rows
    auto dst = [&](int d) -> ValueType * {
        if (exchange == 2)
            return mg->xnext[d] + mg->bounds[d];
        if (exchange == 1 && nd > 1)
            return mg->ypart[d] + mg->bounds[d];
        return d == 0 ? mg->y + mg->bounds[0] : mg->yslice[d];
    };
    for (int d = 0; d < nd; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        hipStream_t s = mg->stream[d];
        SPMV_TRY(hipEventRecord(mg->ev[3 * d], s));
        if (exchange == 1 && nd > 1)  // full-length partial: zero outside the slice
            SPMV_TRY(hipMemsetAsync(mg->ypart[d], 0, nb, s));
        if (mg->rows(d) && spmv_plan_run(mg->plan[d], mg->x[d], dst(d), s))
            return 1;
        SPMV_TRY(hipEventRecord(mg->ev[3 * d + 1], s));
    }
    if (nd > 1 && mg->nr_rows) {
        MG_NCCL(mg->nc->GroupStart());
        for (int d = 0; d < nd; ++d) {
            hipStream_t s = mg->stream[d];
            if (exchange == 0) {
                if (d == 0) {
                    for (int p = 1; p < nd; ++p)
                        if (mg->rows(p))
                            MG_NCCL(mg->nc->Recv(mg->y + mg->bounds[p], mg->rows(p), kNcclValue, p, mg->comm[0], s));
                } else if (mg->rows(d)) {
                    MG_NCCL(mg->nc->Send(mg->yslice[d], mg->rows(d), kNcclValue, 0, mg->comm[d], s));
                }
            } else if (exchange == 1) {
                MG_NCCL(mg->nc->Reduce(mg->ypart[d], d == 0 ? mg->y : nullptr, mg->nr_rows, kNcclValue, ncclSum, 0,
                                       mg->comm[d], s));
            } else {
                for (int r = 0; r < nd; ++r)  // slice r from its owner into every device's next x
                    if (mg->rows(r))
                        MG_NCCL(mg->nc->Broadcast(mg->xnext[d] + mg->bounds[r], mg->xnext[d] + mg->bounds[r],
                                                  mg->rows(r), kNcclValue, r, mg->comm[d], s));
            }
        }
        MG_NCCL(mg->nc->GroupEnd());
    }
    double cmax = 0, tmax = 0;
    for (int d = 0; d < nd; ++d) {
        SPMV_TRY(hipSetDevice(mg->dev[d]));
        SPMV_TRY(hipEventRecord(mg->ev[3 * d + 2], mg->stream[d]));
    }
    for (int d = 0; d < nd; ++d) {
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
        for (int d = 0; d < nd; ++d)
            std::swap(mg->x[d], mg->xnext[d]);  // y becomes the next x on every device
    return 0;
}

// y (nr_rows values) to the host: the root's y after a gather / reduce, device 0's x after an
// all-gather (that run's y)
int spmv_mgpu_get_y(spmv_mgpu *mg, ValueType *h_y, int exchange)
{
    if (!mg || !h_y || exchange < 0 || exchange > 2) {
        set_error("spmv_mgpu_get_y: bad arguments");
        return 1;
    }
    SPMV_TRY(hipSetDevice(mg->dev[0]));
    const ValueType *src = exchange == 2 ? mg->x[0] : mg->y;
    if (mg->nr_rows)
        SPMV_TRY(hipMemcpy(h_y, src, size_t(mg->nr_rows) * sizeof(ValueType), hipMemcpyDeviceToHost));
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

int spmv_mgpu_slice(const spmv_mgpu *mg, int d, IndexType *row_begin, IndexType *row_end, int *device)
{
    if (!mg || d < 0 || d >= mg->ndev) {
        set_error("spmv_mgpu_slice: bad arguments");
        return 1;
    }
    if (row_begin)
        *row_begin = mg->bounds[d];
    if (row_end)
        *row_end = mg->bounds[d + 1];
    if (device)
        *device = mg->dev[d];
    return 0;
}

void spmv_mgpu_destroy(spmv_mgpu *mg) { delete mg; }

}  // extern "C"
