// Host side of the MI355X hw representation: O(rows + nnz/32) metadata build, device
// upload/pack, launch sequence, timing, nnz-balanced partitioning.
//
// Roles taken over from the reference's host format builder (csr_hw.cpp):
//   scan_matrix (:7-146)                  -> one pass over row_ptr (no per-nnz block search)
//   prepare_balanced_hw_matrix (:327-361) -> empty rows become the row_id map; the per-CU
//                                            nnz balance is spmv_partition_rows (units)
//   hw_matrix_alloc (:151-183)            -> hipMalloc of the plan buffers
//   create_block_matrix +
//   generate_balanced_hw_submatrix (:190-318) -> k_pack on the GPU (O(nnz), coalesced)
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "spmv_internal.hpp"

static int run_impl(spmv_plan *p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool timing);

namespace spmvhw {

// Host -> device copy of a pageable buffer through two pinned 32 MiB staging buffers (process
// lifetime): host threads fill one buffer while the DMA engine drains the other. A pageable
// hipMemcpy runs at ~1 GB/s here; this keeps the PCIe link busy instead.
int upload_staged(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    constexpr size_t kChunk = 32u << 20;
    if (bytes < (4u << 20)) {
        SPMV_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        SPMV_TRY(hipStreamSynchronize(s));
        return 0;
    }
    static std::mutex mu;
    static void *buf[2] = {nullptr, nullptr};
    static hipEvent_t done[2] = {nullptr, nullptr};
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < 2; ++i) {
        if (!buf[i])
            SPMV_TRY(hipHostMalloc(&buf[i], kChunk, hipHostMallocPortable));
        if (!done[i])
            SPMV_TRY(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
    }
    bool pending[2] = {false, false};
    const unsigned hc = std::thread::hardware_concurrency();
    const int T = (int)std::min(4u, hc ? hc : 1u);
    int i = 0;
    for (size_t off = 0; off < bytes; off += kChunk, i ^= 1) {
        const size_t n = std::min(kChunk, bytes - off);
        if (pending[i])
            SPMV_TRY(hipEventSynchronize(done[i]));  // the DMA out of this buffer has finished
        auto part = [&](int t) {
            const size_t b = n * t / T, e = n * (t + 1) / T;
            std::memcpy((char *)buf[i] + b, (const char *)src + off + b, e - b);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t)
            th.emplace_back(part, t);
        part(0);
        for (auto &t : th)
            t.join();
        SPMV_TRY(hipMemcpyAsync((char *)dst + off, buf[i], n, hipMemcpyHostToDevice, s));
        SPMV_TRY(hipEventRecord(done[i], s));
        pending[i] = true;
    }
    SPMV_TRY(hipStreamSynchronize(s));
    return 0;
}

// env SPMV_HW_TRACE=1: phase times of plan construction on stderr
struct PhaseTrace {
    const bool on = std::getenv("SPMV_HW_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
    void operator()(const char *phase, hipStream_t s)
    {
        if (!on)
            return;
        (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "spmv_hw trace: %-28s %9.3f ms (total %9.3f ms)\n", phase,
                     std::chrono::duration<double, std::milli>(now - last).count(),
                     std::chrono::duration<double, std::milli>(now - t0).count());
        last = now;
    }
};

constexpr int kKernelTune = -2;

// Which kernel a plan uses: env SPMV_HW_KERNEL = tiles | sweep | gold | tune | auto (default).
static int requested_kernel()
{
    const char *e = std::getenv("SPMV_HW_KERNEL");
    if (!e || !*e || !std::strcmp(e, "auto"))
        return -1;
    if (!std::strcmp(e, "tune"))
        return kKernelTune;
    if (!std::strcmp(e, "tiles"))
        return kKernelTiles;
    if (!std::strcmp(e, "sweep"))
        return kKernelSweep;
    if (!std::strcmp(e, "gold"))
        return kKernelGold;
    if (!std::strcmp(e, "fpga"))
        return kKernelFpga;
    if (!std::strcmp(e, "blocked"))
        return kKernelBlocked;
    if (!std::strcmp(e, "slices"))
        return kKernelSlices;
    if (!std::strcmp(e, "binned"))
        return kKernelBinned;
    return -1;
}

// Gold-order representation (kernel 1): the CSR itself (nlong counts the rows longer than
// kGoldLong, for the stats only).
static int build_gold(spmv_plan &p, const IndexType *h_row_ptr, const IndexType *d_col_src,
                      const ValueType *d_val_src, hipStream_t s)
{
    p.nlong = 0;
    for (IndexType r = 0; r < p.nr_rows; ++r)
        p.nlong += h_row_ptr[r + 1] - h_row_ptr[r] > (IndexType)kGoldLong;
    SPMV_TRY(hipMalloc((void **)&p.d_rp, (size_t(p.nr_rows) + 1) * sizeof(uint32_t)));
    SPMV_TRY(hipMalloc((void **)&p.d_col, std::max<uint64_t>(p.nnz, 1) * sizeof(uint32_t)));
    SPMV_TRY(hipMalloc((void **)&p.d_val, std::max<uint64_t>(p.nnz, 1) * sizeof(ValueType)));
    SPMV_TRY(hipMemcpyAsync(p.d_rp, h_row_ptr, (size_t(p.nr_rows) + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    if (p.nnz) {
        SPMV_TRY(hipMemcpyAsync(p.d_col, d_col_src, p.nnz * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        SPMV_TRY(hipMemcpyAsync(p.d_val, d_val_src, p.nnz * sizeof(ValueType), hipMemcpyDeviceToDevice, s));
    }
    SPMV_TRY(hipStreamSynchronize(s));
    return 0;
}

// Flagged-tile representation (kernel 0): row-end bitmap, tile table, packed col/val.
static int build_tiles(spmv_plan &p, const IndexType *h_row_ptr, const IndexType *d_col_src,
                       const ValueType *d_val_src, hipStream_t s)
{
    const IndexType nr_rows = p.nr_rows;
    const uint64_t nnz = p.nnz;
    p.nnz_pad = (nnz + kTileNnz - 1) / kTileNnz * kTileNnz;
    p.ntiles = p.nnz_pad / kTileNnz;

    std::vector<uint32_t> rowend(p.nnz_pad / 32, 0u);
    std::vector<uint32_t> row_id;
    if (p.has_empty)
        row_id.reserve(p.nzr);
    for (IndexType r = 0; r < nr_rows; ++r) {
        if (h_row_ptr[r + 1] > h_row_ptr[r]) {
            const uint64_t e = h_row_ptr[r + 1] - 1ull;
            rowend[e >> 5] |= 1u << (e & 31);
            if (p.has_empty)
                row_id.push_back(r);
        }
    }
    std::vector<uint32_t> tile_info(p.ntiles + 1, 0u);
    {
        uint64_t rr = 0, c = 0;
        for (uint64_t t = 0; t <= p.ntiles; ++t) {
            const uint64_t k = t * kTileNnz;
            while (rr < nr_rows && h_row_ptr[rr + 1] <= k) {
                if (h_row_ptr[rr + 1] > h_row_ptr[rr])
                    ++c;
                ++rr;
            }
            if (c > 0x7FFFFFFFull) {
                set_error("too many non-empty rows for the tile table");
                return 1;
            }
            const bool cont = k > 0 && k < nnz && !((rowend[(k - 1) >> 5] >> ((k - 1) & 31)) & 1u);
            tile_info[t] = (uint32_t)(c << 1) | (cont ? 1u : 0u);
        }
    }
    // rows crossing tile boundaries (structural): tile t "has a tail" when its last entry is not
    // a row end and entries follow; a crossing starts at a tile with a tail whose row began in
    // it, and ends at the next tile that contains a row end
    std::vector<uint32_t> cross;
    {
        auto bit = [&](uint64_t k) { return (rowend[k >> 5] >> (k & 31)) & 1u; };
        std::vector<uint8_t> has_tail(p.ntiles, 0), has_end(p.ntiles, 0);
        for (uint64_t t = 0; t < p.ntiles; ++t) {
            const uint64_t w0 = t * (kTileNnz / 32);
            for (uint64_t w = 0; w < kTileNnz / 32; ++w)
                has_end[t] |= rowend[w0 + w] != 0;
            const uint64_t last = (t + 1) * kTileNnz - 1;
            has_tail[t] = (last + 1 < nnz) && !bit(last);
        }
        for (uint64_t t = 0; t < p.ntiles; ++t) {
            if (!has_tail[t] || !(has_end[t] || t == 0 || !has_tail[t - 1]))
                continue;
            uint64_t j = t + 1;
            while (j < p.ntiles && !has_end[j])
                ++j;
            if (j >= p.ntiles) {
                set_error("internal: unterminated row crossing");
                return 1;
            }
            cross.push_back(tile_info[t + 1] >> 1);
            cross.push_back((uint32_t)t);
            cross.push_back((uint32_t)j);
        }
        p.ncross = cross.size() / 3;
    }
    auto alloc = [&](void **ptr, size_t bytes) -> hipError_t {
        *ptr = nullptr;
        return bytes ? hipMalloc(ptr, bytes) : hipSuccess;
    };
    SPMV_TRY(alloc((void **)&p.d_col, p.nnz_pad * sizeof(uint32_t)));
    SPMV_TRY(alloc((void **)&p.d_val, p.nnz_pad * sizeof(ValueType)));
    SPMV_TRY(alloc((void **)&p.d_rowend, rowend.size() * sizeof(uint32_t)));
    SPMV_TRY(alloc((void **)&p.d_tile_info, tile_info.size() * sizeof(uint32_t)));
    SPMV_TRY(alloc((void **)&p.d_head, p.ntiles * sizeof(ValueType)));
    SPMV_TRY(alloc((void **)&p.d_tail, p.ntiles * sizeof(ValueType)));
    SPMV_TRY(alloc((void **)&p.d_cross, cross.size() * sizeof(uint32_t)));
    if (p.has_empty)
        SPMV_TRY(alloc((void **)&p.d_row_id, row_id.size() * sizeof(uint32_t)));
    if (!rowend.empty())
        SPMV_TRY(hipMemcpyAsync(p.d_rowend, rowend.data(), rowend.size() * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMemcpyAsync(p.d_tile_info, tile_info.data(), tile_info.size() * 4, hipMemcpyHostToDevice, s));
    if (p.has_empty && !row_id.empty())
        SPMV_TRY(hipMemcpyAsync(p.d_row_id, row_id.data(), row_id.size() * 4, hipMemcpyHostToDevice, s));
    if (!cross.empty())
        SPMV_TRY(hipMemcpyAsync(p.d_cross, cross.data(), cross.size() * 4, hipMemcpyHostToDevice, s));
    if (p.nnz_pad)
        SPMV_TRY(launch_pack(d_col_src, d_val_src, nnz, p.nnz_pad, p.nr_cols, p.d_col, p.d_val, nullptr, s));
    if (const char *xe = ablation_env("SPMV_TILE_XCD"))
        p.tile_xcd = xe[0] == '1';
    // narrow form: 8- or 16-bit column offsets from a per-tile base when every tile allows it
    // (env SPMV_TILE_NARROW: 0 = keep 32-bit columns, 16 = at most 16-bit, default narrowest)
    const char *nenv = ablation_env("SPMV_TILE_NARROW");
    const int narrow_min = !nenv || !*nenv ? 1 : std::atoi(nenv) == 16 ? 2 : std::atoi(nenv) == 0 ? 4 : 1;
    if (p.ntiles && narrow_min < 4) {
        uint32_t *d_span = nullptr;
        SPMV_TRY(alloc((void **)&p.d_tile_cbase, p.ntiles * sizeof(uint32_t)));
        SPMV_TRY(alloc((void **)&d_span, sizeof(uint32_t)));
        uint32_t span = 0xFFFFFFFFu;
        hipError_t e = hipMemsetAsync(d_span, 0, sizeof(uint32_t), s);
        if (e == hipSuccess)
            e = launch_tile_span(p.d_col, nnz, p.ntiles, p.d_tile_cbase, d_span, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(&span, d_span, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess)
            e = hipStreamSynchronize(s);
        (void)hipFree(d_span);
        SPMV_TRY(e);
        const int cb = span < 256u && narrow_min <= 1 ? 1 : span < 65536u ? 2 : 4;
        if (cb < 4) {
            SPMV_TRY(alloc(&p.d_colnar, p.nnz_pad * cb));
            SPMV_TRY(launch_narrow(p.d_col, nnz, p.nnz_pad, p.d_tile_cbase, p.d_colnar, cb, s));
            SPMV_TRY(hipStreamSynchronize(s));
            SPMV_TRY(hipFree(p.d_col));
            p.d_col = nullptr;
            p.tile_col_bytes = cb;
        } else {
            SPMV_TRY(hipFree(p.d_tile_cbase));
            p.d_tile_cbase = nullptr;
            // clustered 16-bit columns: up to four narrow column clusters per tile
            const char *cenv = ablation_env("SPMV_TILE_CLUSTER");
            if (!(cenv && cenv[0] == '0')) {
                uint32_t *d_bad = nullptr;
                SPMV_TRY(alloc((void **)&p.d_tile_cbase, p.ntiles * 4 * sizeof(uint32_t)));
                SPMV_TRY(alloc((void **)&d_bad, sizeof(uint32_t)));
                uint32_t bad = 1;
                e = hipMemsetAsync(d_bad, 0, sizeof(uint32_t), s);
                if (e == hipSuccess)
                    e = launch_tile_clusters(p.d_col, nnz, p.ntiles, p.d_tile_cbase, d_bad, s);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(&bad, d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
                if (e == hipSuccess)
                    e = hipStreamSynchronize(s);
                (void)hipFree(d_bad);
                SPMV_TRY(e);
                if (!bad) {
                    SPMV_TRY(alloc(&p.d_colnar, p.nnz_pad * 2));
                    SPMV_TRY(launch_cluster_encode(p.d_col, nnz, p.nnz_pad, p.d_tile_cbase, (uint16_t *)p.d_colnar, s));
                    SPMV_TRY(hipStreamSynchronize(s));
                    SPMV_TRY(hipFree(p.d_col));
                    p.d_col = nullptr;
                    p.tile_col_bytes = 2;
                    p.tile_clustered = true;
                } else {
                    SPMV_TRY(hipFree(p.d_tile_cbase));
                    p.d_tile_cbase = nullptr;
                }
            }
        }
    }
    // pageable host vectors above go out of scope: make the copies complete first
    SPMV_TRY(hipStreamSynchronize(s));
    return 0;
}

// FPGA order: VF / block width from the environment (the reference's compile-time VF and
// COLS_DIV_BLOCKS, util.h:31-59; defaults VF = 1 as its Makefile:16, 32768 columns), and every
// row's entries stably ordered by column block (the reference walks each block's entries of a
// row in CSR order, create_block_matrix); rows that are already block-ordered stay as they are.
static int fpga_params(spmv_plan &p)
{
    if (const char *v = std::getenv("SPMV_FPGA_VF")) {
        const int vf = std::atoi(v);
        if (vf != 1 && vf != 2 && vf != 4 && vf != 8) {
            set_error("SPMV_FPGA_VF must be 1, 2, 4 or 8");
            return 1;
        }
        p.fpga_vf = vf;
    }
    if (const char *b = std::getenv("SPMV_FPGA_BLOCK")) {
        const long w = std::atol(b);
        if (w < 1 || w > 0x7FFFFFFFL) {
            set_error("SPMV_FPGA_BLOCK must be a positive column count");
            return 1;
        }
        p.fpga_width = (uint32_t)w;
    }
    return 0;
}

static int order_rows_by_block(spmv_plan &p, const IndexType *h_row_ptr, hipStream_t s)
{
    if (fpga_params(p))
        return 1;
    if (!p.nnz)
        return 0;
    std::vector<uint32_t> col(p.nnz);
    SPMV_TRY(hipMemcpyAsync(col.data(), p.d_col, p.nnz * 4, hipMemcpyDeviceToHost, s));
    SPMV_TRY(hipStreamSynchronize(s));
    bool sorted = true;
    for (IndexType r = 0; r < p.nr_rows && sorted; ++r)
        for (uint64_t k = uint64_t(h_row_ptr[r]) + 1; k < h_row_ptr[r + 1]; ++k)
            if (col[k] / p.fpga_width < col[k - 1] / p.fpga_width) {
                sorted = false;
                break;
            }
    if (sorted)
        return 0;
    std::vector<ValueType> val(p.nnz);
    SPMV_TRY(hipMemcpyAsync(val.data(), p.d_val, p.nnz * sizeof(ValueType), hipMemcpyDeviceToHost, s));
    SPMV_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> idx;
    std::vector<uint32_t> c2(col);
    std::vector<ValueType> v2(val);
    for (IndexType r = 0; r < p.nr_rows; ++r) {
        const uint64_t b = h_row_ptr[r], e = h_row_ptr[r + 1];
        idx.resize(e - b);
        for (uint64_t k = b; k < e; ++k)
            idx[k - b] = (uint32_t)k;
        std::stable_sort(idx.begin(), idx.end(),
                         [&](uint32_t i, uint32_t j) { return col[i] / p.fpga_width < col[j] / p.fpga_width; });
        for (uint64_t k = b; k < e; ++k) {
            c2[k] = col[idx[k - b]];
            v2[k] = val[idx[k - b]];
        }
    }
    SPMV_TRY(hipMemcpyAsync(p.d_col, c2.data(), p.nnz * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMemcpyAsync(p.d_val, v2.data(), p.nnz * sizeof(ValueType), hipMemcpyHostToDevice, s));
    SPMV_TRY(hipStreamSynchronize(s));
    return 0;
}

// Builds plan P's layout for `kernel` from the validated device CSR and loads its kernels.
static int build_layout(spmv_plan &P, int kernel, bool automatic, const IndexType *h_row_ptr,
                        const IndexType *d_col, const ValueType *d_val, hipStream_t s)
{
    P.kernel = kernel;
    if (kernel == kKernelBinned) {
        // rc 2: the (window, panel) segment table is too large; automatic plans take the sweep
        const int rc = build_binned(P, h_row_ptr, d_col, d_val, s);
        if (rc == 2 && automatic) {
            P.kernel = kernel = kKernelSweep;
            (void)hipGetLastError();
        } else if (rc) {
            return 1;
        }
    }
    if (kernel == kKernelSweep || kernel == kKernelSlices) {
        // rc 2: the layout cannot hold this matrix (32-bit entry offsets, or the automatic
        // choice's padding limit); automatic plans fall back to the tiles, which have neither
        const int rc = kernel == kKernelSweep ? build_sweep(P, h_row_ptr, d_col, d_val, s)
                                              : build_slices(P, h_row_ptr, d_col, d_val, s);
        if (rc == 2 && automatic)
            P.kernel = kernel = kKernelTiles;
        else if (rc)
            return 1;
    }
    if (kernel == kKernelSweep || kernel == kKernelSlices || kernel == kKernelBinned) {
        // built above
    } else if (kernel == kKernelBlocked) {
        if (fpga_params(P) || build_blocked(P, h_row_ptr, d_col, d_val, s))
            return 1;
    } else if (kernel == kKernelGold || kernel == kKernelFpga) {
        if (build_gold(P, h_row_ptr, d_col, d_val, s))
            return 1;
        if (kernel == kKernelFpga && order_rows_by_block(P, h_row_ptr, s))
            return 1;
    } else {
        if (build_tiles(P, h_row_ptr, d_col, d_val, s))
            return 1;
    }
    SPMV_TRY(hipStreamSynchronize(s));
    // load the code objects of the kernels this plan launches (no launch; best effort: a
    // failure here only means the first run loads them)
    if (P.kernel == kKernelSweep) {
        (void)launch_sweep(P, nullptr, nullptr, s, true);
    } else if (P.kernel == kKernelBinned) {
        (void)launch_binned(P, nullptr, nullptr, s, true);
    } else if (P.kernel == kKernelBlocked) {
        (void)launch_blocked(P, nullptr, nullptr, s, true);
    } else if (P.kernel == kKernelSlices) {
        (void)launch_slices(P, nullptr, nullptr, s, true);
    } else if (P.kernel == kKernelGold || P.kernel == kKernelFpga) {
        (void)launch_gold(P, nullptr, nullptr, s, true);
    } else {
        (void)launch_spmv(P, nullptr, nullptr, s, true);
        (void)launch_fixup(P, nullptr, s, true);
    }
    (void)hipGetLastError();
    return 0;
}

// ms per SpMV of a layout with scratch x/y, for SPMV_HW_KERNEL=tune: kTuneSteps serial SpMVs
// captured into one hipGraph on a private stream (no host launch gap inside a sample), replayed
// once to warm, then kTuneReps replays each timed with its own event pair; the median replay / steps.
// One timed launch per candidate (round 4) let the timer's noise pick the layout.
constexpr int kTuneSteps = 4, kTuneReps = 7;
static int time_layout(spmv_plan &P, const ValueType *d_x, ValueType *d_y, hipStream_t s, double *ms)
{
    SPMV_TRY(hipStreamSynchronize(s));  // the layout was built on s
    struct Res {
        hipStream_t ts = nullptr;
        hipGraphExec_t ge = nullptr;
        hipEvent_t ev[2 * kTuneReps] = {};
        ~Res()
        {
            for (hipEvent_t e : ev)
                if (e)
                    (void)hipEventDestroy(e);
            if (ge)
                (void)hipGraphExecDestroy(ge);
            if (ts)
                (void)hipStreamDestroy(ts);
        }
    } r;
    SPMV_TRY(hipStreamCreateWithFlags(&r.ts, hipStreamNonBlocking));
    for (hipEvent_t &e : r.ev)
        SPMV_TRY(hipEventCreate(&e));
    SPMV_TRY(hipStreamBeginCapture(r.ts, hipStreamCaptureModeRelaxed));
    int rc = 0;
    for (int i = 0; i < kTuneSteps && !rc; ++i)
        rc = ::run_impl(&P, d_x, d_y, r.ts, false);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(r.ts, &g);
    if (rc) {
        if (g)
            (void)hipGraphDestroy(g);
        return rc;
    }
    SPMV_TRY(ec);
    const hipError_t ei = hipGraphInstantiate(&r.ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    SPMV_TRY(ei);
    SPMV_TRY(hipGraphLaunch(r.ge, r.ts));  // warm
    for (int k = 0; k < kTuneReps; ++k) {
        SPMV_TRY(hipEventRecord(r.ev[2 * k], r.ts));
        SPMV_TRY(hipGraphLaunch(r.ge, r.ts));
        SPMV_TRY(hipEventRecord(r.ev[2 * k + 1], r.ts));
    }
    SPMV_TRY(hipStreamSynchronize(r.ts));
    std::vector<double> t(kTuneReps);
    for (int k = 0; k < kTuneReps; ++k) {
        float v = 0.f;
        SPMV_TRY(hipEventElapsedTime(&v, r.ev[2 * k], r.ev[2 * k + 1]));
        t[k] = v / kTuneSteps;
    }
    std::nth_element(t.begin(), t.begin() + kTuneReps / 2, t.end());
    *ms = t[kTuneReps / 2];
    return 0;
}

int plan_create_from_host_rowptr(spmv_plan **out, int device, IndexType nr_rows, IndexType nr_cols,
                                 const IndexType *h_row_ptr, const IndexType *col_src,
                                 const ValueType *val_src, bool src_on_device, hipStream_t s)
{
    *out = nullptr;
    PhaseTrace trace;
    if (nr_rows > 0 && h_row_ptr[0] != 0) {
        set_error("row_ptr must be rebased to 0");
        return 1;
    }
    const uint64_t nnz = nr_rows ? h_row_ptr[nr_rows] : 0;
    uint64_t nzr = 0;
    for (IndexType r = 0; r < nr_rows; ++r) {
        if (h_row_ptr[r + 1] < h_row_ptr[r]) {
            set_error("row_ptr is not non-decreasing at row " + std::to_string(r));
            return 1;
        }
        nzr += h_row_ptr[r + 1] > h_row_ptr[r];
    }
    if (nnz > 0 && nr_cols == 0) {
        set_error("matrix has non-zeros but zero columns");
        return 1;
    }
    SPMV_TRY(hipSetDevice(device));

    std::unique_ptr<spmv_plan> p(new spmv_plan());
    p->device = device;
    p->nr_rows = nr_rows;
    p->nr_cols = nr_cols;
    p->nnz = nnz;
    p->nzr = nzr;
    p->has_empty = nzr < nr_rows;

    // device copies of the CSR entries (host path: upload), validated before any kernel gathers
    struct Tmp {
        void *p = nullptr;
        ~Tmp() { if (p) (void)hipFree(p); }
    } tcol, tval, trp, tbad;
    const IndexType *d_col = col_src;
    const ValueType *d_val = val_src;
    if (!src_on_device && nnz) {
        SPMV_TRY(hipMalloc(&tcol.p, nnz * sizeof(IndexType)));
        SPMV_TRY(hipMalloc(&tval.p, nnz * sizeof(ValueType)));
        if (upload_staged(tcol.p, col_src, nnz * sizeof(IndexType), s) ||
            upload_staged(tval.p, val_src, nnz * sizeof(ValueType), s))
            return 1;
        d_col = (const IndexType *)tcol.p;
        d_val = (const ValueType *)tval.p;
    }
    trace("row_ptr scan + upload", s);
    if (nnz) {
        SPMV_TRY(hipMalloc(&tbad.p, sizeof(uint32_t)));
        SPMV_TRY(hipMemsetAsync(tbad.p, 0, sizeof(uint32_t), s));
        SPMV_TRY(launch_validate(d_col, nnz, nr_cols, (uint32_t *)tbad.p, s));
        uint32_t bad = 0;
        SPMV_TRY(hipMemcpyAsync(&bad, tbad.p, sizeof(bad), hipMemcpyDeviceToHost, s));
        SPMV_TRY(hipStreamSynchronize(s));
        if (bad) {
            set_error("column index out of range (>= nr_cols)");
            return 1;
        }
    }

    int kernel = requested_kernel();
    const bool tune = kernel == kKernelTune;
    if (kernel == -1 || tune) {  // (tune: the automatic choice is the preferred candidate)
        // automatic choice: the sweep pays once x outgrows ~half an XCD's L2 and the columns of a
        // row are scattered: fewer than 30 % of the consecutive column pairs of sampled rows lie
        // < 64 apart (random: ~0; 2-D 5-point stencil 0.5, 3-D 7-point 0.33, 27-point 0.69, where
        // the (clustered) tile layout is as fast or faster). Measured on power-law matrices with
        // 16 nnz/row (profiles/r01_ab_variants.jsonl): tie at x = 1.6 MB, sweep 1.2x faster at
        // 2.4 MB, 2.3x at 8 MB, 3.4x at 16 MB, 3.9x at 80 MB.
        kernel = kKernelTiles;
        if (nnz && uint64_t(nr_cols) * sizeof(ValueType) >= (2ull << 20) && nnz >= 16ull * kSweepThreads) {
            SPMV_TRY(hipMalloc(&trp.p, (size_t(nr_rows) + 1) * sizeof(IndexType)));
            SPMV_TRY(hipMemcpyAsync(trp.p, h_row_ptr, (size_t(nr_rows) + 1) * sizeof(IndexType),
                                    hipMemcpyHostToDevice, s));
            if (probe_locality((const IndexType *)trp.p, d_col, nr_rows, s, &p->locality))
                return 1;
            if (p->locality < 0.3)
                kernel = kKernelSweep;
        }
        // fp32, scattered, x of >= 20 MB: the two-pass binned kernel (binned.hip) streams 15-16 B
        // per non-zero instead of gathering x lines (skewed matrices excepted, build_binned). Measured on the power-law generator
        // (profiles/r02_binned.jsonl, profiles/r02_strong_binned.jsonl): square n x n, 16n nnz:
        // 4M 0.203 vs 0.199 ms (sweep), 6M 0.317 vs 0.374, 10M 0.457 vs 0.616, 20M 0.964 vs
        // 1.450; row slices of the 10M x 10M matrix (x stays 40 MB): 5M rows / 80M nnz 0.251
        // vs 0.312, 2.5M / 40M 0.144 vs 0.178, 1.25M / 20M 0.093 vs 0.106. In fp64 (27-28 B per
        // non-zero) the sweep stays as fast or faster (10M: binned 0.80-0.86 vs 0.78-0.80 ms;
        // slices slower).
        // Its pass 2 adds in timing order; SPMV_SWEEP_DETERMINISTIC=1 asks for fixed bits, which
        // the turn-ordered sweep gives, so the switch keeps the sweep.
        const char *det = std::getenv("SPMV_SWEEP_DETERMINISTIC");
        if (kernel == kKernelSweep && sizeof(ValueType) == 4 && nr_cols >= 5000000u && nnz >= 16000000ull &&
            !(det && det[0] == '1'))
            kernel = kKernelBinned;
    }
    const int auto_kernel = kernel;
    if (tune)
        kernel = kKernelTune;
    trace("validate + kernel choice", s);
    if (const char *t = ablation_env("SPMV_SWEEP_THREADS")) {
        const int v = std::atoi(t);
        if (v == 256 || v == 512 || v == 1024)
            p->sweep_threads = v;
    }
    auto fresh = [&]() {
        std::unique_ptr<spmv_plan> q(new spmv_plan());
        q->device = p->device;
        q->nr_rows = p->nr_rows;
        q->nr_cols = p->nr_cols;
        q->nnz = p->nnz;
        q->nzr = p->nzr;
        q->has_empty = p->has_empty;
        q->sweep_threads = p->sweep_threads;
        q->locality = p->locality;
        return q;
    };
    if (kernel == kKernelTune) {
        // build the tile, sweep, slice and binned layouts one at a time and time each on this
        // matrix (time_layout: median of graph-replayed samples). The candidates go in preference
        // order -- the automatic choice first, then tiles, sweep, slices, binned -- and a later one
        // replaces the kept layout only when it is more than 3 % faster, so two layouts within
        // the timer's noise of each other cannot trade places between two builds of one matrix.
        // Only the kept layout and the candidate are resident; a candidate whose build fails
        // (e.g. out of memory) is dropped, not a plan error. With SPMV_SWEEP_DETERMINISTIC=1 the
        // binned layout (pass-2 adds in timing order) is not a candidate: the switch promises
        // fixed bits.
        const char *det = std::getenv("SPMV_SWEEP_DETERMINISTIC");
        const bool fixed_bits = det && det[0] == '1';
        constexpr double kTuneBand = 0.97;
        Tmp tx, ty;
        SPMV_TRY(hipMalloc(&tx.p, std::max<size_t>(nr_cols, 1) * sizeof(ValueType)));
        SPMV_TRY(hipMalloc(&ty.p, std::max<size_t>(nr_rows, 1) * sizeof(ValueType)));
        SPMV_TRY(hipMemsetAsync(tx.p, 0, std::max<size_t>(nr_cols, 1) * sizeof(ValueType), s));
        const int slot_of[7] = {0, -1, 1, -1, -1, 2, 3};  // kernel id -> tuned_ms slot
        std::vector<int> order = {auto_kernel};
        for (int k : {kKernelTiles, kKernelSweep, kKernelSlices, kKernelBinned})
            if (k != auto_kernel)
                order.push_back(k);
        double tuned[4] = {1e30, 1e30, 1e30, 1e30};
        std::unique_ptr<spmv_plan> kept;
        double kept_ms = 1e30;
        for (int k : order) {
            if (k == kKernelBinned && fixed_bits)
                continue;
            std::unique_ptr<spmv_plan> q = fresh();
            if (k == kKernelSlices)
                q->slice_pad_limit = 2.0;  // a slice layout padded beyond 2x is built as tiles instead
            double t = 1e30;
            if (build_layout(*q, k, true, h_row_ptr, d_col, d_val, s) ||
                time_layout(*q, (const ValueType *)tx.p, (ValueType *)ty.p, s, &t)) {
                q.reset();  // not a candidate
                (void)hipGetLastError();
                continue;
            }
            tuned[slot_of[k]] = t;
            if (!kept || t < kTuneBand * kept_ms) {
                kept.swap(q);
                kept_ms = t;
            }
        }
        if (!kept) {  // every candidate failed: the tiles, untimed (their error is the plan's)
            if (build_layout(*p, kKernelTiles, true, h_row_ptr, d_col, d_val, s))
                return 1;
        } else {
            p.swap(kept);
        }
        if (std::getenv("SPMV_HW_TRACE"))
            std::fprintf(stderr, "spmv_hw trace: tune ms tiles %.4f sweep %.4f slices %.4f binned %.4f -> kernel %d\n",
                         tuned[0], tuned[1], tuned[2], tuned[3], p->kernel);
        for (int c = 0; c < 4; ++c)
            p->tuned_ms[c] = tuned[c];
        trace("tune: build + time each", s);
    } else if (requested_kernel() < 0 && kernel == kKernelTiles && nnz >= 65536) {
        // automatic, local columns: the slice layout when rows of a 64-row slice have about the
        // same length (<= 15 % padding) and every slot fits 16-bit (or clustered 16-bit) offsets
        // -- finite-element / stencil-like matrices, where it is 7-14 % faster than the tiles
        // (fp32: 24-34 %, profiles/r01_ab_variants.jsonl); in fp64, 8-bit spans (narrow bands)
        // keep the tiles, which gather a band's x from fewer lines per instruction (the fp32
        // band is 13 % faster in slices)
        std::unique_ptr<spmv_plan> r = fresh();
        r->slice_pad_limit = 1.15;
        const int rc = build_layout(*r, kKernelSlices, true, h_row_ptr, d_col, d_val, s);
        if (rc == 0 && r->kernel == kKernelSlices &&
            (r->slice_off_bytes == 2 || (r->slice_off_bytes == 1 && sizeof(ValueType) == 4)) &&
            double(r->slice_slots) * kWave <= 1.15 * double(nnz)) {
            p.swap(r);
            trace("build slice layout", s);
        } else if (rc == 0 && r->kernel == kKernelTiles) {  // padding too high: built as tiles
            r->slice_pad_limit = 0.0;
            p.swap(r);
            trace("build tile layout", s);
        } else {
            r.reset();
            (void)hipGetLastError();
            if (build_layout(*p, kKernelTiles, true, h_row_ptr, d_col, d_val, s))
                return 1;
            trace("build tile layout", s);
        }
    } else {
        if (kernel == kKernelBinned && requested_kernel() < 0) {
            p->bin_skew_limit = 2.0;  // automatic: skewed matrices stay on the sweep
            // and so do matrices with a row above 0.3x a panel's mean entries: 2M x 6M fp32 with
            // 64 rows of L (profiles/r03e_skew_rowlimit.jsonl; L / mean 0.12, 0.24, 0.44, 0.81):
            // binned 0.136 / 0.178 / 0.254 / 0.282 ms, sweep 0.155 / 0.183 / 0.225 / 0.298
            p->bin_row_limit = 0.3;
            if (const char *e = std::getenv("SPMV_BIN_ROW_LIMIT"))
                p->bin_row_limit = std::atof(e);
        }
        if (build_layout(*p, kernel, requested_kernel() < 0, h_row_ptr, d_col, d_val, s))
            return 1;
        trace(p->kernel == kKernelSweep ? "build sweep layout" : p->kernel == kKernelBinned ? "build binned layout"
              : p->kernel != kKernelTiles ? "build CSR layout"
                                                                                        : "build tile layout", s);
    }
    *out = p.release();
    return 0;
}

// the variants the product library accepts, per kernel (spmv_plan_set_variant)
bool product_variant(int kernel, int variant)
{
    if (variant == 0)
        return true;
    if (kernel == kKernelSweep)
        return variant == 28 || variant == kSweepTurnOrdered;
    if (kernel == kKernelBinned)
        return variant == 1 || variant == 2;
    return false;
}

}  // namespace spmvhw

using namespace spmvhw;

spmv_plan::~spmv_plan()
{
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    for (void *ptr : {(void *)d_col, (void *)d_val, (void *)d_rowend, (void *)d_tile_info,
                      (void *)d_row_id, (void *)d_head, (void *)d_tail, (void *)d_cross, (void *)d_s_col,
                      (void *)d_s_row, (void *)d_s_val, (void *)d_panel_row, (void *)d_unit_ent, (void *)d_part, (void *)d_gcount, (void *)d_steal, (void *)d_panel_cnt, (void *)d_unit_panel, (void *)d_panel_unit, (void *)d_rp,
                      (void *)d_s_cbase, (void *)d_s_row16, (void *)d_s_d8, (void *)d_s_dbase, (void *)d_s_side, d_colnar, (void *)d_tile_cbase, (void *)d_kptr, (void *)d_kpos,
                      (void *)d_rp2, (void *)d_rl, (void *)d_chunk_row, (void *)d_bpart, (void *)d_slot_off,
                      (void *)d_sbase, (void *)d_slice_len, (void *)d_b_val, (void *)d_b_colw, (void *)d_b_rowp,
                      d_b_prod_alloc, (void *)d_b_seg, (void *)d_b_seg_hi, (void *)d_b_ub, (void *)d_b_uwin})
        if (ptr)
            (void)hipFree(ptr);
    for (void *ptr : gpart)
        (void)hipFree(ptr);
    for (hipEvent_t e : ev)
        (void)hipEventDestroy(e);
    if (gexec)
        (void)hipGraphExecDestroy(gexec);
    if (gstream)
        (void)hipStreamDestroy(gstream);
    if (gstream2)
        (void)hipStreamDestroy(gstream2);
}

uint64_t spmv_plan::device_bytes() const
{
    if (kernel == kKernelGold || kernel == kKernelFpga)
        return (uint64_t(nr_rows) + 1) * 4 + nnz * (4 + sizeof(ValueType));
    if (kernel == kKernelSlices)  // padded entries, slot bases, slice offsets, row lengths
        return slice_slots * kWave * (sizeof(ValueType) + slice_off_bytes) + slice_slots * (slice_clustered ? 16 : 4) +
               (nslices + 1) * 4 +
               uint64_t(nr_rows) * 4;
    if (kernel == kKernelBlocked)  // entries, kptr, kpos, rl, partials, rp2, chunks, units
        return nnz * (2 + sizeof(ValueType)) + (nkpairs + 1) * 4 + nkpairs * (4 + 2 + sizeof(ValueType)) +
               (uint64_t(nr_rows) + 1) * 4 + (nchunks + 1) * 4 + nunits * 8 + 4;
    if (kernel == kKernelBinned)  // entries (value, 2 offsets), products, segments, units, panels
        return ent_pad * (2 * sizeof(ValueType) + 2 + (b_delta ? 1 : 2)) + (uint64_t(b_nwin) * npanels + 1) * 8 +
               (b_nunits + 1) * 12 + (npanels + 1) * 4;
    if (kernel == kKernelSweep)
        return ent_pad * ((d_s_col ? sizeof(uint32_t) : 0) + (sweep_packed ? 0 : sizeof(uint16_t)) + sizeof(ValueType)) +
               (npanels + 1) * 4 + (nunits + 1) * 4 + (sweep_packed ? ent_pad / kSweepChunk * 4 : 0) +
               (sweep_split > 1 ? nunits * (uint64_t(panel_rmax) + 1) * sweep_acc_bytes : 0) + nunits * 4 + (npanels + 1) * 4 +
               (d_panel_cnt ? npanels * 4 : 0) +
               (sweep_delta ? ent_pad * 3 + ent_pad / kSweepChunk * 4 + sweep_side_chunks * kSweepChunk * 4 : 0);
    return nnz_pad * (tile_col_bytes + sizeof(ValueType)) + nnz_pad / 8 + (ntiles + 1) * 4 +
           (tile_col_bytes < 4 ? ntiles * (tile_clustered ? 16 : 4) : 0) +
           (has_empty ? nzr * 4 : 0) + ntiles * 2 * sizeof(ValueType) + ncross * 12;
}

// z*(sizeof(val)+4) + (n+1)*4 + m*sizeof(val) + n*sizeof(val)
uint64_t spmv_plan::algorithmic_bytes() const
{
    return nnz * (sizeof(ValueType) + 4) + (uint64_t(nr_rows) + 1) * 4 +
           uint64_t(nr_cols) * sizeof(ValueType) + uint64_t(nr_rows) * sizeof(ValueType);
}

extern "C" {

int spmv_plan_create_device(spmv_plan **plan, int device, IndexType nr_rows, IndexType nr_cols,
                            IndexType nr_nzeros, const IndexType *d_row_ptr,
                            const IndexType *d_col_ind, const ValueType *d_values, void *stream)
{
    if (!plan || (nr_rows && !d_row_ptr)) {
        set_error("spmv_plan_create_device: null argument");
        return 1;
    }
    hipStream_t s = (hipStream_t)stream;
    SPMV_TRY(hipSetDevice(device));
    std::vector<IndexType> rp(size_t(nr_rows) + 1, 0u);
    if (nr_rows) {
        SPMV_TRY(hipMemcpyAsync(rp.data(), d_row_ptr, rp.size() * sizeof(IndexType), hipMemcpyDeviceToHost, s));
        SPMV_TRY(hipStreamSynchronize(s));
    }
    const IndexType base = rp[0];
    for (auto &e : rp)
        e -= base;
    if (rp[nr_rows] != nr_nzeros) {
        set_error("spmv_plan_create_device: row_ptr[n]-row_ptr[0] != nr_nzeros");
        return 1;
    }
    return plan_create_from_host_rowptr(plan, device, nr_rows, nr_cols, rp.data(),
                                        d_col_ind ? d_col_ind + base : nullptr,
                                        d_values ? d_values + base : nullptr, true, s);
}

int spmv_plan_create_host(spmv_plan **plan, int device, const csr_matrix *m, IndexType row_begin,
                          IndexType row_end)
{
    if (!plan || !m || row_begin > row_end || row_end > m->nr_rows) {
        set_error("spmv_plan_create_host: bad arguments");
        return 1;
    }
    const IndexType n = row_end - row_begin;
    const IndexType base = m->row_ptr[row_begin];
    std::vector<IndexType> rp(size_t(n) + 1);
    for (IndexType r = 0; r <= n; ++r)
        rp[r] = m->row_ptr[row_begin + r] - base;
    hipStream_t s = nullptr;
    return plan_create_from_host_rowptr(plan, device, n, m->nr_cols, rp.data(), m->col_ind + base,
                                        m->values + base, false, s);
}

// Enqueues one SpMV (memset of y when rows can be empty, main kernel, tile fix-up) on s. Only
// kernels and memsets are enqueued, so the sequence is capturable into a hipGraph.
static int run_impl(spmv_plan *p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool timing)
{
    if (p->nr_rows == 0)
        return 0;
    if (p->kernel == kKernelTiles && (p->has_empty || p->nnz == 0))
        SPMV_TRY(hipMemsetAsync(d_y, 0, size_t(p->nr_rows) * sizeof(ValueType), s));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        if (p->ev_used + 2 > p->ev.size()) {
            for (int i = 0; i < 2; ++i) {
                hipEvent_t e;
                SPMV_TRY(hipEventCreate(&e));
                p->ev.push_back(e);
            }
        }
        e0 = p->ev[p->ev_used];
        e1 = p->ev[p->ev_used + 1];
        p->ev_used += 2;
        SPMV_TRY(hipEventRecord(e0, s));
    }
    if (p->kernel != kKernelTiles) {
        SPMV_TRY(p->kernel == kKernelSweep     ? launch_sweep(*p, d_x, d_y, s)
                 : p->kernel == kKernelBinned  ? launch_binned(*p, d_x, d_y, s)
                 : p->kernel == kKernelBlocked ? launch_blocked(*p, d_x, d_y, s)
                 : p->kernel == kKernelSlices  ? launch_slices(*p, d_x, d_y, s)
                                               : launch_gold(*p, d_x, d_y, s));
        if (timing)
            SPMV_TRY(hipEventRecord(e1, s));
        return 0;
    }
    SPMV_TRY(launch_spmv(*p, d_x, d_y, s));
    if (timing)
        SPMV_TRY(hipEventRecord(e1, s));
    SPMV_TRY(launch_fixup(*p, d_y, s));
    return 0;
}

int spmv_plan_run(const spmv_plan *cp, const ValueType *d_x, ValueType *d_y, void *stream)
{
    if (!cp) {
        set_error("spmv_plan_run: null plan");
        return 1;
    }
    spmv_plan *p = const_cast<spmv_plan *>(cp);
    SPMV_TRY(hipSetDevice(p->device));
    return run_impl(p, d_x, d_y, (hipStream_t)stream, p->timing);
}

// The "dag" form, for split plans whose sweep launch cannot carry the combine (the behind form
// below measured faster; SPMV_GRAPH_FORM=dag forces this one in the tools build): the combine
// of step k runs on a second capture stream beside the
// sweep of step k + 1, the steps' partial sums alternate between two buffers, and the sweep of
// step k + 2 waits for the combine of step k (its buffer). The combine needs no LDS, so its
// workgroups fit beside the sweep's one 1024-thread workgroup per CU. Every step still computes
// all of y = A x; the y of the last step is complete when the graph ends. Not for the tools
// build's stealing variants (the combine re-arms their counters) or the fused combine.
static bool graph_overlaps(const spmv_plan *p)
{
    return p->kernel == kKernelSweep && p->sweep_split > 1 && !p->d_panel_cnt && p->d_part &&
           !(p->sweep_variant >= 37 && p->sweep_variant <= 39);
}

static int graph_part2(spmv_plan *p)
{
    if (p->gpart.empty()) {
        void *b = nullptr;
        SPMV_TRY(hipMalloc(&b, p->nunits * (uint64_t(p->panel_rmax) + 1) * p->sweep_acc_bytes));
        p->gpart.push_back(b);
    }
    return 0;
}

static int capture_overlapped(spmv_plan *p, const ValueType *d_x, ValueType *d_y, int iters)
{
    constexpr int R = 2;  // partial buffers (longer rings measured slower)
    if (graph_part2(p))
        return 1;
    if (!p->gstream2)
        SPMV_TRY(hipStreamCreateWithFlags(&p->gstream2, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * size_t(iters), nullptr);
    auto destroy = [&] {
        for (hipEvent_t e : ev)
            if (e)
                (void)hipEventDestroy(e);
    };
    for (auto &e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            destroy();
            set_error("spmv_plan_run_graph: hipEventCreate failed");
            return 1;
        }
    hipStream_t a = p->gstream, b = p->gstream2;
    hipError_t e = hipStreamBeginCapture(a, hipStreamCaptureModeRelaxed);
    for (int k = 0; k < iters && e == hipSuccess; ++k) {
        void *part = k % R ? p->gpart[k % R - 1] : p->d_part;
        if (k >= R)  // this buffer's previous combine is done
            e = hipStreamWaitEvent(a, ev[2 * (k - R) + 1], 0);
        if (e == hipSuccess)
            e = launch_sweep(*p, d_x, d_y, a, false, 1, part);
        if (e == hipSuccess)
            e = hipEventRecord(ev[2 * k], a);
        if (e == hipSuccess)
            e = hipStreamWaitEvent(b, ev[2 * k], 0);
        if (e == hipSuccess)
            e = launch_sweep(*p, d_x, d_y, b, false, 2, part);
        if (e == hipSuccess)
            e = hipEventRecord(ev[2 * k + 1], b);
    }
    if (e == hipSuccess)  // join: the last combine (the combines are in order on b)
        e = hipStreamWaitEvent(a, ev[2 * (iters - 1) + 1], 0);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(a, &g);
    destroy();
    if (e != hipSuccess || ec != hipSuccess) {
        if (g)
            (void)hipGraphDestroy(g);
        set_error(std::string("spmv_plan_run_graph: overlapped capture: ") +
                  hipGetErrorString(e != hipSuccess ? e : ec));
        return 1;
    }
    const hipError_t ei = hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    SPMV_TRY(ei);
    return 0;
}

// The "behind" form (default for split plans whose sweep can carry it, sweep_behind_ok): one
// stream, one launch per step, and the combine of step k rides in step k + 1's sweep launch as
// extra blocks that start on the CUs no unit holds and in the sweep's tail (sweep.hip,
// combine_behind); a last k_sweep_combine finishes the last step. Partials alternate between
// d_part and gpart[0]. No second stream, so no cross-queue hand-off between the steps.
static int capture_behind(spmv_plan *p, const ValueType *d_x, ValueType *d_y, int iters)
{
    if (graph_part2(p))
        return 1;
    if (!p->d_gcount) {
        SPMV_TRY(hipMalloc(&p->d_gcount, 2 * sizeof(uint32_t)));
        SPMV_TRY(hipMemset(p->d_gcount, 0, 2 * sizeof(uint32_t)));
    }
    int ncu = 0;
    SPMV_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->device));
    auto part_of = [&](int k) { return (k & 1) ? p->gpart[0] : p->d_part; };
    hipStream_t a = p->gstream;
    hipError_t e = hipStreamBeginCapture(a, hipStreamCaptureModeRelaxed);
    for (int k = 0; k < iters && e == hipSuccess; ++k) {
        sweep_behind bh;
        bh.cpart = k ? part_of(k - 1) : nullptr;
        bh.ccount = p->d_gcount + (k & 1);
        bh.cnext = p->d_gcount + ((k + 1) & 1);
        bh.blocks = (uint32_t)std::max(ncu, 1);
        if (const char *v = ablation_env("SPMV_BEHIND_BLOCKS"))  // tools build: measured settings
            bh.blocks = (uint32_t)std::max(1, atoi(v));
        if (const char *v = ablation_env("SPMV_BEHIND_ROWS"))
            bh.rows_per_thread = (uint32_t)std::max(1, atoi(v) / std::max(1, p->sweep_threads));
        e = launch_sweep(*p, d_x, d_y, a, false, 1, part_of(k), &bh);
    }
    if (e == hipSuccess)  // the last step's combine
        e = launch_sweep(*p, d_x, d_y, a, false, 2, part_of(iters - 1));
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(a, &g);
    if (e != hipSuccess || ec != hipSuccess) {
        if (g)
            (void)hipGraphDestroy(g);
        set_error(std::string("spmv_plan_run_graph: behind capture: ") + hipGetErrorString(e != hipSuccess ? e : ec));
        return 1;
    }
    const hipError_t ei = hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    SPMV_TRY(ei);
    return 0;
}

// the capture form of a run_graph: 0 serial chain, 1 two-stream DAG, 2 behind. The tools build's
// SPMV_GRAPH_FORM=serial|dag|behind forces one (where the plan allows it)
static int graph_form(const spmv_plan *p)
{
    const int best = p->kernel == kKernelSweep && sweep_behind_ok(*p) ? 2 : graph_overlaps(p) ? 1 : 0;
    if (const char *f = ablation_env("SPMV_GRAPH_FORM")) {
        const std::string v(f);
        if (v == "serial")
            return 0;
        if (v == "dag" && best >= 1)
            return 1;
    }
    return best;
}

int spmv_plan_run_graph(spmv_plan *p, const ValueType *d_x, ValueType *d_y, int iters, void *stream)
{
    if (!p || iters < 1) {
        set_error("spmv_plan_run_graph: null plan or iters < 1");
        return 1;
    }
    hipStream_t s = (hipStream_t)stream;
    SPMV_TRY(hipSetDevice(p->device));
    if (!p->gexec || p->gx != d_x || p->gy != d_y || p->giters != iters) {
        if (p->gexec) {
            SPMV_TRY(hipGraphExecDestroy(p->gexec));
            p->gexec = nullptr;
        }
        if (!p->gstream)
            SPMV_TRY(hipStreamCreateWithFlags(&p->gstream, hipStreamNonBlocking));
        const int form = iters >= 2 ? graph_form(p) : 0;
        if (form == 2) {
            if (capture_behind(p, d_x, d_y, iters))
                return 1;
        } else if (form == 1) {
            if (capture_overlapped(p, d_x, d_y, iters))
                return 1;
        } else {
            SPMV_TRY(hipStreamBeginCapture(p->gstream, hipStreamCaptureModeRelaxed));
            int rc = 0;
            for (int i = 0; i < iters && !rc; ++i)
                rc = run_impl(p, d_x, d_y, p->gstream, false);
            hipGraph_t g = nullptr;
            const hipError_t ec = hipStreamEndCapture(p->gstream, &g);
            if (rc) {
                if (g)
                    (void)hipGraphDestroy(g);
                return rc;
            }
            SPMV_TRY(ec);
            const hipError_t ei = hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            SPMV_TRY(ei);
        }
        p->gx = d_x;
        p->gy = d_y;
        p->giters = iters;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (p->timing) {
        for (int i = 0; p->ev_used + 2 > p->ev.size() && i < 2; ++i) {
            hipEvent_t e;
            SPMV_TRY(hipEventCreate(&e));
            p->ev.push_back(e);
        }
        e0 = p->ev[p->ev_used];
        e1 = p->ev[p->ev_used + 1];
        p->ev_used += 2;
        SPMV_TRY(hipEventRecord(e0, s));
    }
    SPMV_TRY(hipGraphLaunch(p->gexec, s));
    if (p->timing)
        SPMV_TRY(hipEventRecord(e1, s));
    return 0;
}

int spmv_plan_get_stats(const spmv_plan *p, spmv_plan_stats *st)
{
    if (!p || !st) {
        set_error("spmv_plan_get_stats: null argument");
        return 1;
    }
    std::memset(st, 0, sizeof(*st));
    st->nr_rows = p->nr_rows;
    st->nr_cols = p->nr_cols;
    st->nr_nzeros = p->nnz;
    st->nr_nonempty_rows = p->nzr;
    // work units of the main kernel: tiles, sweep units (panel pieces), or long rows (gold)
    const bool csr = p->kernel == kKernelGold || p->kernel == kKernelFpga;
    st->nr_tiles = (p->kernel == kKernelSweep || p->kernel == kKernelBlocked) ? p->nunits
                   : p->kernel == kKernelBinned                               ? p->npanels
                   : p->kernel == kKernelSlices                               ? p->nslices
                   : csr                                                      ? p->nlong
                                                                              : p->ntiles;
    st->tile_nnz = p->kernel == kKernelSlices   ? p->slice_slots * kWave  // stored entries with padding
                   : p->kernel == kKernelSweep  ? (p->nunits ? p->ent_pad / p->nunits : 0)
                   : p->kernel == kKernelBinned ? (p->npanels ? p->ent_pad / p->npanels : 0)
                   : p->kernel == kKernelBlocked ? (p->nunits ? p->nnz / p->nunits : 0)
                   : csr                         ? (uint64_t)kGoldLong
                                                 : kTileNnz;
    st->device_bytes = p->device_bytes();
    st->algorithmic_bytes = p->algorithmic_bytes();
    st->device = p->device;
    st->kernel = p->kernel;
    st->blocks = p->kernel == kKernelBlocked ? (uint32_t)((uint64_t(p->nr_cols) + p->fpga_width - 1) / p->fpga_width) : 1;
    st->format = (p->kernel == kKernelSlices && p->slice_off_bytes < 4 ? 1 : 0) | (p->slice_clustered ? 16 : 0) |
                 (p->kernel == kKernelSlices && p->slice_off_bytes == 1 ? 8 : 0) | (p->tile_col_bytes < 4 ? 1 : 0) | (p->sweep_packed ? 2 : 0) | (p->sweep_lane_order ? 4 : 0) | (p->sweep_delta ? 64 : 0) |
                 (p->tile_col_bytes == 1 ? 8 : 0) | (p->tile_clustered ? 16 : 0) |
                 (p->kernel == kKernelBinned && p->b_delta ? 32 : 0) |
                 (p->kernel == kKernelSweep && p->sweep_steal &&
                          (p->sweep_variant == 37 || p->sweep_variant == 38 || p->sweep_variant == 39) ? 128 : 0) |
                 (graph_form(p) == 2 ? 256 : graph_form(p) == 1 ? 512 : 0) |
                 (p->kernel == kKernelSweep && p->sweep_split > 1 && p->xbias_split > 0.0 ? 1024 : 0) |
                 (p->kernel == kKernelSweep && p->sweep_split > 1 && p->xbias_split < 0.0 ? 2048 : 0) |
                 (p->kernel == kKernelSweep && p->sweep_wide ? 4096 : 0);
    return 0;
}

int spmv_plan_set_variant(spmv_plan *p, int variant)
{
    if (!p || variant < 0 || (variant > 63 && variant != kSweepTurn && variant != kSweepTurnOrdered)) {
        set_error("spmv_plan_set_variant: bad arguments");
        return 1;
    }
#ifndef SPMV_ABLATIONS
    // The product library takes only what a caller needs (the reference exposes no tuning
    // surface, csr_hw_wrapper.h:9-17): 0 = the plan's default kernel form (the sweep's default is
    // 28, also accepted by number), the sweep's deterministic kernel 94 (bitwise reproducible y,
    // the form of SPMV_SWEEP_DETERMINISTIC=1), and binned 1 / 2 (segment offsets rebased past
    // 2^31 / 2^32: the same y, for the tests of the 64-bit offset path). Every other variant is a
    // performance experiment or an ablation (some give a wrong y by design) and exists only in
    // the tools library built with -DSPMV_ABLATIONS (Makefile target `ablations`).
    if (!product_variant(p->kernel, variant)) {
        set_error("spmv_plan_set_variant: measurement variant (tools library only)");
        return 1;
    }
#endif
    // 0 = the plan's default form in both builds: for a sweep plan that is 28 (the tools
    // library's unpacked measurement form that used to sit at 0 is variant 40)
    if (p->kernel == kKernelSweep && variant == 0)
        variant = 28;
    if (p->kernel == kKernelSweep) {
        // every variant but the default (28), 36 (the same) and the measurement build's stealing
        // variants 37-39 reads the 12-byte rc words, which a delta plan rebuilds on first use
        if ((variant < 36 || variant > 39) && variant != 28 && sweep_materialize_rc(*p))
            return 1;
        p->sweep_variant = variant;
    } else if (p->kernel == kKernelBinned) {
        // 1 / 2 (tests, same y): pass 2 reads segment offsets rebased so that they straddle 2^31 /
        // 2^32 entries (prod and rowp rebased the other way: the same addresses), which drives the
        // 64-bit bound widening after readlane (binned.hip, k_bin_acc) without a 2^31-entry matrix
        // 3-6 (same y): pass-1 cache policy (3: temporal product stores, 4: temporal entry
        // loads, 5: both, 6: non-temporal stores; 0 = the plan's choice); 7 (same y): mirrored
        // products (stored down the array while the entries stream up it); 51 / 52 (tools
        // library): pass-2 ablations, binned.hip
        if (variant > 7 && !(variant >= 51 && variant <= 52)) {
            set_error("spmv_plan_set_variant: binned variants are 0-7");
            return 1;
        }
        if (p->d_b_seg_hi) {
            SPMV_TRY(hipSetDevice(p->device));
            SPMV_TRY(hipFree(p->d_b_seg_hi));
            p->d_b_seg_hi = nullptr;
            p->b_seg_base = 0;
        }
        if (variant == 1 || variant == 2) {
            SPMV_TRY(hipSetDevice(p->device));
            const uint64_t nseg = uint64_t(p->b_nwin) * p->npanels + 1;
            std::vector<uint64_t> h(nseg);
            SPMV_TRY(hipMemcpy(h.data(), p->d_b_seg, nseg * 8, hipMemcpyDeviceToHost));
            const uint64_t base = (variant == 1 ? (1ull << 31) : (1ull << 32)) - h[nseg - 1] / 2;
            for (auto &v : h)
                v += base;
            SPMV_TRY(hipMalloc((void **)&p->d_b_seg_hi, nseg * 8));
            SPMV_TRY(hipMemcpy(p->d_b_seg_hi, h.data(), nseg * 8, hipMemcpyHostToDevice));
            p->b_seg_base = base;
        }
        p->variant = variant;
    } else {
        p->variant = variant & 3;
    }
    // a graph captured with the previous variant must not be replayed
    if (p->gexec) {
        (void)hipSetDevice(p->device);
        (void)hipGraphExecDestroy(p->gexec);
        p->gexec = nullptr;
    }
    return 0;
}

int spmv_plan_set_timing(spmv_plan *p, int enable)
{
    if (!p) {
        set_error("spmv_plan_set_timing: null plan");
        return 1;
    }
    p->timing = enable != 0;
    p->ev_used = 0;
    return 0;
}

int spmv_plan_get_timing(spmv_plan *p, double *mean_ms, double *total_ms, int *launches)
{
    if (!p) {
        set_error("spmv_plan_get_timing: null plan");
        return 1;
    }
    SPMV_TRY(hipSetDevice(p->device));
    double tot = 0.0;
    int n = 0;
    for (size_t i = 0; i + 1 < p->ev_used; i += 2) {
        SPMV_TRY(hipEventSynchronize(p->ev[i + 1]));
        float ms = 0.f;
        SPMV_TRY(hipEventElapsedTime(&ms, p->ev[i], p->ev[i + 1]));
        tot += ms;
        ++n;
    }
    p->ev_used = 0;
    if (mean_ms)
        *mean_ms = n ? tot / n : 0.0;
    if (total_ms)
        *total_ms = tot;
    if (launches)
        *launches = n;
    return 0;
}

void spmv_plan_destroy(spmv_plan *p) { delete p; }

}  // extern "C"
