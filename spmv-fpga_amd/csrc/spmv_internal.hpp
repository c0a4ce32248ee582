// Internal declarations of libspmv_hw (not part of the C-ABI).
//
// The MI355X hw representation of one unit's row slice ("plan"), DESIGN.md §3:
//   col      u32[nnz_pad]   column index of every stored non-zero, CSR order
//   val      V[nnz_pad]     values; fp64 is pair-interleaved inside each 256-entry wave step so
//                           that every lane's 4 consecutive entries arrive by two fully coalesced
//                           1-KiB dwordx4 wave loads (fp32 keeps CSR order: one dwordx4)
//   rowend   u32[nnz_pad/32] bit k set <=> entry k is the last entry of its row. This is the
//                           reference's "last element of row" flag (csr_hw.cpp:288-292, bit 15 of
//                           each 16-bit column field) moved to a bitmap: 1 bit/nnz instead of 16.
//   tile_info u32[ntiles+1]  (compact row index of the tile's first entry << 1) | (1 if that
//                           entry continues a row begun in an earlier tile)
//   row_id   u32[nzr]       slice row of each non-empty row; absent when no row is empty. This
//                           replaces the reference's empty_rows_bitmap scatter
//                           (csr_hw.cpp:1531-1565) with an index map.
// Entries past nnz (padding to a whole tile) have col 0, value 0 and no row-end bit.
// Narrow form (default when every tile's columns span < 65536, e.g. banded matrices): col is
// replaced by colnar u16[nnz_pad] (u8 when every span < 256) = col - tile_cbase[tile] and
// tile_cbase u32[ntiles], i.e. the reference's block-relative 16-bit column field
// (csr_hw.cpp:288-292) with a per-tile block base: 10 (9) B/nnz fp64 and 6 (5) B/nnz fp32 are
// streamed instead of 12 and 8.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "csr_hw_wrapper.h"
#include "spmv_host.hpp"

namespace spmvhw {

constexpr int kWave = 64;
constexpr int kLaneEntries = 4;                    // entries per lane per wave step
constexpr int kStep = kWave * kLaneEntries;        // 256 entries per wave step
constexpr int kTileSteps = 2;                      // wave steps per tile
constexpr int kTileNnz = kStep * kTileSteps;       // 512 entries per wave tile
constexpr int kBlockThreads = 256;                 // 4 waves = 4 tiles per workgroup
constexpr int kSweepThreads = 1024;                // default panel-sweep workgroup (16 waves, 1/CU)
constexpr uint64_t kSweepLdsBytes = 160 * 1024;    // LDS of one CU holds the panel's y
constexpr uint64_t kSweepChunk = 128;              // entries per packed chunk (one wave, 2 per lane)
constexpr int kSweepTurn = 91;         // sweep variant: ordered LDS adds (deterministic y), the
constexpr int kSweepTurnOrdered = 94;  // form of SPMV_SWEEP_DETERMINISTIC=1; 94: adds awaited

// plan kernels (spmv_plan_stats.kernel)
constexpr int kKernelTiles = 0;  // flagged-tile wave kernel, x gathered through the caches
constexpr int kKernelGold = 1;   // spmv_gold's exact order (bitwise reference results)
constexpr int kKernelSweep = 2;  // panel sweep: y in LDS, columns swept in order (x from L2)
constexpr int kKernelFpga = 3;   // the reference FPGA path's order for (VF, block width), bitwise
constexpr int kKernelBlocked = 4;  // the same order by the reference's dataflow: x blocks in LDS,
                                   // per-block partials, block-ordered merge (blocked.hip)
constexpr int kKernelSlices = 5;   // wave per 64 rows, entries slot-major (slices.hip)
constexpr int kKernelBinned = 6;   // two passes: products per column window, summed per row panel
                                   // (propagation blocking, binned.hip)
constexpr int kGoldLong = 128;   // gold plan stats: rows longer than this count as long

// 64-lane inclusive prefix sum (the GCN DPP sequence: row_shr 1/2/3 of the source, row_shr 4/8
// with bank masks, row_bcast 15/31 with row masks); tools/delta_probe.hip checks it. Used by the
// binned kernel's row deltas and the sweep's column deltas.
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v0)
{
    uint32_t v = v0;
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x113, 0xf, 0xf, true);  // row_shr:3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xe, true);   // row_shr:4, banks 1-3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xc, true);   // row_shr:8, banks 2-3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15, rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31, rows 2, 3
    return v;
}

}  // namespace spmvhw

struct spmv_plan {
    int device = 0;
    IndexType nr_rows = 0, nr_cols = 0;
    uint64_t nnz = 0, nnz_pad = 0;
    uint64_t nzr = 0;          // non-empty rows
    uint64_t ntiles = 0;
    bool has_empty = false;
    int kernel = 0;
    int variant = 0;           // tile-kernel variant bits (spmv_plan_set_variant)
    int sweep_variant = 28;    // sweep-kernel variant bits (spmv_plan_set_variant, kernel 2)

    uint32_t *d_col = nullptr;
    void *d_colnar = nullptr;        // narrow form: u16 or u8 offsets from tile_cbase (d_col freed)
    uint32_t *d_tile_cbase = nullptr;
    int tile_col_bytes = 4;          // 4 (d_col), 2 or 1 (d_colnar)
    bool tile_clustered = false;     // 2-byte columns as (cluster << 14) | offset, 4 bases per tile
    bool tile_xcd = false;           // XCD-contiguous tile order (env SPMV_TILE_XCD=1); measured
                                     // slower on stencils (+6 %), 2 % faster on banded
    ValueType *d_val = nullptr;
    uint32_t *d_rowend = nullptr;
    uint32_t *d_tile_info = nullptr;
    uint32_t *d_row_id = nullptr;
    ValueType *d_head = nullptr;
    ValueType *d_tail = nullptr;
    uint32_t *d_cross = nullptr;   // rows crossing tile boundaries: (row, first tile, last tile)
    uint64_t ncross = 0;

    // gold-order representation (kernel 1, gold.hip): plain CSR in d_rp / d_col / d_val
    uint32_t *d_rp = nullptr;         // rebased row_ptr[nr_rows + 1]
    uint64_t nlong = 0;               // rows with more than kGoldLong entries (stats)
    int fpga_vf = 1;                  // kernel 3: vectorisation factor (env SPMV_FPGA_VF)
    uint32_t fpga_width = 32768;      // kernel 3: column-block width (env SPMV_FPGA_BLOCK)

    // blocked representation (kernel 4, blocked.hip): entries by (block, row) in d_val (values)
    // and d_colnar (u16 block-relative columns); units in d_unit_panel (block) / d_unit_ent
    // (compact-row ranges)
    uint32_t *d_kptr = nullptr;       // first entry of each compact row [nkpairs + 1]
    uint32_t *d_kpos = nullptr;       // partial slot of each compact row
    uint32_t *d_rp2 = nullptr;        // row-major offsets of each row's partials [nr_rows + 1]
    uint16_t *d_rl = nullptr;         // row-major: chunk-local slot of each partial
    uint32_t *d_chunk_row = nullptr;  // row ranges of the merge chunks [nchunks + 1]
    ValueType *d_bpart = nullptr;     // block partials (scratch)
    uint64_t nkpairs = 0, nchunks = 0;
    bool blocked_xlds = false;        // x block staged in LDS (W * sizeof(V) <= 128 KiB)

    // slice representation (kernel 5, slices.hip): slot-major entries in d_val / d_colnar
    uint32_t *d_slot_off = nullptr;   // slots of each 64-row slice [nslices + 1]
    uint32_t *d_sbase = nullptr;      // base column of each slot
    uint32_t *d_slice_len = nullptr;  // row lengths
    uint64_t nslices = 0, slice_slots = 0;
    int slice_off_bytes = 4;          // 1, 2 (offsets from the slot base) or 4 (absolute columns)
    bool slice_clustered = false;     // 2-byte offsets as (cluster << 14) | offset, 4 bases per slot
    bool slice_acc_native = false;    // fp32 library: accumulate in fp32 (env SPMV_SLICE_ACC=32)
    double slice_pad_limit = 0.0;     // automatic choice: give up when stored / real entries exceeds it

    // panel-sweep representation (kernel 2, sweep.hip)
    uint64_t npanels = 0, ent_pad = 0;
    uint64_t nunits = 0;               // workgroups of a launch = npanels * sweep_split
    uint32_t sweep_split = 1;          // > 1: some panel is cut into pieces (partials + combine)
    uint32_t *d_unit_panel = nullptr;  // panel of each work unit
    uint32_t *d_panel_unit = nullptr;  // first unit of each panel [npanels + 1]
    void *d_part = nullptr;            // split > 1: nunits x (panel_rmax + 1) partial sums (accumulator type)
    std::vector<void *> gpart;         // spmv_plan_run_graph: a second partial buffer beside d_part, so
                                       // that step k + 1's sweep can run while step k's partials wait
                                       // for their combine
    uint32_t *d_gcount = nullptr;      // spmv_plan_run_graph, "behind" form: two chunk counters
    double xbias_split = 0.0;          // the pieces' XCC bias in use (split plans; env SPMV_SWEEP_XCC_BIAS)
    unsigned long long *d_steal = nullptr;  // tools build, split > 1: per unit, iterations claimed
                                            // from the front (low word) and back (high word) by the
                                            // work-stealing variants 37-39; re-armed by k_sweep_combine
    bool sweep_steal = false;          // the stealing variants can run on this plan (tools build)
    uint32_t *d_panel_cnt = nullptr;   // split > 1 with env SPMV_SWEEP_COMBINE=fused: per-panel count of
                                       // finished pieces (the last one combines, sweep.hip
                                       // write_panel); null (default): k_sweep_combine
    int sweep_acc_bytes = 8;           // LDS accumulator: 8 (fp64) or 4 (fp32 via CAS, env SPMV_SWEEP_ACC=32)
    uint32_t panel_rmax = 0;
    int sweep_threads = spmvhw::kSweepThreads;  // workgroup size: 1024, 512 or 256 (env SPMV_SWEEP_THREADS)
    uint32_t *d_s_col = nullptr;
    uint16_t *d_s_row = nullptr;
    ValueType *d_s_val = nullptr;
    uint32_t *d_panel_row = nullptr;
    uint32_t *d_unit_ent = nullptr;
    uint32_t *d_s_cbase = nullptr;   // packed form: base column per 128-entry chunk
    bool sweep_packed = false;
    bool sweep_lane_order = false;   // packed chunks stored in lane order (k_sweep_lane_order)
    bool sweep_det = false;          // env SPMV_SWEEP_DETERMINISTIC=1: ordered LDS adds (k_spmv_sweep_turn)
    // delta-coded columns (default for packed lane-ordered plans, env SPMV_SWEEP_DELTA=0 off): the
    // default kernel streams 11 B/entry fp64 (7 fp32) instead of 12 (8); the 12-byte rc words
    // (d_s_col) are freed and rebuilt on demand for the kernels that read them
    // (sweep_materialize_rc: deterministic variants, variant 35, ablations)
    uint16_t *d_s_row16 = nullptr;   // row in panel per entry (bits 0-14) + bit 8 of its delta (lane order)
    uint8_t *d_s_d8 = nullptr;       // low 8 bits of the column minus the previous entry's column of
                                     // the same wave instruction (the first from the chunk base)
    uint32_t *d_s_dbase = nullptr;   // per chunk: base column, or bit 31 | index into d_s_side
    uint32_t *d_s_side = nullptr;    // absolute columns (lane order) of chunks with a gap > 511
    uint64_t sweep_side_chunks = 0;
    bool sweep_delta = false;
    bool sweep_wide = false;         // some chunks span >= 65536 columns: their columns live only in
                                     // the side table (delta plans; no 12-byte rc words can be rebuilt)
    // binned representation (kernel 6, binned.hip): reuses npanels, panel_rmax, d_panel_row and
    // ent_pad of the sweep fields; entries ordered (window, panel), segments padded
    uint32_t b_nwin = 0, b_W = 0;      // column windows of b_W columns (x staged in LDS by pass 1)
    uint32_t b_W1 = 0;                 // width of the odd windows (b_W: the even ones; XCC bias)
    uint64_t b_nunits = 0;             // pass-1 work units
    ValueType *d_b_val = nullptr;
    uint16_t *d_b_colw = nullptr;      // column - window base
    void *d_b_rowp = nullptr;          // u16 row - panel base, or (b_delta) u8 row deltas
    bool b_delta = false;              // segments sorted by row, 1-byte deltas (binned.hip)
    bool b_prod_temporal = false;      // pass 1 stores the products with the default cache policy
                                       // (they stay partly in MALL for pass 2): products <= 1 GiB
    ValueType *d_b_prod = nullptr;     // products, written by pass 1 and read by pass 2
    void *d_b_prod_alloc = nullptr;    // its allocation (d_b_prod may start past its base)
    uint64_t *d_b_seg = nullptr;       // padded segment offsets [b_nwin * npanels + 1]
    uint64_t *d_b_seg_hi = nullptr;    // variants 1 / 2 (tests): d_b_seg + b_seg_base, read by pass 2
    uint64_t b_seg_base = 0;           // with prod / rowp rebased by -b_seg_base (same addresses)
    uint64_t *d_b_ub = nullptr;        // pass-1 unit boundaries [b_nunits + 1]
    uint32_t *d_b_uwin = nullptr;      // window of each pass-1 unit
    double bin_skew_limit = 0.0;       // automatic choice: give up (rc 2) when a panel holds more than
                                       // this many times the mean entries (long rows: pass 2 would
                                       // serialise their LDS adds on one address)
    double bin_row_limit = 0.0;        // automatic choice: give up (rc 2) when one row holds more than
                                       // this fraction of a panel's mean entries (same reason; env
                                       // SPMV_BIN_ROW_LIMIT overrides the automatic value)
    // spmv_hw's streamed copy-back (csr_hw_wrapper.cpp): while set, the sweep kernel stores
    // y_epoch into y_flag[panel] (host memory) once the panel's rows of y are in memory
    uint32_t *y_flag = nullptr;
    uint32_t y_epoch = 0;
    ValueType *y_host = nullptr;  // (tools build, SPMV_HW_DIRECT=1) the sweep stores y here instead
                                  // of d_y: mapped pinned host memory
    double locality = -1.0;    // probe result used by the automatic kernel choice
    double tuned_ms[4] = {-1.0, -1.0, -1.0, -1.0};  // SPMV_HW_KERNEL=tune: tiles / sweep / slices / binned ms

    // timing (HIP events around the main kernel, on the launch stream)
    bool timing = false;
    std::vector<hipEvent_t> ev;   // pairs
    size_t ev_used = 0;

    // spmv_plan_run_graph: `giters` SpMVs on (gx, gy) captured once, replayed per call
    hipGraphExec_t gexec = nullptr;
    hipStream_t gstream = nullptr;
    hipStream_t gstream2 = nullptr;  // second capture stream (the tools build's "dag" form: the combines)
    const ValueType *gx = nullptr;
    ValueType *gy = nullptr;
    int giters = 0;

    uint64_t device_bytes() const;
    uint64_t algorithmic_bytes() const;
    ~spmv_plan();  // frees every device buffer and event (also on error paths)
};

namespace spmvhw {

// Launch, or (warm) only have the runtime load the kernel's code object: plan creation runs the
// launchers warm so that the first SpMV of a plan does not pay the lazy module load (~8 ms).
template <typename K, typename... Args>
inline void launch_or_warm(bool warm, K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args)
{
    if (warm) {
        hipFuncAttributes a;
        (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(kernel));
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}

// kernels.hip
hipError_t launch_spmv(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false);
hipError_t launch_fixup(const spmv_plan &p, ValueType *d_y, hipStream_t s, bool warm = false);
hipError_t launch_pack(const IndexType *d_col_src, const ValueType *d_val_src, uint64_t nnz,
                       uint64_t nnz_pad, uint32_t ncols, uint32_t *d_col, ValueType *d_val,
                       uint32_t *d_bad, hipStream_t s);
hipError_t launch_validate(const IndexType *d_col, uint64_t nnz, uint32_t ncols, uint32_t *d_bad, hipStream_t s);
// tile column bases (min column of each tile's real entries); *d_maxspan = max over tiles of
// (max column - min column)
hipError_t launch_tile_span(const uint32_t *d_col, uint64_t nnz, uint64_t ntiles, uint32_t *d_cbase,
                            uint32_t *d_maxspan, hipStream_t s);
// up to 4 cluster bases per tile (bases u32[4 ntiles]); *d_bad |= 1 when a tile needs more
hipError_t launch_tile_clusters(const uint32_t *d_col, uint64_t nnz, uint64_t ntiles, uint32_t *d_bases,
                                uint32_t *d_bad, hipStream_t s);
hipError_t launch_cluster_encode(const uint32_t *d_col, uint64_t nnz, uint64_t nnz_pad, const uint32_t *d_bases,
                                 uint16_t *d_out, hipStream_t s);
// col - cbase[tile] as `bytes`-wide offsets (2 or 1)
hipError_t launch_narrow(const uint32_t *d_col, uint64_t nnz, uint64_t nnz_pad, const uint32_t *d_cbase,
                         void *d_out, int bytes, hipStream_t s);

// gold.hip
hipError_t launch_gold(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false);

// blocked.hip
hipError_t launch_blocked(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false);
int build_blocked(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                  hipStream_t s);

// slices.hip
hipError_t launch_slices(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false);
int build_slices(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                 hipStream_t s);

// binned.hip
hipError_t launch_binned(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false);
// 0 ok, 1 error, 2 the segment table would be too large (caller may use another kernel)
int build_binned(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                 hipStream_t s);

// sweep.hip
// phase 0: the sweep and (split plans) the combine; 1: the sweep only; 2: the combine only.
// part: the partial-sum buffer of a split plan (null: the plan's own d_part)
// behind: (spmv_plan_run_graph of a split plan) the previous step's combine, run by extra blocks
// of this sweep launch (sweep.hip, combine_behind); only where sweep_behind_ok
struct sweep_behind {
    const void *cpart = nullptr;  // the previous step's partial sums (null: nothing to combine)
    uint32_t *ccount = nullptr;   // this launch's chunk counter (zero when it starts)
    uint32_t *cnext = nullptr;    // zeroed by this launch: the next launch's counter
    uint32_t blocks = 0;          // extra blocks when cpart is set
    uint32_t rows_per_thread = 4; // a chunk is rows_per_thread x block rows (2, 4 or 8)
};
hipError_t launch_sweep(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm = false,
                        int phase = 0, void *part = nullptr, const sweep_behind *behind = nullptr);
bool sweep_behind_ok(const spmv_plan &p);  // the plan's sweep launch can carry a combine behind
bool product_variant(int kernel, int variant);  // spmv_plan_set_variant: accepted by the product library
// 0 ok, 1 error, 2 the padded layout would overflow 32-bit entry offsets (caller may use tiles)
int build_sweep(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                hipStream_t s);
int probe_locality(const IndexType *d_rp, const IndexType *d_col, IndexType n, hipStream_t s, double *frac);
int sweep_materialize_rc(spmv_plan &p);  // delta plan: rebuild the 12-byte rc words (once)
// the plan's default launch is the packed sweep with one workgroup per panel (no combine), whose
// workgroups can flag each panel's y as it is stored (spmv_plan::y_flag)
bool sweep_can_flag_panels(const spmv_plan &p);

// plan.cpp helpers shared with the wrapper
int upload_staged(void *dst, const void *src, size_t bytes, hipStream_t s);  // pageable H2D, synchronous
int plan_create_from_host_rowptr(spmv_plan **out, int device, IndexType nr_rows, IndexType nr_cols,
                                 const IndexType *h_row_ptr /* rebased, nr_rows+1 */,
                                 const IndexType *col_src, const ValueType *val_src,
                                 bool src_on_device, hipStream_t s);

// mgpu.cpp helpers for spmv_hw's RCCL merge (csr_hw_wrapper.cpp): a clique over n distinct
// devices (one rank each, ncclCommInitAll) that borrows the units' plans and takes each device's
// x per run; y of a gather / reduce lands in rank 0's full-length buffer
int mgpu_create_borrowed(spmv_mgpu **out, int n, const int *devices, const IndexType *bounds, IndexType nr_cols,
                         const spmv_plan *const *plans);
int mgpu_run_on(spmv_mgpu *mg, int exchange, const ValueType *const *x_dev);
const ValueType *mgpu_root_y(const spmv_mgpu *mg);
int mgpu_rccl_calls(const spmv_mgpu *mg);  // RCCL calls per step of the last run (run, _pipelined, _graph)
}  // namespace spmvhw

#define SPMV_TRY(expr)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            spmvhw::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));             \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)
