/*
 * csr_hw_wrapper.h — C-ABI of libspmv_hw_{f64,f32}.so, the MI355X drop-in for the reference's
 * FPGA path (csr_hw_wrapper.cpp + csr_hw.cpp + spmv.cpp of euroexa/spmv-fpga).
 *
 * Part 1 — the reference API, same names / argument meaning / ownership
 * -------------------------------------------------------------------
 *   create_csr_hw_matrix     replaces csr_hw_wrapper.h:9,   csr_hw_wrapper.cpp:3-80
 *   create_csr_hw_y_vector   replaces csr_hw_wrapper.h:10,  csr_hw_wrapper.cpp:82-185
 *   create_csr_hw_x_vector   replaces csr_hw_wrapper.h:11,  csr_hw_wrapper.cpp:187-191
 *   spmv_hw                  replaces csr_hw_wrapper.h:13,  csr_hw_wrapper.cpp:193-288
 *   delete_csr_hw_matrix     replaces csr_hw_wrapper.h:15,  csr_hw_wrapper.cpp:291-296
 *   delete_csr_hw_y_vector   replaces csr_hw_wrapper.h:16,  csr_hw_wrapper.cpp:298-303
 *   delete_csr_hw_x_vector   replaces csr_hw_wrapper.h:17,  csr_hw_wrapper.cpp:305-308
 *   storage_overhead         replaces csr_hw.h:140,         csr_hw.cpp:1401-1409
 *   verification             replaces csr_hw.h:148,         csr_hw.cpp:1571-1590
 *
 * Semantics kept from the reference:
 *   - *hw_matrix is a malloc'd array of spmv_hw_units() handles ("ComputeUnits", util.h:41-59),
 *     one per unit; each handle's public fields are valid host memory (main.cpp:69,86-87).
 *   - *empty_rows_bitmap is malloc'd; the caller frees ONLY the outer array (main.cpp:95). Here
 *     the inner rows live inside the same allocation, so that free() releases everything.
 *   - spmv_hw is synchronous and ACCUMULATES (+=) into y_fpga->values (csr_hw.cpp:1555,
 *     main.cpp:74 hands in a zeroed vector). It prints the same three timing lines
 *     (csr_hw_wrapper.cpp:274,284-285).
 *   - verification: absolute threshold 1e-5, NaN counts as an error (csr_hw.cpp:1573-1580).
 *   - storage_overhead: MB of one unit's hw representation; computed in 64 bits (the reference
 *     sums in 32-bit IndexType and overflows past 512 MB).
 * Error behaviour: the reference has no error channel (all void, nothing checked). This library
 * fails fast: a HIP error or invalid input prints "spmv_hw: <what>" to stderr and exit(1)s, for
 * the Part-1 API. Part 2 returns error codes instead and records spmv_hw_last_error().
 *
 * Part 2 — device-resident extensions (used by bench.py, the tests and multi-process runs)
 * -------------------------------------------------------------------------------------
 *   A spmv_plan is ONE unit's matrix slice in the MI355X hw representation.
 *   Pointers named d_* are device addresses on the plan's device; `stream` is a hipStream_t
 *   (NULL = default stream). All Part-2 calls return 0 on success, nonzero on error.
 */
#ifndef CSR_HW_WRAPPER_H
#define CSR_HW_WRAPPER_H

#include "spmv_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- Part 1: reference API ---------------- */
void create_csr_hw_matrix(csr_matrix *matrix, csr_hw_matrix ***hw_matrix, bool ***empty_rows_bitmap);
void create_csr_hw_y_vector(csr_hw_matrix **hw_matrix, csr_hw_vector ***hw_vector);
void create_csr_hw_x_vector(csr_hw_vector **hw_x, csr_vector *x, int blocks, IndexType *nr_cols);
void spmv_hw(csr_hw_matrix **hw_matrix, csr_hw_vector *hw_x, csr_vector *y_fpga, bool **empty_rows_bitmap);
void delete_csr_hw_matrix(csr_hw_matrix **hw_matrix);
void delete_csr_hw_y_vector(csr_hw_vector **hw_vector);
void delete_csr_hw_x_vector(csr_hw_vector *hw_vector);
ValueType storage_overhead(csr_hw_matrix *matrix);
/* nr_values is a plain 32-bit count at the C-ABI (the reference's IndexType is ap_uint<32>, the
 * same 4 bytes; a caller-typed overload follows below for SPMV_USE_CALLER_CSR_TYPES builds) */
int verification(uint32_t nr_values, ValueType *sw_values, ValueType *hw_values, int verbose);

/* ---------------- Part 2: extensions ---------------- */

/* Number of units ("ComputeUnits"): the last spmv_hw_set_units() value, else env SPMV_NGPUS
 * (default 1). Unit u runs on HIP device (u % device_count); more units than devices gives
 * virtual units sharing a GPU. create_csr_hw_matrix's *hw_matrix always holds at least 12 + 1
 * slots (the reference's largest CU build, util.h:41-59) with the unused ones NULL, so a loop
 * over a compile-time ComputeUnits (main.cpp:86-87) never reads past the array. */
int spmv_hw_units(void);
/* Set the unit count from the caller's compile-time CU (include/dropin/csr_hw_wrapper.h does
 * this before main() when util.h defines ComputeUnits); 0 returns to env SPMV_NGPUS. Returns the
 * previous setting. */
int spmv_hw_set_units(int units);
/* Bytes of sizeof(ValueType) this library was built for (8 = DOUBLE=1, 4 = DOUBLE=0). */
int spmv_hw_value_bytes(void);
/* Last error message of a Part-2 call on this thread ("" if none). */
const char *spmv_hw_last_error(void);

typedef struct spmv_plan spmv_plan;

typedef struct spmv_plan_stats {
    uint64_t nr_rows;            /* rows of the slice */
    uint64_t nr_cols;            /* columns (length of x) */
    uint64_t nr_nzeros;          /* stored non-zeros */
    uint64_t nr_nonempty_rows;   /* rows with >= 1 non-zero */
    uint64_t nr_tiles;           /* work units of the main kernel: wave tiles (0), long rows (1, 3),
                                    panel pieces (2), phase-1 units (4), 64-row slices (5),
                                    row panels of pass 2 (6) */
    uint64_t tile_nnz;           /* non-zeros per unit (kernel 5: stored entries with padding) */
    uint64_t device_bytes;       /* bytes of the hw representation resident in HBM */
    uint64_t algorithmic_bytes;  /* compulsory CSR bytes per SpMV, SURVEY.md §8(d) */
    int32_t device;              /* HIP device ordinal */
    int32_t kernel;              /* 0 = flagged-tile gather, 1 = spmv_gold order (bitwise), 2 = panel
                                    sweep, 3 = the reference FPGA path's order for env
                                    SPMV_FPGA_VF / SPMV_FPGA_BLOCK (bitwise), 4 = the same order
                                    by the reference's column-blocked dataflow (x blocks in LDS),
                                    5 = slices (wave per 64 rows, slot-major; DESIGN.md §3-4;
                                    fp64: bitwise spmv_gold; fp32 too with env SPMV_SLICE_ACC=32),
                                    6 = binned (two passes: products per column window, summed
                                    per row panel in LDS; binned.hip).
                                    Chosen automatically (0, 2, 5, or 6 for large scattered fp32
                                    matrices), or by env SPMV_HW_KERNEL = tiles | gold | sweep |
                                    fpga | blocked | slices | binned | tune (build
                                    tiles, sweep, slices and binned, time them on the matrix, keep the
                                    fastest) */
    int32_t blocks;              /* column blocks of the representation (kernel 4; 1 otherwise) */
    int32_t format;              /* bit 0: 16- or 8-bit column offsets (per tile, kernel 0; per
                                    slot, kernel 5), bit 3: 8-bit, bit 4: 16-bit (cluster, offset)
                                    with 4 bases per tile / slot; bit 1: packed 12/8-byte sweep
                                    entries; bit 2: lane-ordered chunks (kernel 2); bit 5: row-
                                    sorted segments with 1-byte row deltas (kernel 6); bit 6:
                                    delta-coded columns, 11-byte fp64 / 7-byte fp32 sweep entries
                                    (kernel 2); bit 7: the tools library's work-stealing
                                    variants 37-39 are selected (kernel 2, split plans); bit 8:
                                    spmv_plan_run_graph pipelines the steps, each step's combine
                                    behind the next sweep launch; bit 9: the same with the
                                    combines on a second stream (split plans, 2+ steps);
                                    bits 10 / 11: the pieces of a split sweep plan are cut with
                                    the even / the odd XCCs' units lighter (env
                                    SPMV_SWEEP_XCC_BIAS > 0 / < 0; the default cuts them evenly,
                                    so a plan's layout depends only on the matrix and the chip);
                                    bit 12: some 128-entry chunks span >= 65536 columns and keep
                                    their absolute columns in the side table (kernel 2, delta
                                    entries; variants reading 12-byte entries are refused) */
} spmv_plan_stats;

/* Build a plan from a device-resident CSR slice (row_ptr may start at any offset: entries are
 * rebased to d_row_ptr[0]). The CSR arrays are only read; the plan owns its own copies. */
int spmv_plan_create_device(spmv_plan **plan, int device, uint32_t nr_rows, uint32_t nr_cols,
                            uint32_t nr_nzeros, const IndexType *d_row_ptr,
                            const IndexType *d_col_ind, const ValueType *d_values, void *stream);
/* Build a plan from rows [row_begin, row_end) of a host CSR matrix. */
int spmv_plan_create_host(spmv_plan **plan, int device, const csr_matrix *matrix,
                          uint32_t row_begin, uint32_t row_end);
/* d_y[0:nr_rows) = A * d_x  (overwrite; empty rows get 0). Asynchronous on `stream`. Enqueues
 * only kernels and memsets (when timing is off), so callers may capture it into their own
 * hipGraph, e.g. an iterative solver's SpMV + update + RCCL all-gather step.
 * The split sweep's partial sums and the binned kernel's products live in plan-owned scratch:
 * runs of ONE plan must be ordered (same stream, or events between streams); distinct plans
 * may run concurrently. */
int spmv_plan_run(const spmv_plan *plan, const ValueType *d_x, ValueType *d_y, void *stream);
/* Iterative / persistent mode: `iters` consecutive SpMVs d_y = A * d_x, captured once into a
 * hipGraph (re-captured when d_x, d_y or iters change) and replayed on `stream` per call, so
 * back-to-back SpMVs pay no per-launch host cost. With timing on, one event pair brackets the
 * whole graph (spmv_plan_get_timing then reports ms per graph). The SpMVs of one replay are
 * independent (same x), so a split sweep plan pipelines them: step k's partial sums are added by
 * extra blocks of step k + 1's sweep launch, and a last combine kernel ends the graph (the first
 * capture allocates a second partial-sum buffer for this). d_y is complete when the graph
 * has run. */
int spmv_plan_run_graph(spmv_plan *plan, const ValueType *d_x, ValueType *d_y, int iters, void *stream);
int spmv_plan_get_stats(const spmv_plan *plan, spmv_plan_stats *stats);
/* Kernel variants. The product library accepts: 0 = the plan's default kernel form (every
 * kernel; for the sweep the same as 28), sweep 94 = the deterministic kernel of
 * SPMV_SWEEP_DETERMINISTIC=1 on any sweep plan (LDS adds in a fixed order, bitwise reproducible
 * y), and binned (kernel 6) 1 / 2 = segment offsets rebased past 2^31 / 2^32 (the same y; the
 * tests' handle on the 64-bit offset path). Any other variant returns an error ("tools library
 * only"): the performance experiments (sweep 15-35 and 91, the unpacked sweep's forms, tile and
 * slice load/store forms, binned cache policies 3-7) and the measurement-only ablations (some
 * give a wrong y by design) are built only into the tools library (-DSPMV_ABLATIONS, Makefile
 * target `ablations`). The reference exposes no tuning surface (csr_hw_wrapper.h:9-17). */
int spmv_plan_set_variant(spmv_plan *plan, int variant);
/* Per-plan kernel timing with HIP events recorded around the main kernel on the launch
 * stream: enable, then read back the mean duration (ms) and count of timed launches. */
int spmv_plan_set_timing(spmv_plan *plan, int enable);
int spmv_plan_get_timing(spmv_plan *plan, double *mean_ms, double *total_ms, int *launches);
void spmv_plan_destroy(spmv_plan *plan);

/* nnz-balanced contiguous row partition into `units` slices: bounds[0]=0, bounds[units]=nr_rows,
 * slice u = rows [bounds[u], bounds[u+1]) with ~nnz/units non-zeros each (the
 * reference's S1 rule, csr_hw.cpp:459, without the FPGA alignment rules S2/S3). Host only. */
int spmv_partition_rows(const IndexType *row_ptr, uint32_t nr_rows, int units, IndexType *bounds);

/* ---------------- Part 4: one process, several GPUs, RCCL exchange ----------
 * A spmv_mgpu splits a host CSR matrix into nnz-balanced row slices, one per device (the
 * per-CU split of prepare_balanced_hw_matrix, csr_hw.cpp:459-468), builds a plan per device,
 * replicates x by an RCCL broadcast (x per CU, spmv.cpp:280-294) and exchanges y over xGMI with
 * RCCL instead of merging on the host (accum_results, csr_hw.cpp:1531-1565;
 * csr_hw_wrapper.cpp:276-281). One RCCL clique (ncclCommInitAll) over `devices` (NULL = 0..ndev-1,
 * each at most once); RCCL is loaded at run time (librccl.so.1). All calls are synchronous and
 * return 0 on success (spmv_hw_last_error() otherwise). */
typedef struct spmv_mgpu spmv_mgpu;
#define SPMV_MGPU_GATHER 0    /* send/recv of the disjoint row slices into the root's y */
#define SPMV_MGPU_REDUCE 1    /* ncclReduce(sum) of full-length partials: accum_results' += */
#define SPMV_MGPU_ALLGATHER 2 /* every device's next x = this y (square matrices; iterative use) */
int spmv_mgpu_create(spmv_mgpu **mg, int ndev, const int *devices, const csr_matrix *matrix);
/* host x[nr_cols] -> device devices[0], then an RCCL broadcast to every device */
int spmv_mgpu_set_x(spmv_mgpu *mg, const ValueType *h_x);
/* the SpMV on every device, then the `exchange` (SPMV_MGPU_*) */
int spmv_mgpu_run(spmv_mgpu *mg, int exchange);
/* `steps` SpMVs of the handle's x, the exchange (SPMV_MGPU_GATHER or _REDUCE) of step k on a
 * second stream overlapping the kernels of step k + 1 (double-buffered y); rank 0's y then holds
 * the last step's result. *ms_per_step = first kernel to last exchange / steps (this process's
 * devices, max). For a stream of SpMVs; one SpMV's exchange cannot overlap its own kernels. */
int spmv_mgpu_run_pipelined(spmv_mgpu *mg, int exchange, int steps, double *ms_per_step);
/* `iters` steps (SpMV + exchange) replayed from one hipGraph (captured on first use; re-captured
 * when exchange, iters or the x buffer change), for a handle driving ONE device (one process per
 * GPU, or a one-device clique). SPMV_MGPU_ALLGATHER iterates x <- A x and leaves A^iters x as the
 * handle's x (spmv_mgpu_get_y / _y_device with ALLGATHER); gather / reduce repeat y = A x.
 * *ms_per_step = the graph's duration / iters. */
int spmv_mgpu_run_graph(spmv_mgpu *mg, int exchange, int iters, double *ms_per_step);
/* y[nr_rows] of the last run to host memory (pass the exchange form of that run) */
int spmv_mgpu_get_y(spmv_mgpu *mg, ValueType *h_y, int exchange);
/* last run: kernels (max over devices) and exchange time, ms (HIP events on each device) */
int spmv_mgpu_get_timing(const spmv_mgpu *mg, double *compute_ms, double *exchange_ms);
/* row slice and device of rank r (device -1 when rank r lives in another process) */
int spmv_mgpu_slice(const spmv_mgpu *mg, int r, IndexType *row_begin, IndexType *row_end, int *device);
void spmv_mgpu_destroy(spmv_mgpu *mg);
/* One process per GPU (e.g. one torch.distributed rank per GPU): rank 0 makes a 128-byte RCCL id
 * with spmv_mgpu_unique_id, the caller shares it, and every rank joins with its own plan for rows
 * [bounds[rank], bounds[rank+1]) (bounds[0..nranks], e.g. spmv_partition_rows) on `device`; the
 * handle borrows the plan. set_x / run / get_y / get_timing then work as above, collectively:
 * every rank calls them; set_x reads x on rank 0 only, get_y of a gather / reduce answers on rank 0
 * only. spmv_mgpu_set_x_device takes rank 0's x already on its device; it first waits for all
 * work this process queued on that device (hipDeviceSynchronize), so an x still being written
 * by any stream is complete before the copy. spmv_mgpu_set_x_device_on orders the copy after
 * the producer's `stream` only (an event wait, no host wait; NULL = the legacy default stream). */
int spmv_mgpu_unique_id(unsigned char *id128);
int spmv_mgpu_create_rank(spmv_mgpu **mg, int rank, int nranks, const unsigned char *id128, int device,
                          const IndexType *bounds, uint32_t nr_cols, const spmv_plan *plan);
int spmv_mgpu_set_x_device(spmv_mgpu *mg, const ValueType *d_x);
int spmv_mgpu_set_x_device_on(spmv_mgpu *mg, const ValueType *d_x, void *stream);
/* device address of this process's y (rank 0's y for a gather / reduce; the local x = y after
 * an all-gather), for callers that keep y on the GPU */
int spmv_mgpu_y_device(spmv_mgpu *mg, int exchange, ValueType **d_y);
/* Ranks in the handle's RCCL communicator (ncclCommCount of its first local device). */
int spmv_mgpu_comm_count(const spmv_mgpu *mg, int *count);

/* The schedule of one SpMV step of rank `rank` (of `nranks`, slices bounds[0..nranks]): the ops
 * that spmv_mgpu_run, _run_pipelined and _run_graph issue for that rank, in order. It is the
 * reference's merge loop (accum_results, csr_hw.cpp:1531-1565, over the CUs of
 * csr_hw_wrapper.cpp:276-281) as data: every RCCL call of the exchange iterates over this list,
 * and tests/test_exchange_schedule.py replays the same lists over torch.distributed (gloo) on the
 * CPU. Local ops (ZERO, COMPUTE) come first and run on the compute stream; the exchange ops
 * (SEND and up) follow inside one RCCL group. Host only, no GPU needed. Returns the number of
 * ops (only the first `cap` are written; ops may be NULL to count), or -1 on bad arguments. */
typedef struct spmv_xop {
    int32_t kind;    /* SPMV_XOP_* */
    int32_t buf;     /* SPMV_XBUF_*: the rank's buffer the op writes or sends */
    int32_t peer;    /* SEND: destination rank, RECV: source rank, REDUCE / BCAST: root; else -1 */
    int32_t out;     /* REDUCE: SPMV_XBUF_Y on the root (the sum lands there), else -1 */
    uint32_t offset; /* first element of the op within buf */
    uint32_t count;  /* elements */
} spmv_xop;
#define SPMV_XOP_ZERO 0    /* buf[offset, offset + count) = 0 */
#define SPMV_XOP_COMPUTE 1 /* buf[offset, offset + count) = rows [bounds[rank], bounds[rank + 1]) of A x */
#define SPMV_XOP_SEND 2    /* ncclSend(buf + offset, count, peer) */
#define SPMV_XOP_RECV 3    /* ncclRecv(buf + offset, count, peer) */
#define SPMV_XOP_REDUCE 4  /* ncclReduce(buf + offset -> out + offset, count, sum, root = peer) */
#define SPMV_XOP_BCAST 5   /* ncclBroadcast(buf + offset, in place, count, root = peer) */
#define SPMV_XBUF_Y 0      /* rank 0's full y (nr_rows) */
#define SPMV_XBUF_SLICE 1  /* rank > 0, gather: its own rows (bounds[rank + 1] - bounds[rank]) */
#define SPMV_XBUF_PART 2   /* reduce: the full-length partial (zero outside the rank's rows) */
#define SPMV_XBUF_XNEXT 3  /* all-gather: the full-length next x of every rank */
int spmv_mgpu_schedule(int exchange, int rank, int nranks, const IndexType *bounds, spmv_xop *ops, int cap);

/* ---------------- synthetic inputs (bench/test infrastructure) ---------------- */
/* Banded: n x n, `width` non-zeros per row, columns [clamp(i - width/2, 0, n - width), +width),
 * values U(-1,1) from splitmix64(seed). Writes d_row_ptr[n+1], d_col[n*width], d_val. */
int spmv_gen_banded(uint32_t n, uint32_t width, uint64_t seed, IndexType *d_row_ptr,
                    IndexType *d_col, ValueType *d_val, void *stream);
/* Power-law row lengths (host): l_i = clamp(floor(s * u_i^-1/2), 1, max_len), s bisected so that
 * sum(l) == nnz exactly (residual spread as +-1 over the last rows). Writes h_row_ptr[n+1]. */
int spmv_gen_powerlaw_row_ptr(uint32_t n, uint64_t nnz, uint32_t max_len, uint64_t seed,
                              IndexType *h_row_ptr, double *scale_out);
/* Fill columns/values of rows [0,n) given d_row_ptr (device): row i with l non-zeros splits
 * [0,m) into l integer strata [floor(j*m/l), floor((j+1)*m/l)) and draws entry j uniformly in
 * stratum j (hash(seed,i,j)): columns strictly increase and spread over [0,m) (needs l <= m).
 * Values U(-1,1). Row i's entries depend only on (seed, i + row_offset, l, m). */
int spmv_gen_fill(uint32_t n, uint32_t m, uint64_t seed, uint64_t row_offset,
                  const IndexType *d_row_ptr, IndexType *d_col, ValueType *d_val, void *stream);
/* d_x[i] = lo + (hi-lo)*u_i, u_i = splitmix64(seed, i + offset) in [0,1). */
int spmv_gen_vector(uint32_t n, uint64_t seed, uint64_t offset, double lo, double hi,
                    ValueType *d_x, void *stream);

/* ---------------- Part 3: fast matrix reader (host only) ----------------
 * Parallel, memory-mapped replacements of the reference's text reader with the same call
 * pattern and results (reader.cpp; threads: env SPMV_READ_THREADS, default min(16, cores)).
 * Superset: MatrixMarket banner/comments (real|integer|pattern, general|symmetric|
 * skew-symmetric, expanded), rows in any order, CRLF, index and count checks. */
/* replaces read_csr_header (csr.cpp:10-46): 0 ok, 1 cannot open / EOF, 2 I/O, 3 parse error.
 * nr_nzeros is the stored count (symmetric files expanded); blocks = 1. */
int spmv_read_csr_header(csr_header *hdr, const char *filename);
/* replaces read_csr_matrix (csr.cpp:87-136) on a matrix from create_csr_matrix(hdr)
 * (csr.cpp:51-67): 0 ok, 1 parse error, 2 I/O error. Trailing empty rows are filled. */
int spmv_read_csr_matrix(csr_matrix *matrix, const char *filename);
/* header + malloc + read in one call; release the arrays with spmv_free_csr (or free()). */
int spmv_read_csr(const char *filename, csr_matrix *out);
void spmv_free_csr(csr_matrix *matrix);

#ifdef __cplusplus
}
#if defined(SPMV_USE_CALLER_CSR_TYPES)
/* the caller's IndexType may be a class (ap_uint<32>, passed by hidden reference under the C++
 * ABI because of its user-provided copy constructor): a template forward converts it to the
 * 32-bit value the C-ABI takes. For a plain uint32_t argument the non-template C-ABI function is
 * the exact match and wins, so a caller whose IndexType is a uint32_t typedef sees no clash.
 * Every other by-value count of this header is declared uint32_t for the same reason. */
template <typename I>
inline int verification(I nr_values, ValueType *sw_values, ValueType *hw_values, int verbose)
{
    return verification((uint32_t)nr_values, sw_values, hw_values, verbose);
}
#endif
#endif

#endif /* CSR_HW_WRAPPER_H */
