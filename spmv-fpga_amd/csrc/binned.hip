// Kernel 6 (SPMV_HW_KERNEL=binned): two-pass SpMV by propagation blocking, for matrices whose
// columns are scattered over an x far larger than L2 (the power-law configs 3 and 5).
//
// Why: the panel sweep (sweep.hip) keeps a row panel's y in LDS and gathers x through L2. Its
// cost is about the x-line gathers (~0.79 L2 line requests per non-zero at the LDS-bound panel
// density) plus the entry stream, because both use the same L2 channels. In fp32
// the stream is only 8 B per entry while the gathers cost the same per line as in fp64. Here the
// gathers become a second stream instead (Beamer, Asanovic, Patterson, "Reducing PageRank
// communication via propagation blocking", IPDPS 2017):
//   pass 1 (k_bin_mul): one workgroup per column window (W columns of x staged in LDS, 156 KiB)
//       streams the window's entries (u16 column offset + value), multiplies by x from LDS and
//       streams the products out in the same order;
//   pass 2 (k_bin_acc): one workgroup per row panel (its y in LDS, fp64) reads the panel's
//       segment of every window (product + u16 row offset), adds into LDS and writes y once.
// This is the reference's 2-D blocking (row slices x column blocks, csr_hw.cpp:25-76, x of a
// block on chip as in spmv.cpp:180) with the per-block partial sums of `compute_results`
// (spmv.cpp:66-104) kept per non-zero and reduced per row by `accum_results`'s `+=`
// (csr_hw.cpp:1531-1565) in LDS.
//
// Layout (built on the GPU): entries ordered (window, panel); a segment = the entries of one
// (window, panel) pair, padded to a multiple of PER = 16 / sizeof(V) entries so every lane's
// group of PER entries is one 16-byte load; each window's range starts on a 128-entry boundary
// (whole 128-byte lines for pass 1's wave loads and stores). Pad (and escape) entries: value 0,
// column offset kBinSent, for which pass 1 writes an exact +0 product (0 * x would be NaN for
// a non-finite x); row offset 0 / delta 0 (or 255 for an escape).
//   d_b_val   V[ent_pad]    values, window-major
//   d_b_colw  u16[ent_pad]  column - window base
//   d_b_rowp  u16[ent_pad]  row - panel base, or (b_delta: segments sorted by row) u8 deltas
//             from the previous entry of the segment (the first from row 0), gaps above 255
//             bridged by escape entries (delta 255, product 0)
//   d_b_prod  V[ent_pad]    products (scratch written by pass 1, read by pass 2)
//   d_b_seg   u64[nwin * npan + 1]  padded segment offsets, index w * npan + p
//   d_b_ub    u64[nunits + 1], d_b_uwin u32[nunits]: pass-1 work units (a window, or a piece of
//             a window holding > 2x the mean entries)
// Bytes per non-zero: fp32 4 + 2 read, 4 written, 4 + 2 (1 with deltas) read = 16 (15); fp64
// 28 (27). Both passes are
// HBM-bound (pass 1's reads and writes add up at ~6 TB/s). Measured on 10M x 10M / 160M
// (profiles/r02_binned.jsonl): fp32 0.457-0.51 ms against 0.60-0.62 ms for the sweep; fp64
// 0.80-0.86 ms against 0.78-0.79, so the automatic choice takes it for fp32 only (plan.cpp),
// and not for skewed matrices (a panel of long rows would serialise pass 2's LDS adds).
//
// fp32 rows: products rounded to fp32 (the reference's fp32 multiply), summed in fp64, rounded
// once. Like the sweep, the LDS adds land in timing order: y is not bitwise reproducible run to
// run (scaled error <= 1e-15 fp64 / one fp32 rounding).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <tuple>
#include <vector>

#include "spmv_internal.hpp"

namespace spmvhw {

namespace {

typedef float binf4 __attribute__((ext_vector_type(4)));
typedef double bind2 __attribute__((ext_vector_type(2)));
typedef uint16_t binh4 __attribute__((ext_vector_type(4)));
typedef uint16_t binh2 __attribute__((ext_vector_type(2)));

template <typename V> struct BinVec;
template <> struct BinVec<float> { typedef binf4 T; typedef binh4 I; };
template <> struct BinVec<double> { typedef bind2 T; typedef binh2 I; };

constexpr int kBinT = 1024;  // one workgroup per CU (LDS-bound in both passes)
constexpr int kBinU = 4;     // pass 1: 64-lane steps of loads in flight per wave
constexpr int kBinD = 8;     // pass 2: steps in flight per wave
constexpr int kBinStageLoads = 10;  // pass 1: 16-B x loads per thread staging a window
constexpr uint64_t kBinAlign = 128;  // entries: window ranges and pass-1 units start at multiples
constexpr double kBinXccBias = 0.0;  // pass-1 window bias by default on a 256-CU chip (build_binned)
constexpr uint16_t kBinSent = 0xFFFF;  // column offset of a pad entry: its product is exactly +0
                                       // (W <= 40960, so no real offset takes this value)

// Window geometry: even windows W0 columns wide, odd ones W1 (W0 = W1 = W unless the pass-1 XCC
// bias is on, build_binned); window pair k spans columns [k (W0 + W1), (k + 1) (W0 + W1)).
__host__ __device__ __forceinline__ uint32_t bin_win_of(uint32_t c, uint32_t W0, uint32_t W1)
{
    const uint32_t pw = W0 + W1, k = c / pw;
    return 2 * k + (c - k * pw >= W0 ? 1u : 0u);
}
__host__ __device__ __forceinline__ uint64_t bin_win_base(uint32_t w, uint32_t W0, uint32_t W1)
{
    return uint64_t(w >> 1) * (W0 + W1) + (w & 1u) * W0;
}

// delta bytes of one lane's PER entries (delta layout)
template <int PER> struct BinDelta;
template <> struct BinDelta<4> { typedef uint32_t T; };
template <> struct BinDelta<2> { typedef uint16_t T; };

#ifdef SPMV_ABLATIONS
// measurement build only: per workgroup of the last launch of pass K (0 = k_bin_mul, 1 =
// k_bin_acc) the 100 MHz real-time clock at its start and after its last store (behind a
// barrier), and its XCC id (tools/wg_timeline.py --binned reads them with spmv_abl_bin_times)
__device__ unsigned long long g_abl_bin[2][4 * 4096];
#define BN_STAMP(K, k)                                                                             \
    do {                                                                                           \
        if ((k) == 1)                                                                              \
            __syncthreads();                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < 4096) {                                               \
            g_abl_bin[K][4 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();                 \
            if ((k) == 0)                                                                          \
                g_abl_bin[K][4 * blockIdx.x + 3] = (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32; \
        }                                                                                          \
    } while (0)
#else
#define BN_STAMP(K, k) \
    do {               \
    } while (0)
#endif

// Pass 1: unit u = entries [ub[u], ub[u+1]) of window uwin[u] (both multiples of PER).
// AL: x is 16-byte aligned, so the window is staged with 16-byte loads.
// mirror != 0 (variant 7, same y): the 16-byte product vector of entries [i, i + PER) is stored at
// mirror - i instead of i (mirror = the last vector's index), so the product stores run down the
// array while the entry loads run up it, and the two streams keep no fixed address distance
// (config 5's per-plan modes). Pass 2 reads them back at the same place.
// POL (variants 3-5, the same y): bit 0 = temporal (default-policy) product stores instead of
// non-temporal ones, bit 1 = temporal entry loads
template <typename V, bool AL, int POL = 0>
__global__ __launch_bounds__(kBinT) void k_bin_mul(const V *__restrict__ x, uint32_t ncols, uint32_t W0, uint32_t W1,
                                                   const uint64_t *__restrict__ ub, const uint32_t *__restrict__ uwin,
                                                   const uint16_t *__restrict__ colw, const V *__restrict__ val,
                                                   V *__restrict__ prod, uint64_t mirror)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *xs = reinterpret_cast<V *>(smem);
    typedef typename BinVec<V>::T VT;
    typedef typename BinVec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    BN_STAMP(0, 0);
    const uint32_t u = blockIdx.x;
    const uint64_t c0 = bin_win_base(uwin[u], W0, W1);
    const uint32_t wn = (uint32_t)std::min<uint64_t>(uwin[u] & 1 ? W1 : W0, ncols - c0);  // columns of this window
    if (AL) {
        VT t[kBinStageLoads];
#pragma unroll
        for (int r = 0; r < kBinStageLoads; ++r) {
            const uint32_t i = (r * kBinT + threadIdx.x) * PER;
            if (i + PER <= wn) {
                t[r] = *reinterpret_cast<const VT *>(x + c0 + i);
            } else if (i < wn) {
#pragma unroll
                for (int k = 0; k < PER; ++k)
                    t[r][k] = i + k < wn ? x[c0 + i + k] : V(0);
            }
        }
#pragma unroll
        for (int r = 0; r < kBinStageLoads; ++r) {
            const uint32_t i = (r * kBinT + threadIdx.x) * PER;
            if (i < wn)
                *reinterpret_cast<VT *>(xs + i) = t[r];
        }
    } else {
        for (uint32_t i0 = 0; i0 < wn; i0 += 8 * kBinT) {
            V t[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t i = i0 + r * kBinT + threadIdx.x;
                if (i < wn)
                    t[r] = x[c0 + i];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t i = i0 + r * kBinT + threadIdx.x;
                if (i < wn)
                    xs[i] = t[r];
            }
        }
    }
    __syncthreads();
    const uint64_t e0 = ub[u], e1 = ub[u + 1];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint64_t STEP = 64 * PER;
    for (uint64_t s = e0 + wv * STEP * kBinU; s < e1; s += (kBinT / 64) * STEP * kBinU) {
        VT v[kBinU];
        IT c[kBinU];
#pragma unroll
        for (int k = 0; k < kBinU; ++k) {
            const uint64_t i = s + k * STEP + lane * PER;
            if (i < e1) {
                if constexpr (POL & 2) {
                    v[k] = *reinterpret_cast<const VT *>(val + i);
                    c[k] = *reinterpret_cast<const IT *>(colw + i);
                } else {
                    v[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(val + i));
                    c[k] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(colw + i));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kBinU; ++k) {
            const uint64_t i = s + k * STEP + lane * PER;
            if (i < e1) {
                VT pr;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const uint16_t cq = c[k][q];
                    const V xq = xs[cq == kBinSent ? 0 : cq];
                    pr[q] = cq == kBinSent ? V(0) : v[k][q] * xq;
                }
                const uint64_t o = mirror ? mirror - i : i;
                if constexpr (POL & 1)
                    *reinterpret_cast<VT *>(prod + o) = pr;
                else
                    __builtin_nontemporal_store(pr, reinterpret_cast<VT *>(prod + o));
            }
        }
    }
    BN_STAMP(0, 1);
}

// Pass 2: workgroup = panel p (rows [panel_row[p], panel_row[p+1])). Wave v takes windows v,
// v + 16, ...; its segments form one stream of 64-lane steps of PER entries (the last step of a
// segment masked), kBinD steps of loads in flight before the adds. The bounds of the wave's next
// 64 segments sit in a lane table (lane l: segment 64c + l) read with readlane, so crossing a
// segment costs no scalar load (whose wait would also drain the outstanding LDS adds).
// DELTA: `rowp` holds 1-byte row deltas (segments sorted by row, each starting from row 0); a
// step's rows are its deltas' running sum: a 64-lane prefix sum of the lanes' PER-delta totals
// plus the carry of the segment's earlier steps.
// ABL (measurement-only ablations, tools library; wrong y): 1 = no LDS adds (products summed into
// a register, added once at the end: the memory stream alone), 2 = loads re-read the wave's first
// 16 steps (L2-resident: the LDS adds and decode alone)
// FL...: empty, or (uint32_t *yflag, uint32_t yepoch) for spmv_hw's streamed copy-back -- each
// panel's flag in host memory set to the call's epoch once its rows of y are published (the
// sweep's scheme, sweep.hip k_spmv_sweep_packed); the plain instantiation is untouched by it.
template <typename V, bool DELTA, int ABL = 0, typename... FL>
__global__ __launch_bounds__(kBinT) void k_bin_acc(const V *__restrict__ prod, const void *__restrict__ rowp,
                                                   const uint64_t *__restrict__ seg,
                                                   const uint32_t *__restrict__ panel_row, uint32_t nwin,
                                                   uint32_t npan, uint32_t slots, V *__restrict__ y, uint64_t mirror,
                                                   FL... fl)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *ys = reinterpret_cast<double *>(smem);
    typedef typename BinVec<V>::T VT;
    typedef typename BinVec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    constexpr uint32_t STEP = 64 * PER;
    constexpr uint32_t WAVES = kBinT / 64;
    BN_STAMP(1, 0);
    for (uint32_t i = threadIdx.x; i < slots; i += kBinT)
        ys[i] = 0.0;
    __syncthreads();
    const uint32_t p = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nmine = nwin > wv ? (nwin - wv + WAVES - 1) / WAVES : 0;  // segments of this wave
    uint32_t tlo = 0, thi = 0, tlo2 = 0, thi2 = 0;  // lane table: start / end of segment 64c + lane
    auto table = [&](uint32_t c) {
        const uint32_t o = c * 64 + lane;
        uint64_t a = 0, b = 0;
        if (o < nmine) {
            const uint64_t k = (uint64_t)(wv + o * WAVES) * npan + p;
            a = seg[k];
            b = seg[k + 1];
        }
        tlo = (uint32_t)a;
        thi = (uint32_t)(a >> 32);
        tlo2 = (uint32_t)b;
        thi2 = (uint32_t)(b >> 32);
    };
    auto bounds = [&](uint32_t o, uint64_t &a, uint64_t &b) {
        const uint32_t l = o & 63;
        // readlane returns a signed int: widen through uint32_t, or a low word >= 2^31 (offsets past
        // 2^31 entries) would sign-extend into the high word
        a = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(tlo, l) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(thi, l) << 32);
        b = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(tlo2, l) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(thi2, l) << 32);
    };
    uint32_t o = 0;  // ordinal of the wave's current segment
    uint64_t pos = 0, end = 0;
    if (nmine) {
        table(0);
        bounds(0, pos, end);
    }
    typedef typename BinDelta<PER>::T DT;
    const uint16_t *__restrict__ rows16 = reinterpret_cast<const uint16_t *>(rowp);
    const uint8_t *__restrict__ rows8 = reinterpret_cast<const uint8_t *>(rowp);
    uint32_t carry = 0;  // DELTA: row of the segment's last entry so far
    double sink = 0.0;   // ABL 1 only
    while (o < nmine) {
        VT v[kBinD];
        IT r[kBinD];
        DT dl[kBinD];
        uint64_t at[kBinD], en[kBinD];
        bool fresh[kBinD];  // DELTA: the step starts a segment (uniform)
#pragma unroll
        for (int k = 0; k < kBinD; ++k) {
            bool moved = false;
            while (pos >= end && o < nmine) {  // next non-empty segment (uniform)
                ++o;
                moved = true;
                if (o < nmine) {
                    if ((o & 63) == 0)
                        table(o >> 6);
                    bounds(o, pos, end);
                }
            }
            at[k] = pos + lane * PER;
            en[k] = o < nmine ? end : 0;
            fresh[k] = moved;
            if (at[k] < en[k]) {
                uint64_t ld = at[k];
                if constexpr (ABL == 2)
                    ld = (ld & ~(uint64_t)(16 * STEP - 1)) == 0 ? ld : (ld & (16 * STEP - 1));
                v[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(prod + (mirror ? mirror - ld : ld)));
                if (DELTA)
                    dl[k] = __builtin_nontemporal_load(reinterpret_cast<const DT *>(rows8 + ld));
                else
                    r[k] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(rows16 + ld));
            } else {
                dl[k] = 0;
            }
            pos += STEP;
        }
#pragma unroll
        for (int k = 0; k < kBinD; ++k) {
            if (DELTA) {
                if (fresh[k])
                    carry = 0;
                uint32_t d[PER], t = 0;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    d[q] = ((uint32_t)dl[k] >> (8 * q)) & 0xFFu;
                    t += d[q];
                }
                const uint32_t inc = wave_inclusive_sum(t);
                uint32_t row = carry + inc - t;
                carry += (uint32_t)__builtin_amdgcn_readlane(inc, 63);
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    row += d[q];
                    r[k][q] = (uint16_t)row;
                }
            }
            if (at[k] < en[k]) {
                if constexpr (ABL == 1) {
#pragma unroll
                    for (int q = 0; q < PER; ++q)
                        sink += (double)v[k][q] * (double)(r[k][q] + 1);
                } else {
#pragma unroll
                    for (int q = 0; q < PER; ++q)
                        atomicAdd(&ys[r[k][q]], (double)v[k][q]);
                }
            }
        }
    }
    if constexpr (ABL == 1)
        atomicAdd(&ys[0], sink);
    __syncthreads();
    const uint32_t r0 = panel_row[p], nr = panel_row[p + 1] - r0;
    for (uint32_t i = threadIdx.x; i < nr; i += kBinT)
        y[r0 + i] = (V)ys[i];
    if constexpr (sizeof...(FL) != 0) {
        // every wave's stores complete, then one lane's system-scope release publishes the
        // panel's rows and sets its flag
        const auto args = std::make_tuple(fl...);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(std::get<0>(args) + p, std::get<1>(args), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    BN_STAMP(1, 1);
}

// row of entry j: the last row r < n with rp[r] <= j (empty rows are skipped over)
__device__ __forceinline__ uint32_t bin_row_of(const IndexType *__restrict__ rp, IndexType n, uint64_t j)
{
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (rp[mid] <= j)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// per entry: segment key (window * npan + panel), row offset in its panel; segment counts
__global__ void k_bin_keys(const IndexType *__restrict__ rp, IndexType n, const IndexType *__restrict__ col,
                           uint64_t nnz, const uint32_t *__restrict__ panel_row, uint32_t npan, uint32_t W0,
                           uint32_t W1, uint32_t *__restrict__ key, uint16_t *__restrict__ rowp, uint32_t *__restrict__ cnt)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz)
        return;
    const uint32_t r = bin_row_of(rp, n, j);
    uint32_t lo = 0, hi = npan;  // last panel q with panel_row[q] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (panel_row[mid] <= r)
            lo = mid;
        else
            hi = mid;
    }
    const uint32_t k = bin_win_of(col[j], W0, W1) * npan + lo;
    key[j] = k;
    rowp[j] = (uint16_t)(r - panel_row[lo]);
    atomicAdd(&cnt[k], 1u);
}

template <typename V>
__global__ void k_bin_scatter(const uint32_t *__restrict__ key, const uint16_t *__restrict__ rowp_in,
                              const IndexType *__restrict__ col, const V *__restrict__ val_in, uint64_t nnz,
                              uint32_t npan, uint32_t W0, uint32_t W1, const uint64_t *__restrict__ seg,
                              uint32_t *__restrict__ cursor, V *__restrict__ val, uint16_t *__restrict__ colw,
                              uint16_t *__restrict__ rowp)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz)
        return;
    const uint32_t k = key[j];
    const uint64_t d = seg[k] + atomicAdd(&cursor[k], 1u);
    val[d] = val_in[j];
    colw[d] = (uint16_t)(col[j] - bin_win_base(k / npan, W0, W1));
    rowp[d] = rowp_in[j];
}

// escape entries before sorted entry k of the delta layout: a row gap above 255 is bridged by
// pad entries of delta 255 (product 0), the entry itself keeps the remainder (1..255)
__device__ __forceinline__ uint32_t bin_escapes(uint32_t gap) { return gap > 255u ? (gap - 1u) / 255u : 0u; }

// sort key of the delta layout: (segment << 16) | row offset, and the entry's CSR index
__global__ void k_bin_key64(const uint32_t *__restrict__ key, const uint16_t *__restrict__ rowp, uint64_t nnz,
                            uint64_t *__restrict__ k64, uint32_t *__restrict__ idx)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz)
        return;
    k64[j] = ((uint64_t)key[j] << 16) | rowp[j];
    idx[j] = (uint32_t)j;
}

// per sorted entry: its escape count (segments start from row 0); per segment: their sum
__global__ void k_bin_gaps(const uint64_t *__restrict__ k64, uint64_t nnz, uint32_t *__restrict__ pads,
                           uint32_t *__restrict__ esc)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz)
        return;
    const uint64_t sg = k64[k] >> 16;
    const uint32_t row = (uint32_t)(k64[k] & 0xFFFFu);
    const uint32_t prev = (k > 0 && (k64[k - 1] >> 16) == sg) ? (uint32_t)(k64[k - 1] & 0xFFFFu) : 0u;
    const uint32_t e = bin_escapes(row - prev);
    pads[k] = e;
    if (e)
        atomicAdd(&esc[sg], e);
}

// delta layout: sorted entry k (and the escapes before it) to its padded position
template <typename V>
__global__ void k_bin_scatter_delta(const uint64_t *__restrict__ k64, const uint32_t *__restrict__ idx,
                                    const uint32_t *__restrict__ pscan, const uint64_t *__restrict__ sorted_off,
                                    uint64_t nnz, uint32_t npan, uint32_t W0, uint32_t W1,
                                    const IndexType *__restrict__ col,
                                    const V *__restrict__ val_in, const uint64_t *__restrict__ seg,
                                    V *__restrict__ val, uint16_t *__restrict__ colw, uint8_t *__restrict__ delta)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz)
        return;
    const uint64_t sg = k64[k] >> 16;
    const uint32_t row = (uint32_t)(k64[k] & 0xFFFFu);
    const uint64_t k0 = sorted_off[sg];
    const uint32_t prev = k > k0 ? (uint32_t)(k64[k - 1] & 0xFFFFu) : 0u;
    const uint32_t gap = row - prev, e = bin_escapes(gap);
    // entries of this segment before k, plus all their escapes, plus this entry's own escapes
    const uint64_t d = seg[sg] + (k - k0) + (uint64_t)(pscan[k] - pscan[k0]) + e;
    for (uint32_t t = 0; t < e; ++t) {
        val[d - e + t] = V(0);
        colw[d - e + t] = kBinSent;
        delta[d - e + t] = 255;
    }
    const uint32_t j = idx[k];
    val[d] = val_in[j];
    colw[d] = (uint16_t)(col[j] - bin_win_base((uint32_t)(sg / npan), W0, W1));
    delta[d] = (uint8_t)(gap - 255u * e);
}

// pad entries at the end of every segment: value 0, the sentinel column (product exactly +0),
// row offset 0 / delta 0 (adding +0 to a row sum changes nothing: a sum that starts at +0 is
// never -0)
template <typename V, bool DELTA>
__global__ void k_bin_pad(uint64_t nseg, const uint64_t *__restrict__ seg, const uint32_t *__restrict__ cnt,
                          const uint32_t *__restrict__ esc, V *__restrict__ val, uint16_t *__restrict__ colw,
                          void *__restrict__ rowp)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nseg)
        return;
    for (uint64_t d = seg[k] + cnt[k] + (DELTA ? esc[k] : 0u); d < seg[k + 1]; ++d) {
        val[d] = V(0);
        colw[d] = kBinSent;
        if (DELTA)
            reinterpret_cast<uint8_t *>(rowp)[d] = 0;
        else
            reinterpret_cast<uint16_t *>(rowp)[d] = 0;
    }
}

}  // namespace

hipError_t launch_binned(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    constexpr uint64_t PERV = 16 / sizeof(ValueType);
    // variant 7: mirrored products (k_bin_mul); the index of the last product vector
    const uint64_t mirror = p.variant == 7 ? std::max<uint64_t>(p.ent_pad, PERV) - PERV : 0;
    if (p.b_nunits) {
        const size_t lds1 = size_t(std::max(p.b_W, p.b_W1)) * sizeof(ValueType);
        const bool al = (reinterpret_cast<uintptr_t>(d_x) & 15u) == 0;
        // pass-1 cache policy: temporal product stores when the products fit well within
        // reach of the 256 MB MALL (fp32 10M/160M: 640 MB, 0.460 vs 0.487 ms; fp64 1.28 GB:
        // 0.852 vs 0.835, profiles/r03s_binned_policy.jsonl); variants 3-5 force a policy, 6 the
        // non-temporal stores
        const int pol = p.variant >= 3 && p.variant <= 5 ? p.variant - 2
                        : p.variant == 6                ? 0
                                                        : (p.b_prod_temporal ? 1 : 0);
        if (pol && al) {
#define BINPOL(P)                                                                                          \
    launch_or_warm(warm, k_bin_mul<ValueType, true, P>, dim3((unsigned)p.b_nunits), dim3(kBinT), lds1, s, d_x, \
                   (uint32_t)p.nr_cols, p.b_W, p.b_W1, p.d_b_ub, p.d_b_uwin, p.d_b_colw, p.d_b_val, p.d_b_prod, mirror)
            if (pol == 1) BINPOL(1); else if (pol == 2) BINPOL(2); else BINPOL(3);
#undef BINPOL
        } else if (al || warm)
            launch_or_warm(warm, k_bin_mul<ValueType, true>, dim3((unsigned)p.b_nunits), dim3(kBinT), lds1, s, d_x,
                           (uint32_t)p.nr_cols, p.b_W, p.b_W1, p.d_b_ub, p.d_b_uwin, p.d_b_colw, p.d_b_val, p.d_b_prod, mirror);
        if (!al || warm)
            launch_or_warm(warm, k_bin_mul<ValueType, false>, dim3((unsigned)p.b_nunits), dim3(kBinT), lds1, s, d_x,
                           (uint32_t)p.nr_cols, p.b_W, p.b_W1, p.d_b_ub, p.d_b_uwin, p.d_b_colw, p.d_b_val, p.d_b_prod, mirror);
    }
    const size_t lds2 = (size_t(p.panel_rmax) + 1) * sizeof(double);
    // variants 1 / 2 (tests): segment offsets rebased past 2^31 / 2^32, the product and row arrays
    // rebased the other way, so pass 2 touches the same addresses through 64-bit offsets whose low
    // word has bit 31 set (spmv_plan_set_variant)
    const uint64_t base = p.d_b_seg_hi ? p.b_seg_base : 0;
    const uint64_t *seg = p.d_b_seg_hi ? p.d_b_seg_hi : p.d_b_seg;
    const ValueType *prod = reinterpret_cast<const ValueType *>(
        reinterpret_cast<uintptr_t>(p.d_b_prod) - base * sizeof(ValueType));
    const void *rowp = reinterpret_cast<const void *>(reinterpret_cast<uintptr_t>(p.d_b_rowp) -
                                                      base * (p.b_delta ? 1 : 2));
    // pass 2 sees offsets ld + base against prod - base: the mirrored index is mirror + 2 base - ld
    const uint64_t mirror2 = mirror ? mirror + 2 * base : 0;
#ifdef SPMV_ABLATIONS
    if (p.b_delta && (p.variant == 51 || p.variant == 52)) {
        if (p.variant == 51)
            launch_or_warm(warm, k_bin_acc<ValueType, true, 1>, dim3((unsigned)p.npanels), dim3(kBinT), lds2, s, prod,
                           rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels, p.panel_rmax + 1, d_y, mirror2);
        else
            launch_or_warm(warm, k_bin_acc<ValueType, true, 2>, dim3((unsigned)p.npanels), dim3(kBinT), lds2, s, prod,
                           rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels, p.panel_rmax + 1, d_y, mirror2);
        return hipGetLastError();
    }
#endif
    // spmv_hw's streamed copy-back: the flagged pass 2 (sweep_can_flag_panels)
    if (p.y_flag || warm) {
        if (p.b_delta)
            launch_or_warm(warm, k_bin_acc<ValueType, true, 0, uint32_t *, uint32_t>, dim3((unsigned)p.npanels),
                           dim3(kBinT), lds2, s, prod, rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels,
                           p.panel_rmax + 1, d_y, mirror2, p.y_flag, p.y_epoch);
        else
            launch_or_warm(warm, k_bin_acc<ValueType, false, 0, uint32_t *, uint32_t>, dim3((unsigned)p.npanels),
                           dim3(kBinT), lds2, s, prod, rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels,
                           p.panel_rmax + 1, d_y, mirror2, p.y_flag, p.y_epoch);
    }
    if (!p.y_flag) {
        if (p.b_delta)
            launch_or_warm(warm, k_bin_acc<ValueType, true>, dim3((unsigned)p.npanels), dim3(kBinT), lds2, s, prod,
                           rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels, p.panel_rmax + 1, d_y, mirror2);
        else
            launch_or_warm(warm, k_bin_acc<ValueType, false>, dim3((unsigned)p.npanels), dim3(kBinT), lds2, s, prod,
                           rowp, seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels, p.panel_rmax + 1, d_y, mirror2);
    }
    return hipGetLastError();
}

// Host: windows (W columns, a whole number of rounds of workgroups where x allows), panels
// (nnz-balanced, <= rmax rows, whole rounds), then keys + counts, padded segment offsets, the
// pass-1 units, and the scatter. rc 2: the segment table would be too large (the caller may use
// another kernel).
int build_binned(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                 hipStream_t s)
{
    constexpr uint32_t PER = 16 / sizeof(ValueType);
    const IndexType n = p.nr_rows;
    const uint64_t nnz = p.nnz, ncols = p.nr_cols;
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, p.device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
    }
    // windows: W <= what 160 KiB of LDS holds (and the u16 offsets), a multiple of PER
    const uint64_t wmax = std::min<uint64_t>((kSweepLdsBytes - 256) / sizeof(ValueType) / PER * PER, 65536);
    uint64_t nwin = 1, W = PER;
    if (ncols) {
        const uint64_t rounds = std::max<uint64_t>(1, (ncols + cus * wmax - 1) / (cus * wmax));
        nwin = std::min<uint64_t>(cus * rounds, (ncols + PER - 1) / PER);
        W = ((ncols + nwin - 1) / nwin + PER - 1) / PER * PER;
        nwin = (ncols + W - 1) / W;
    }
    // Pass-1 XCC bias: unit u runs on XCC u % 8 (tools/xcc_map_probe.py), and on the boxes
    // measured pass 1's one-window workgroups take 266 us on even XCCs against 280 us on odd ones
    // (tools/wg_timeline.py --binned, profiles/r03bn_binned_timeline.jsonl). With one unit per
    // window (nwin a whole number of rounds) even windows get W (1 + d) columns, odd ones
    // W (1 - d): every pair still spans 2W, so a column's window stays closed-form
    // (bin_win_of). Env SPMV_BIN_XCC_BIAS=d (0 = even widths); only on a whole 256-CU chip.
    uint64_t W0 = W, W1 = W;
    {
        const char *xb = ablation_env("SPMV_BIN_XCC_BIAS");
        double d = xb ? std::atof(xb) : (cus == 256 ? kBinXccBias : 0.0);
        if (!(d > -0.25 && d < 0.25) || nwin < (uint64_t)cus || nwin % cus)
            d = 0.0;
        const uint64_t w0 = std::min<uint64_t>(wmax, (uint64_t(std::llround(W * (1.0 + d))) + PER / 2) / PER * PER);
        if (d != 0.0 && w0 >= PER && w0 < 2 * W) {
            W0 = w0;
            W1 = 2 * W - w0;
            if (W1 > wmax) {  // a negative bias past the LDS: even widths
                W0 = W1 = W;
            }
            const uint64_t pw = W0 + W1, k = ncols / pw, rem = ncols - k * pw;
            nwin = 2 * k + (rem == 0 ? 0 : rem <= W0 ? 1 : 2);
        }
    }
    // panels: y of <= rmax rows in LDS (fp64), plus the scratch slot of the pad entries
    const uint32_t rmax = (uint32_t)std::min<uint64_t>((kSweepLdsBytes - 256) / 8 - 1, 65534);
    std::vector<uint32_t> prow;
    // subdivide: as in build_sweep, a run of (nearly) empty rows longer than a panel that no
    // nnz-balanced cut reaches ends a bounded search; the first P's cuts are then kept and any
    // panel above rmax rows is split into panels of at most rmax rows
    const uint64_t P_first = std::max<uint64_t>({1, (n + rmax - 1) / rmax, std::min<uint64_t>(cus, n)});
    bool subdivide = false;
    for (uint64_t P = P_first;; ++P) {
        if (P > (uint64_t)cus && P % cus)
            P = (P + cus - 1) / cus * cus;  // whole rounds of workgroups
        P = std::min<uint64_t>(P, std::max<uint64_t>(n, 1));
        prow.assign(1, 0);
        bool ok = true;
        IndexType r = 0;
        for (uint64_t q = 1; q <= P && ok; ++q) {
            const uint64_t target = nnz * q / P;
            IndexType e = (q == P) ? n : (IndexType)(std::lower_bound(h_rp, h_rp + n + 1, (IndexType)target) - h_rp);
            e = std::max(e, r);
            if (e - r > rmax && subdivide)
                for (; e - r > rmax; r += rmax)
                    prow.push_back(r + rmax);
            if (e - r > rmax)
                ok = false;
            prow.push_back(e);
            r = e;
        }
        if (ok)
            break;
        if (P >= n || P > 8 * std::max<uint64_t>(P_first, (uint64_t)cus)) {
            if (subdivide) {
                set_error("build_binned: cannot form panels");
                return 1;
            }
            subdivide = true;
            P = P_first - 1;  // (++P)
        }
    }
    const uint32_t P = (uint32_t)(prow.size() - 1);
    uint32_t rmax_used = 0;
    uint64_t emax = 0;
    for (uint32_t q = 0; q < P; ++q) {
        rmax_used = std::max(rmax_used, prow[q + 1] - prow[q]);
        emax = std::max<uint64_t>(emax, uint64_t(h_rp[prow[q + 1]]) - h_rp[prow[q]]);
    }
    // A panel far above the mean holds long rows; pass 2 would add their products into one LDS
    // address each, serialised (2M rows of ~16 plus two rows of 2M entries, fp32: 2.60 ms here
    // against 0.42 ms for the sweep, which cuts such panels into pieces). The automatic choice
    // then takes the sweep.
    if (p.bin_skew_limit > 0.0 && P > 1 && double(emax) > p.bin_skew_limit * double(nnz) / P) {
        set_error("build_binned: a panel holds long rows (skewed)");
        return 2;
    }
    // Balanced panels still let a row of up to ~2x the mean panel entries pass the test above;
    // its adds all land on one LDS address. The longest row is checked on its own.
    if (p.bin_row_limit > 0.0 && P > 0) {
        uint64_t lmax = 0;
        for (IndexType r = 0; r < n; ++r)
            lmax = std::max<uint64_t>(lmax, uint64_t(h_rp[r + 1]) - h_rp[r]);
        if (double(lmax) > p.bin_row_limit * double(nnz) / P) {
            set_error("build_binned: a row holds " + std::to_string(lmax) + " entries (long row)");
            return 2;
        }
    }
    const uint64_t nseg = nwin * P;
    if (nseg >= (1ull << 28)) {
        set_error("build_binned: too many (window, panel) segments");
        return 2;
    }
    p.npanels = P;
    p.panel_rmax = rmax_used;
    p.b_nwin = (uint32_t)nwin;
    p.b_W = (uint32_t)W0;
    p.b_W1 = (uint32_t)W1;
    SPMV_TRY(hipMalloc((void **)&p.d_panel_row, (P + 1) * 4));
    SPMV_TRY(hipMemcpyAsync(p.d_panel_row, prow.data(), (P + 1) * 4, hipMemcpyHostToDevice, s));

    IndexType *d_rp = nullptr;
    uint32_t *d_key = nullptr, *d_cnt = nullptr, *d_cur = nullptr;
    uint16_t *d_rowp_tmp = nullptr;
    // delta layout temporaries
    uint64_t *d_k64 = nullptr, *d_k64s = nullptr, *d_soff = nullptr;
    uint32_t *d_idx = nullptr, *d_idxs = nullptr, *d_pads = nullptr, *d_pscan = nullptr, *d_esc = nullptr;
    void *d_tmp = nullptr;
    auto free_delta = [&]() {
        for (void **q : {(void **)&d_k64, (void **)&d_k64s, (void **)&d_soff, (void **)&d_idx, (void **)&d_idxs,
                         (void **)&d_pads, (void **)&d_pscan, (void **)&d_esc, &d_tmp})
            if (*q) {
                (void)hipFree(*q);
                *q = nullptr;
            }
    };
    auto cleanup = [&]() {
        for (void *q : {(void *)d_rp, (void *)d_key, (void *)d_cnt, (void *)d_cur, (void *)d_rowp_tmp})
            if (q)
                (void)hipFree(q);
        free_delta();
    };
    auto fail = [&](hipError_t e, const char *what) {
        set_error(std::string("build_binned: ") + what + ": " + hipGetErrorString(e));
        cleanup();
        return 1;
    };
#define BN_TRY(x)                              \
    do {                                       \
        hipError_t e_ = (x);                   \
        if (e_ != hipSuccess)                  \
            return fail(e_, #x);               \
    } while (0)
    std::vector<uint32_t> cnt(nseg, 0);
    BN_TRY(hipMalloc((void **)&d_cnt, std::max<uint64_t>(nseg, 1) * 4));
    BN_TRY(hipMemsetAsync(d_cnt, 0, std::max<uint64_t>(nseg, 1) * 4, s));
    if (nnz) {
        BN_TRY(hipMalloc((void **)&d_rp, (size_t(n) + 1) * 4));
        BN_TRY(hipMemcpyAsync(d_rp, h_rp, (size_t(n) + 1) * 4, hipMemcpyHostToDevice, s));
        BN_TRY(hipMalloc((void **)&d_key, nnz * 4));
        BN_TRY(hipMalloc((void **)&d_rowp_tmp, nnz * 2));
        hipLaunchKernelGGL(k_bin_keys, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_rp, n, d_col_src, nnz,
                           p.d_panel_row, P, (uint32_t)W0, (uint32_t)W1, d_key, d_rowp_tmp, d_cnt);
        BN_TRY(hipGetLastError());
        BN_TRY(hipMemcpyAsync(cnt.data(), d_cnt, nseg * 4, hipMemcpyDeviceToHost, s));
        BN_TRY(hipStreamSynchronize(s));
    }
    // Delta layout (env SPMV_BIN_DELTA: 0 never, 1 always, default when its escape entries stay
    // under 1 % of nnz): each segment sorted by row, 1-byte row deltas, pass 2 reading 1 B less
    // per non-zero (tools/delta_probe.hip: pass 2 0.159 vs 0.180 ms on the 10M/160M fp32 shape).
    // Sparse segments (small matrices, gaps over 255 rows) would need many escapes: u16 offsets.
    std::vector<uint32_t> esc(nseg, 0);
    bool delta = false;
    {
        const char *denv = ablation_env("SPMV_BIN_DELTA");
        const bool never = denv && denv[0] == '0', always = denv && denv[0] == '1';
        delta = !nnz && always;  // an empty slice: either form reads nothing
        if (nnz && !never) {
            BN_TRY(hipMalloc((void **)&d_k64, nnz * 8));
            BN_TRY(hipMalloc((void **)&d_k64s, nnz * 8));
            BN_TRY(hipMalloc((void **)&d_idx, nnz * 4));
            BN_TRY(hipMalloc((void **)&d_idxs, nnz * 4));
            hipLaunchKernelGGL(k_bin_key64, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_key, d_rowp_tmp,
                               nnz, d_k64, d_idx);
            BN_TRY(hipGetLastError());
            int end_bit = 17;
            while (end_bit < 64 && (1ull << (end_bit - 16)) < nseg)
                ++end_bit;
            size_t tb = 0;
            BN_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_k64, d_k64s, d_idx, d_idxs, nnz, 0, end_bit, s));
            BN_TRY(hipMalloc(&d_tmp, tb));
            BN_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb, d_k64, d_k64s, d_idx, d_idxs, nnz, 0, end_bit, s));
            BN_TRY(hipFree(d_k64));
            d_k64 = nullptr;
            BN_TRY(hipFree(d_idx));
            d_idx = nullptr;
            BN_TRY(hipFree(d_tmp));
            d_tmp = nullptr;
            BN_TRY(hipMalloc((void **)&d_pads, nnz * 4));
            BN_TRY(hipMalloc((void **)&d_esc, std::max<uint64_t>(nseg, 1) * 4));
            BN_TRY(hipMemsetAsync(d_esc, 0, std::max<uint64_t>(nseg, 1) * 4, s));
            hipLaunchKernelGGL(k_bin_gaps, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_k64s, nnz, d_pads,
                               d_esc);
            BN_TRY(hipGetLastError());
            BN_TRY(hipMemcpyAsync(esc.data(), d_esc, nseg * 4, hipMemcpyDeviceToHost, s));
            BN_TRY(hipStreamSynchronize(s));
            uint64_t total = 0;
            for (uint32_t e : esc)
                total += e;
            delta = always || total * 100 <= nnz;
            if (delta) {
                BN_TRY(hipMalloc((void **)&d_pscan, nnz * 4));
                tb = 0;
                BN_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, d_pads, d_pscan, nnz, s));
                BN_TRY(hipMalloc(&d_tmp, tb));
                BN_TRY(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb, d_pads, d_pscan, nnz, s));
                std::vector<uint64_t> soff(nseg + 1, 0);
                for (uint64_t k = 0; k < nseg; ++k)
                    soff[k + 1] = soff[k] + cnt[k];
                BN_TRY(hipMalloc((void **)&d_soff, (nseg + 1) * 8));
                BN_TRY(hipMemcpyAsync(d_soff, soff.data(), (nseg + 1) * 8, hipMemcpyHostToDevice, s));
                BN_TRY(hipStreamSynchronize(s));
            } else {
                free_delta();
                std::fill(esc.begin(), esc.end(), 0u);
            }
        }
    }
    p.b_delta = delta;
    // padded segment offsets (window-major), then the pass-1 units
    // Each window's range also starts on a 128-entry boundary (the last segment of the window
    // takes the extra pad entries): pass 1's 1-KiB wave loads and stores then cover whole
    // 128-byte lines instead of straddling them (partial-line stores).
    std::vector<uint64_t> seg(nseg + 1, 0);
    for (uint64_t k = 0; k < nseg; ++k) {
        seg[k + 1] = seg[k] + (uint64_t(cnt[k]) + esc[k] + PER - 1) / PER * PER;
        if ((k + 1) % P == 0)
            seg[k + 1] = (seg[k + 1] + kBinAlign - 1) / kBinAlign * kBinAlign;
    }
    const uint64_t ent_pad = seg[nseg];
    p.ent_pad = ent_pad;
    p.b_prod_temporal = ent_pad * sizeof(ValueType) <= (1ull << 30);
    std::vector<uint64_t> ub(1, 0);
    std::vector<uint32_t> uwin;
    {
        const double mean = nwin ? double(ent_pad) / double(nwin) : 0.0;
        const uint64_t fill = nwin < (uint64_t)cus ? (cus + nwin - 1) / nwin : 1;  // few windows: pieces
        for (uint64_t w = 0; w < nwin; ++w) {
            const uint64_t a = seg[w * P], b = seg[(w + 1) * P], e = b - a;
            if (!e)
                continue;
            uint64_t k = std::max<uint64_t>(fill, (uint64_t)std::ceil(double(e) / std::max(2.0 * mean, 1.0)));
            k = std::max<uint64_t>(1, std::min<uint64_t>(k, e / kBinAlign));  // e: whole 128-entry groups
            ub.back() = a;
            for (uint64_t t = 1; t <= k; ++t) {
                ub.push_back(a + (e / kBinAlign) * t / k * kBinAlign);
                uwin.push_back((uint32_t)w);
            }
        }
    }
    p.b_nunits = uwin.size();
    BN_TRY(hipMalloc((void **)&p.d_b_seg, (nseg + 1) * 8));
    BN_TRY(hipMemcpyAsync(p.d_b_seg, seg.data(), (nseg + 1) * 8, hipMemcpyHostToDevice, s));
    BN_TRY(hipMalloc((void **)&p.d_b_ub, ub.size() * 8));
    BN_TRY(hipMemcpyAsync(p.d_b_ub, ub.data(), ub.size() * 8, hipMemcpyHostToDevice, s));
    BN_TRY(hipMalloc((void **)&p.d_b_uwin, std::max<size_t>(uwin.size(), 1) * 4));
    if (!uwin.empty())
        BN_TRY(hipMemcpyAsync(p.d_b_uwin, uwin.data(), uwin.size() * 4, hipMemcpyHostToDevice, s));
    const uint64_t alloc = std::max<uint64_t>(ent_pad, PER);
    BN_TRY(hipMalloc((void **)&p.d_b_val, alloc * sizeof(ValueType)));
    {
        // env SPMV_BIN_PROD_SKEW=bytes (measurement): the products start that far (a multiple of
        // 256 B) into their allocation, shifting their address bits against the entry arrays'
        const char *sk = ablation_env("SPMV_BIN_PROD_SKEW");
        const uint64_t skew = sk ? (uint64_t)std::strtoull(sk, nullptr, 10) / 256 * 256 : 0;
        BN_TRY(hipMalloc(&p.d_b_prod_alloc, alloc * sizeof(ValueType) + skew));
        p.d_b_prod = reinterpret_cast<ValueType *>(static_cast<unsigned char *>(p.d_b_prod_alloc) + skew);
    }
    BN_TRY(hipMalloc((void **)&p.d_b_colw, alloc * 2));
    BN_TRY(hipMalloc((void **)&p.d_b_rowp, alloc * (delta ? 1 : 2)));
    if (nnz && delta) {
        hipLaunchKernelGGL((k_bin_scatter_delta<ValueType>), dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s,
                           d_k64s, d_idxs, d_pscan, d_soff, nnz, P, (uint32_t)W0, (uint32_t)W1, d_col_src, d_val_src, p.d_b_seg,
                           p.d_b_val, p.d_b_colw, reinterpret_cast<uint8_t *>(p.d_b_rowp));
        BN_TRY(hipGetLastError());
        BN_TRY(hipMemcpyAsync(d_esc, esc.data(), nseg * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL((k_bin_pad<ValueType, true>), dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, nseg,
                           p.d_b_seg, d_cnt, d_esc, p.d_b_val, p.d_b_colw, (void *)p.d_b_rowp);
        BN_TRY(hipGetLastError());
    } else if (nnz) {
        BN_TRY(hipMalloc((void **)&d_cur, nseg * 4));
        BN_TRY(hipMemsetAsync(d_cur, 0, nseg * 4, s));
        hipLaunchKernelGGL((k_bin_scatter<ValueType>), dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_key,
                           d_rowp_tmp, d_col_src, d_val_src, nnz, P, (uint32_t)W0, (uint32_t)W1, p.d_b_seg, d_cur, p.d_b_val,
                           p.d_b_colw, reinterpret_cast<uint16_t *>(p.d_b_rowp));
        BN_TRY(hipGetLastError());
        hipLaunchKernelGGL((k_bin_pad<ValueType, false>), dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, nseg,
                           p.d_b_seg, d_cnt, (const uint32_t *)nullptr, p.d_b_val, p.d_b_colw, (void *)p.d_b_rowp);
        BN_TRY(hipGetLastError());
    }
    BN_TRY(hipStreamSynchronize(s));
    cleanup();
#undef BN_TRY
    return 0;
}

}  // namespace spmvhw

#ifdef SPMV_ABLATIONS
// measurement build only: n words of pass `pass`'s workgroup timeline (4 per workgroup)
extern "C" int spmv_abl_bin_times(int pass, unsigned long long *out, unsigned n)
{
    if (!out || pass < 0 || pass > 1 || n > 4 * 4096)
        return 1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(spmvhw::g_abl_bin), size_t(n) * 8, size_t(pass) * 4 * 4096 * 8,
                               hipMemcpyDeviceToHost) != hipSuccess;
}
#endif
