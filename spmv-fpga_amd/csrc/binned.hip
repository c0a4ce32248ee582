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
// (whole 128-byte lines for pass 1's wave loads and stores). Pad entries: value 0, column offset
// 0, row offset = the scratch slot `panel_rmax` (their product, possibly 0 * inf = NaN, never
// reaches y).
//   d_b_val   V[ent_pad]    values, window-major
//   d_b_colw  u16[ent_pad]  column - window base
//   d_b_rowp  u16[ent_pad]  row - panel base
//   d_b_prod  V[ent_pad]    products (scratch written by pass 1, read by pass 2)
//   d_b_seg   u64[nwin * npan + 1]  padded segment offsets, index w * npan + p
//   d_b_ub    u64[nunits + 1], d_b_uwin u32[nunits]: pass-1 work units (a window, or a piece of
//             a window holding > 2x the mean entries)
// Bytes per non-zero: fp32 4 + 2 read, 4 written, 4 + 2 read = 16; fp64 28. Both passes are
// HBM-bound (pass 1's reads and writes add up at ~6 TB/s). Measured on 10M x 10M / 160M
// (profiles/r02_binned.jsonl): fp32 0.457-0.51 ms against 0.60-0.62 ms for the sweep; fp64
// 0.80-0.86 ms against 0.78-0.79, so the automatic choice takes it for fp32 only (plan.cpp),
// and not for skewed matrices (a panel of long rows would serialise pass 2's LDS adds).
//
// fp32 rows: products rounded to fp32 (the reference's fp32 multiply), summed in fp64, rounded
// once. Like the sweep, the LDS adds land in timing order: y is not bitwise reproducible run to
// run (scaled error <= 1e-15 fp64 / one fp32 rounding).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
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

// Pass 1: unit u = entries [ub[u], ub[u+1]) of window uwin[u] (both multiples of PER).
// AL: x is 16-byte aligned, so the window is staged with 16-byte loads.
template <typename V, bool AL>
__global__ __launch_bounds__(kBinT) void k_bin_mul(const V *__restrict__ x, uint32_t ncols, uint32_t W,
                                                   const uint64_t *__restrict__ ub, const uint32_t *__restrict__ uwin,
                                                   const uint16_t *__restrict__ colw, const V *__restrict__ val,
                                                   V *__restrict__ prod)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *xs = reinterpret_cast<V *>(smem);
    typedef typename BinVec<V>::T VT;
    typedef typename BinVec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    const uint32_t u = blockIdx.x;
    const uint64_t c0 = (uint64_t)uwin[u] * W;
    const uint32_t wn = (uint32_t)std::min<uint64_t>(W, ncols - c0);  // columns of this window
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
                v[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(val + i));
                c[k] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(colw + i));
            }
        }
#pragma unroll
        for (int k = 0; k < kBinU; ++k) {
            const uint64_t i = s + k * STEP + lane * PER;
            if (i < e1) {
                VT pr;
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    pr[q] = v[k][q] * xs[c[k][q]];
                __builtin_nontemporal_store(pr, reinterpret_cast<VT *>(prod + i));
            }
        }
    }
}

// Pass 2: workgroup = panel p (rows [panel_row[p], panel_row[p+1])). Wave v takes windows v,
// v + 16, ...; its segments form one stream of 64-lane steps of PER entries (the last step of a
// segment masked), kBinD steps of loads in flight before the adds. The bounds of the wave's next
// 64 segments sit in a lane table (lane l: segment 64c + l) read with readlane, so crossing a
// segment costs no scalar load (whose wait would also drain the outstanding LDS adds).
template <typename V>
__global__ __launch_bounds__(kBinT) void k_bin_acc(const V *__restrict__ prod, const uint16_t *__restrict__ rowp,
                                                   const uint64_t *__restrict__ seg,
                                                   const uint32_t *__restrict__ panel_row, uint32_t nwin,
                                                   uint32_t npan, uint32_t slots, V *__restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *ys = reinterpret_cast<double *>(smem);
    typedef typename BinVec<V>::T VT;
    typedef typename BinVec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    constexpr uint32_t STEP = 64 * PER;
    constexpr uint32_t WAVES = kBinT / 64;
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
    while (o < nmine) {
        VT v[kBinD];
        IT r[kBinD];
        uint64_t at[kBinD], en[kBinD];
#pragma unroll
        for (int k = 0; k < kBinD; ++k) {
            while (pos >= end && o < nmine) {  // next non-empty segment (uniform)
                ++o;
                if (o < nmine) {
                    if ((o & 63) == 0)
                        table(o >> 6);
                    bounds(o, pos, end);
                }
            }
            at[k] = pos + lane * PER;
            en[k] = o < nmine ? end : 0;
            if (at[k] < en[k]) {
                v[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(prod + at[k]));
                r[k] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(rowp + at[k]));
            }
            pos += STEP;
        }
#pragma unroll
        for (int k = 0; k < kBinD; ++k) {
            if (at[k] < en[k]) {
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    atomicAdd(&ys[r[k][q]], (double)v[k][q]);
            }
        }
    }
    __syncthreads();
    const uint32_t r0 = panel_row[p], nr = panel_row[p + 1] - r0;
    for (uint32_t i = threadIdx.x; i < nr; i += kBinT)
        y[r0 + i] = (V)ys[i];
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
                           uint64_t nnz, const uint32_t *__restrict__ panel_row, uint32_t npan, uint32_t W,
                           uint32_t *__restrict__ key, uint16_t *__restrict__ rowp, uint32_t *__restrict__ cnt)
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
    const uint32_t k = (col[j] / W) * npan + lo;
    key[j] = k;
    rowp[j] = (uint16_t)(r - panel_row[lo]);
    atomicAdd(&cnt[k], 1u);
}

template <typename V>
__global__ void k_bin_scatter(const uint32_t *__restrict__ key, const uint16_t *__restrict__ rowp_in,
                              const IndexType *__restrict__ col, const V *__restrict__ val_in, uint64_t nnz,
                              uint32_t npan, uint32_t W, const uint64_t *__restrict__ seg,
                              uint32_t *__restrict__ cursor, V *__restrict__ val, uint16_t *__restrict__ colw,
                              uint16_t *__restrict__ rowp)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nnz)
        return;
    const uint32_t k = key[j];
    const uint64_t d = seg[k] + atomicAdd(&cursor[k], 1u);
    val[d] = val_in[j];
    colw[d] = (uint16_t)(col[j] - (k / npan) * W);
    rowp[d] = rowp_in[j];
}

// pad entries of every segment: value 0, column offset 0, the scratch row slot
template <typename V>
__global__ void k_bin_pad(uint64_t nseg, const uint64_t *__restrict__ seg, const uint32_t *__restrict__ cnt,
                          uint16_t scratch, V *__restrict__ val, uint16_t *__restrict__ colw,
                          uint16_t *__restrict__ rowp)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nseg)
        return;
    for (uint64_t d = seg[k] + cnt[k]; d < seg[k + 1]; ++d) {
        val[d] = V(0);
        colw[d] = 0;
        rowp[d] = scratch;
    }
}

}  // namespace

hipError_t launch_binned(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    if (p.b_nunits) {
        const size_t lds1 = size_t(p.b_W) * sizeof(ValueType);
        const bool al = (reinterpret_cast<uintptr_t>(d_x) & 15u) == 0;
        if (al || warm)
            launch_or_warm(warm, k_bin_mul<ValueType, true>, dim3((unsigned)p.b_nunits), dim3(kBinT), lds1, s, d_x,
                           (uint32_t)p.nr_cols, p.b_W, p.d_b_ub, p.d_b_uwin, p.d_b_colw, p.d_b_val, p.d_b_prod);
        if (!al || warm)
            launch_or_warm(warm, k_bin_mul<ValueType, false>, dim3((unsigned)p.b_nunits), dim3(kBinT), lds1, s, d_x,
                           (uint32_t)p.nr_cols, p.b_W, p.d_b_ub, p.d_b_uwin, p.d_b_colw, p.d_b_val, p.d_b_prod);
    }
    const size_t lds2 = (size_t(p.panel_rmax) + 1) * sizeof(double);
    launch_or_warm(warm, k_bin_acc<ValueType>, dim3((unsigned)p.npanels), dim3(kBinT), lds2, s, p.d_b_prod, p.d_b_rowp,
                   p.d_b_seg, p.d_panel_row, p.b_nwin, (uint32_t)p.npanels, p.panel_rmax + 1, d_y);
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
    // panels: y of <= rmax rows in LDS (fp64), plus the scratch slot of the pad entries
    const uint32_t rmax = (uint32_t)std::min<uint64_t>((kSweepLdsBytes - 256) / 8 - 1, 65534);
    std::vector<uint32_t> prow;
    for (uint64_t P = std::max<uint64_t>({1, (n + rmax - 1) / rmax, std::min<uint64_t>(cus, n)});; ++P) {
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
            if (e - r > rmax)
                ok = false;
            prow.push_back(e);
            r = e;
        }
        if (ok)
            break;
        if (P >= n) {
            set_error("build_binned: cannot form panels");
            return 1;
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
    const uint64_t nseg = nwin * P;
    if (nseg >= (1ull << 28)) {
        set_error("build_binned: too many (window, panel) segments");
        return 2;
    }
    p.npanels = P;
    p.panel_rmax = rmax_used;
    p.b_nwin = (uint32_t)nwin;
    p.b_W = (uint32_t)W;
    SPMV_TRY(hipMalloc((void **)&p.d_panel_row, (P + 1) * 4));
    SPMV_TRY(hipMemcpyAsync(p.d_panel_row, prow.data(), (P + 1) * 4, hipMemcpyHostToDevice, s));

    IndexType *d_rp = nullptr;
    uint32_t *d_key = nullptr, *d_cnt = nullptr, *d_cur = nullptr;
    uint16_t *d_rowp_tmp = nullptr;
    auto cleanup = [&]() {
        for (void *q : {(void *)d_rp, (void *)d_key, (void *)d_cnt, (void *)d_cur, (void *)d_rowp_tmp})
            if (q)
                (void)hipFree(q);
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
                           p.d_panel_row, P, (uint32_t)W, d_key, d_rowp_tmp, d_cnt);
        BN_TRY(hipGetLastError());
        BN_TRY(hipMemcpyAsync(cnt.data(), d_cnt, nseg * 4, hipMemcpyDeviceToHost, s));
        BN_TRY(hipStreamSynchronize(s));
    }
    // padded segment offsets (window-major), then the pass-1 units
    // Each window's range also starts on a 128-entry boundary (the last segment of the window
    // takes the extra pad entries): pass 1's 1-KiB wave loads and stores then cover whole
    // 128-byte lines instead of straddling them (partial-line stores).
    std::vector<uint64_t> seg(nseg + 1, 0);
    for (uint64_t k = 0; k < nseg; ++k) {
        seg[k + 1] = seg[k] + (cnt[k] + PER - 1) / PER * PER;
        if ((k + 1) % P == 0)
            seg[k + 1] = (seg[k + 1] + kBinAlign - 1) / kBinAlign * kBinAlign;
    }
    const uint64_t ent_pad = seg[nseg];
    p.ent_pad = ent_pad;
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
    BN_TRY(hipMalloc((void **)&p.d_b_prod, alloc * sizeof(ValueType)));
    BN_TRY(hipMalloc((void **)&p.d_b_colw, alloc * 2));
    BN_TRY(hipMalloc((void **)&p.d_b_rowp, alloc * 2));
    if (nnz) {
        BN_TRY(hipMalloc((void **)&d_cur, nseg * 4));
        BN_TRY(hipMemsetAsync(d_cur, 0, nseg * 4, s));
        hipLaunchKernelGGL((k_bin_scatter<ValueType>), dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_key,
                           d_rowp_tmp, d_col_src, d_val_src, nnz, P, (uint32_t)W, p.d_b_seg, d_cur, p.d_b_val,
                           p.d_b_colw, p.d_b_rowp);
        BN_TRY(hipGetLastError());
        hipLaunchKernelGGL((k_bin_pad<ValueType>), dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, nseg,
                           p.d_b_seg, d_cnt, (uint16_t)rmax_used, p.d_b_val, p.d_b_colw, p.d_b_rowp);
        BN_TRY(hipGetLastError());
    }
    BN_TRY(hipStreamSynchronize(s));
#undef BN_TRY
    cleanup();
    return 0;
}

}  // namespace spmvhw
