// Kernel 5 — "slices": one wave per 64 consecutive rows, entries stored slot-major.
//
// For matrices whose rows have similar lengths and local columns (finite-element / stencil
// matrices), the flagged tiles (kernels.hip) spend their x requests badly: a tile's wave
// instruction gathers for 64 entries of ~2-10 consecutive rows, i.e. for every stencil offset
// of those rows at once, so each instruction touches one x line per (offset cluster, row run)
// -- ~14 lines for a 27-point stencil. Here a wave owns 64 consecutive rows (lane = row) and
// walks their entries slot by slot: slot j holds entry j of every row, so one gather
// instruction covers the same stencil offset of 64 consecutive rows: 64 consecutive x values,
// 4 lines (fp64). The row sum stays in a register: no segmented scan, no tile fix-up.
// This is the reference's row-wise compute_results (spmv.cpp:66-104) with the rows of a CU's
// slice (csr_hw.cpp:459-468) mapped to the lanes of a wave.
//
// Representation (built on the GPU in O(nnz)):
//   slot_off u32[S+1]   slice s owns slots [slot_off[s], slot_off[s+1]): as many as its longest row
//   val V[64 * slots]   slots of a slice in pairs: entry (slot 2p+i, lane) at
//                       (slot_off[s] + 2p) * 64 + 2 * lane + i, so one 16-byte (fp64) / 8-byte
//                       (fp32) load per lane brings two slots; an odd last slot is stored plainly
//   off u8/u16[same]    column - sbase[slot] (the slot's smallest column): the reference's
//                       block-relative 16-bit column field (csr_hw.cpp:288-292), per slot;
//                       clustered u16 = (cluster << 14) | offset from one of the slot's four
//                       bases when a slot spans >= 65536 columns in <= 4 clusters of < 16384
//                       (the grid planes of a 3-D stencil); else u32 absolute columns (sbase 0)
//   sbase u32[slots]    wave-uniform: scalar loads
//   len u32[n]          row lengths: lanes past their row's end add nothing (padding entries
//                       have value 0 and column sbase, and a non-finite x there is masked out)
// Roofline: HBM stream of (sizeof(V) + OB) bytes per stored entry plus 4 B per row; the x
// requests are ~4 lines per 64 entries on stencils.
#include <algorithm>
#include <cstdlib>

#include "spmv_internal.hpp"

namespace spmvhw {

constexpr int kSliceThreads = 256;  // 4 waves = 4 slices per workgroup

typedef double sl_f64x2 __attribute__((ext_vector_type(2)));
typedef float sl_f32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t sl_u16x2 __attribute__((ext_vector_type(2)));
typedef uint8_t sl_u8x2 __attribute__((ext_vector_type(2)));

template <typename V>
struct SliceVec;
template <>
struct SliceVec<double> {
    typedef sl_f64x2 T;
};
template <>
struct SliceVec<float> {
    typedef sl_f32x2 T;
};
template <int OB>
struct SliceOff;
template <>
struct SliceOff<1> {
    typedef uint8_t S;
    typedef sl_u8x2 T;
};
template <>
struct SliceOff<2> {
    typedef uint16_t S;
    typedef sl_u16x2 T;
};
template <>
struct SliceOff<3> {  // clustered 16-bit: (cluster << 14) | offset from one of the slot's 4 bases
    typedef uint16_t S;
    typedef sl_u16x2 T;
};
template <>
struct SliceOff<4> {  // absolute 32-bit columns (sbase = 0), when a slot spans >= 65536 columns
    typedef uint32_t S;
    typedef uint32_t T __attribute__((ext_vector_type(2)));
};

// PU pairs of slots per iteration; every load of the iteration is issued before the first
// gather (pairs past the slice's end re-read its first pair and add nothing; TAIL: they are
// skipped by a wave-uniform branch instead). A: the row accumulator, fp64 by default; A = V for
// an fp32 matrix (env SPMV_SLICE_ACC=32) sums like spmv_gold in fp32. Each row's products are
// added in CSR order from +0, and the select between each multiply and its add keeps them
// apart (no fused multiply-add in the ISA), so y is bit for bit spmv_gold's when A == V.
template <typename V, int OB, int PU, bool TAIL = false, typename A = double>
__global__ __launch_bounds__(kSliceThreads) void k_spmv_slices(const V *__restrict__ val, const void *__restrict__ offv,
                                                             const uint32_t *__restrict__ sbase,
                                                             const uint32_t *__restrict__ slot_off,
                                                             const uint32_t *__restrict__ len, const V *__restrict__ x,
                                                             V *__restrict__ y, uint32_t nrows, uint32_t nslices)
{
    // separate multiply and add (no contraction to fma): the fp64 row sums are bitwise spmv_gold
    // (csr.cpp:184-194), as in gold.hip and blocked.hip
#pragma clang fp contract(off)
    typedef typename SliceVec<V>::T VT;
    typedef typename SliceOff<OB>::S OS;
    typedef typename SliceOff<OB>::T OT;
    const OS *__restrict__ off = reinterpret_cast<const OS *>(offv);
    const uint32_t s = blockIdx.x * (kSliceThreads / kWave) + (threadIdx.x >> 6);
    if (s >= nslices)
        return;  // wave-uniform
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t row = s * kWave + lane;
    const uint32_t j0 = __builtin_amdgcn_readfirstlane(slot_off[s]);
    const uint32_t L = __builtin_amdgcn_readfirstlane(slot_off[s + 1]) - j0;
    const uint32_t mylen = row < nrows ? len[row] : 0u;
    const uint32_t npairs = L / 2;
    A acc = A(0);
    for (uint32_t p = 0; p < npairs; p += PU) {
        VT v[PU];
        OT o[PU];
        uint32_t b0[PU], b1[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            if (TAIL && p + u >= npairs) {  // wave-uniform
                v[u] = VT(0);
                o[u] = OT(0);
                b0[u] = b1[u] = 0u;
                continue;
            }
            const uint32_t pp = p + u < npairs ? p + u : 0u;  // wave-uniform
            const uint64_t e = (uint64_t)(j0 + 2 * pp) * kWave + 2 * lane;
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(val + e));
            o[u] = __builtin_nontemporal_load(reinterpret_cast<const OT *>(off + e));
            if constexpr (OB == 3) {  // per-lane pick among the slot's 4 bases (scalar loads)
                const uint32_t *b = sbase + 4 * (j0 + 2 * pp);
                const uint32_t k0 = o[u].x >> 14, k1 = o[u].y >> 14;
                b0[u] = k0 == 0 ? b[0] : k0 == 1 ? b[1] : k0 == 2 ? b[2] : b[3];
                b1[u] = k1 == 0 ? b[4] : k1 == 1 ? b[5] : k1 == 2 ? b[6] : b[7];
            } else {
                b0[u] = sbase[j0 + 2 * pp];
                b1[u] = sbase[j0 + 2 * pp + 1];
            }
        }
        V xv0[PU], xv1[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            if (TAIL && p + u >= npairs) {  // wave-uniform: no gather for a skipped pair
                xv0[u] = xv1[u] = V(0);
                continue;
            }
            constexpr uint32_t m = OB == 3 ? 0x3FFFu : 0xFFFFFFFFu;
            xv0[u] = x[b0[u] + (o[u].x & m)];
            xv1[u] = x[b1[u] + (o[u].y & m)];
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const uint32_t j = 2 * (p + u);  // slot of the pair's first entry
            const A t0 = A(v[u].x) * A(xv0[u]);
            const A t1 = A(v[u].y) * A(xv1[u]);
            acc += (p + u < npairs && j < mylen) ? t0 : A(0);
            acc += (p + u < npairs && j + 1 < mylen) ? t1 : A(0);
        }
    }
    if (L & 1) {  // odd last slot, stored plainly
        const uint64_t e = (uint64_t)(j0 + L - 1) * kWave + lane;
        const V v = __builtin_nontemporal_load(val + e);
        const OS o = __builtin_nontemporal_load(off + e);
        uint32_t b;
        if constexpr (OB == 3) {
            const uint32_t *bb = sbase + 4 * (j0 + L - 1);
            const uint32_t k = o >> 14;
            b = k == 0 ? bb[0] : k == 1 ? bb[1] : k == 2 ? bb[2] : bb[3];
        } else {
            b = sbase[j0 + L - 1];
        }
        const V xv = x[b + (OB == 3 ? (o & 0x3FFFu) : (uint32_t)o)];
        const A t = A(v) * A(xv);
        acc += (L - 1 < mylen) ? t : A(0);
    }
    if (row < nrows)
        y[row] = V(acc);
}

hipError_t launch_slices(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    const uint32_t nsl = (uint32_t)p.nslices;
    const dim3 grid((nsl + kSliceThreads / kWave - 1) / (kSliceThreads / kWave));
#define SLV(OB, PU, TAIL)                                                                                        \
    launch_or_warm(warm, k_spmv_slices<ValueType, OB, PU, TAIL>, grid, dim3(kSliceThreads), 0, s,                 \
                   (const ValueType *)p.d_val, (const void *)p.d_colnar, (const uint32_t *)p.d_sbase,             \
                   (const uint32_t *)p.d_slot_off, (const uint32_t *)p.d_slice_len, d_x, d_y, p.nr_rows, nsl)
    // variant (spmv_plan_set_variant): 0 = 4 pairs per iteration, pairs past the slice's end
    // skipped (default: 27-point 0.450 vs 0.508 ms, 7-point 0.126 vs 0.131 when they re-read the
    // first pair); 1 = 2 pairs, 2 = 7 pairs, 3 = 4 pairs re-reading
#define SL(OB)                                                                                                   \
    do {                                                                                                         \
        if (p.variant == 1)                                                                                      \
            SLV(OB, 2, true);                                                                                    \
        else if (p.variant == 2)                                                                                 \
            SLV(OB, 7, true);                                                                                    \
        else if (p.variant == 3)                                                                                 \
            SLV(OB, 4, false);                                                                                   \
        else                                                                                                     \
            SLV(OB, 4, true);                                                                                    \
    } while (0)
    if constexpr (sizeof(ValueType) == 4) {
        if (p.slice_acc_native) {  // fp32 accumulator (default variant only)
#define SLF(OB)                                                                                                  \
    launch_or_warm(warm, k_spmv_slices<ValueType, OB, 4, true, ValueType>, grid, dim3(kSliceThreads), 0, s,       \
                   (const ValueType *)p.d_val, (const void *)p.d_colnar, (const uint32_t *)p.d_sbase,             \
                   (const uint32_t *)p.d_slot_off, (const uint32_t *)p.d_slice_len, d_x, d_y, p.nr_rows, nsl)
            if (p.slice_off_bytes == 1)
                SLF(1);
            else if (p.slice_off_bytes == 2 && p.slice_clustered)
                SLF(3);
            else if (p.slice_off_bytes == 2)
                SLF(2);
            else
                SLF(4);
#undef SLF
            return hipGetLastError();
        }
    }
    if (p.slice_off_bytes == 1)
        SL(1);
    else if (p.slice_off_bytes == 2 && p.slice_clustered)
        SL(3);
    else if (p.slice_off_bytes == 2)
        SL(2);
    else
        SL(4);
#undef SL
#undef SLV
    return hipGetLastError();
}

// ---- build ----

__device__ __forceinline__ uint64_t slice_pos(uint32_t j0, uint32_t L, uint32_t j, uint32_t lane)
{
    if (j < (L & ~1u))
        return (uint64_t)(j0 + (j & ~1u)) * kWave + 2 * lane + (j & 1u);
    return (uint64_t)(j0 + j) * kWave + lane;  // odd last slot
}

// pass 1: values (0 past the row's end) and absolute columns (0xFFFFFFFF past the end)
__global__ void k_slices_fill(const IndexType *__restrict__ rp, const IndexType *__restrict__ col,
                              const ValueType *__restrict__ valsrc, IndexType nrows, const uint32_t *__restrict__ slot_off,
                              ValueType *__restrict__ val, uint32_t *__restrict__ col32)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows)
        return;
    const uint32_t s = r / kWave, lane = r % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    const uint32_t b = rp[r], n = rp[r + 1] - b;
    for (uint32_t j = 0; j < L; ++j) {
        const uint64_t e = slice_pos(j0, L, j, lane);
        val[e] = j < n ? valsrc[b + j] : ValueType(0);
        col32[e] = j < n ? col[b + j] : 0xFFFFFFFFu;
    }
}

// lanes of the last slice past nrows: padding too
__global__ void k_slices_tail(IndexType nrows, uint32_t nslices, const uint32_t *__restrict__ slot_off,
                              ValueType *__restrict__ val, uint32_t *__restrict__ col32)
{
    const uint32_t r = nrows + blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nslices * (uint32_t)kWave)
        return;
    const uint32_t s = r / kWave, lane = r % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    for (uint32_t j = 0; j < L; ++j) {
        const uint64_t e = slice_pos(j0, L, j, lane);
        val[e] = ValueType(0);
        col32[e] = 0xFFFFFFFFu;
    }
}

// pass 2: per slot, the smallest column of its real entries (every slot has one: the slice's
// longest row fills all its slots) and the span
__global__ void k_slices_base(const uint32_t *__restrict__ slot_off, uint32_t nslices,
                              const uint32_t *__restrict__ col32, uint32_t *__restrict__ sbase,
                              uint32_t *__restrict__ maxspan)
{
    const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (s >= nslices)
        return;
    const uint32_t lane = threadIdx.x % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    uint32_t span = 0;
    for (uint32_t j = 0; j < L; ++j) {
        const uint32_t c = col32[slice_pos(j0, L, j, lane)];
        uint32_t lo = c, hi = c == 0xFFFFFFFFu ? 0u : c;
        for (int d = 1; d < kWave; d <<= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, d, kWave));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, d, kWave));
        }
        if (lane == 0)
            sbase[j0 + j] = lo;
        span = max(span, hi - lo);
    }
    if (lane == 0)
        atomicMax(maxspan, span);
}

// pass 3: offsets from the slot base (padding: 0)
template <typename OS>
__global__ void k_slices_off(const uint32_t *__restrict__ slot_off, uint32_t nslices,
                             const uint32_t *__restrict__ col32, const uint32_t *__restrict__ sbase, OS *__restrict__ off)
{
    const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (s >= nslices)
        return;
    const uint32_t lane = threadIdx.x % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    for (uint32_t j = 0; j < L; ++j) {
        const uint64_t e = slice_pos(j0, L, j, lane);
        const uint32_t c = col32[e];
        off[e] = (OS)(c == 0xFFFFFFFFu ? 0u : c - sbase[j0 + j]);
    }
}

// clustered form, per slot: up to 4 bases, each the smallest column >= the previous base +
// 16384 (14-bit offsets); *bad when a column lies beyond the fourth cluster
__global__ void k_slices_clusters(const uint32_t *__restrict__ slot_off, uint32_t nslices,
                                  const uint32_t *__restrict__ col32, uint32_t *__restrict__ sbase4,
                                  uint32_t *__restrict__ bad)
{
    const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (s >= nslices)
        return;
    const uint32_t lane = threadIdx.x % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    for (uint32_t j = 0; j < L; ++j) {
        const uint32_t c = col32[slice_pos(j0, L, j, lane)];  // 0xFFFFFFFF: padding
        uint32_t floor = 0, base[4];
        bool have = true;
        for (int k = 0; k < 4; ++k) {
            uint32_t lo = (c != 0xFFFFFFFFu && c >= floor && have) ? c : 0xFFFFFFFFu;
            for (int d = 1; d < kWave; d <<= 1)
                lo = min(lo, (uint32_t)__shfl_xor((int)lo, d, kWave));
            base[k] = lo == 0xFFFFFFFFu ? (k ? base[k - 1] : 0u) : lo;
            have = have && lo != 0xFFFFFFFFu;
            floor = lo == 0xFFFFFFFFu ? 0xFFFFFFFFu : (lo > 0xFFFFFFFFu - 16384u ? 0xFFFFFFFFu : lo + 16384u);
        }
        if (c != 0xFFFFFFFFu && floor != 0xFFFFFFFFu && c >= floor)
            atomicOr(bad, 1u);
        if (lane < 4)
            sbase4[4 * (j0 + j) + lane] = base[lane];
    }
}

__global__ void k_slices_off_cl(const uint32_t *__restrict__ slot_off, uint32_t nslices,
                                const uint32_t *__restrict__ col32, const uint32_t *__restrict__ sbase4,
                                uint16_t *__restrict__ off)
{
    const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (s >= nslices)
        return;
    const uint32_t lane = threadIdx.x % kWave;
    const uint32_t j0 = slot_off[s], L = slot_off[s + 1] - j0;
    for (uint32_t j = 0; j < L; ++j) {
        const uint64_t e = slice_pos(j0, L, j, lane);
        const uint32_t c = col32[e];
        uint32_t v = 0;
        if (c != 0xFFFFFFFFu) {
            const uint32_t *b = sbase4 + 4 * (j0 + j);
            uint32_t k = 0;
            for (uint32_t t = 1; t < 4; ++t)
                if (b[t] > b[k] && b[t] <= c)
                    k = t;
            v = (k << 14) | (c - b[k]);
        }
        off[e] = (uint16_t)v;
    }
}

// absolute-column form: padding markers become column 0 (their value is 0 and they are masked)
__global__ void k_slices_abs(uint32_t *__restrict__ col32, uint64_t E)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E && col32[e] == 0xFFFFFFFFu)
        col32[e] = 0u;
}

// 0 ok, 1 error, 2 not representable (more than 2^32 stored entries with the padding)
int build_slices(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                 hipStream_t s)
{
    const IndexType n = p.nr_rows;
    const uint64_t S = (uint64_t(n) + kWave - 1) / kWave;
    std::vector<uint32_t> so(S + 1, 0), len(n);
    uint64_t slots = 0;
    for (uint64_t q = 0; q < S; ++q) {
        uint32_t L = 0;
        for (uint64_t r = q * kWave; r < std::min<uint64_t>(n, (q + 1) * kWave); ++r) {
            len[r] = h_rp[r + 1] - h_rp[r];
            L = std::max(L, len[r]);
        }
        so[q] = (uint32_t)slots;
        slots += L;
        if (slots * kWave > 0xFFFFFFFFull) {
            set_error("slices: more than 2^32 stored entries with the per-slice padding");
            return 2;
        }
    }
    so[S] = (uint32_t)slots;
    if (p.slice_pad_limit > 0.0 && double(slots) * kWave > p.slice_pad_limit * double(p.nnz)) {
        set_error("slices: padding above the automatic choice's limit");
        return 2;  // decided from row_ptr alone, before any allocation
    }
    p.nslices = S;
    p.slice_slots = slots;
    const uint64_t E = slots * kWave;
    struct Tmp {
        void *q = nullptr;
        ~Tmp() { if (q) (void)hipFree(q); }
    } tcol, tspan, trp;
    SPMV_TRY(hipMalloc((void **)&p.d_slot_off, (S + 1) * 4));
    SPMV_TRY(hipMalloc((void **)&p.d_slice_len, std::max<size_t>(n, 1) * 4));
    SPMV_TRY(hipMalloc((void **)&p.d_val, std::max<uint64_t>(E, 2) * sizeof(ValueType)));
    SPMV_TRY(hipMalloc((void **)&p.d_sbase, std::max<uint64_t>(slots, 1) * 4));
    SPMV_TRY(hipMalloc(&tcol.q, std::max<uint64_t>(E, 2) * 4));
    SPMV_TRY(hipMalloc(&tspan.q, 4));
    SPMV_TRY(hipMalloc(&trp.q, (size_t(n) + 1) * 4));
    SPMV_TRY(hipMemcpyAsync(p.d_slot_off, so.data(), (S + 1) * 4, hipMemcpyHostToDevice, s));
    if (n)
        SPMV_TRY(hipMemcpyAsync(p.d_slice_len, len.data(), size_t(n) * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMemcpyAsync(trp.q, h_rp, (size_t(n) + 1) * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMemsetAsync(tspan.q, 0, 4, s));
    uint32_t span = 0;
    if (n) {
        hipLaunchKernelGGL(k_slices_fill, dim3((n + 255) / 256), dim3(256), 0, s, (const IndexType *)trp.q, d_col_src,
                           d_val_src, n, p.d_slot_off, p.d_val, (uint32_t *)tcol.q);
        SPMV_TRY(hipGetLastError());
        const uint32_t rest = (uint32_t)(S * kWave - n);
        if (rest)
            hipLaunchKernelGGL(k_slices_tail, dim3((rest + 63) / 64), dim3(64), 0, s, n, (uint32_t)S, p.d_slot_off,
                               p.d_val, (uint32_t *)tcol.q);
        SPMV_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_slices_base, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, s, p.d_slot_off, (uint32_t)S,
                           (const uint32_t *)tcol.q, p.d_sbase, (uint32_t *)tspan.q);
        SPMV_TRY(hipGetLastError());
        SPMV_TRY(hipMemcpyAsync(&span, tspan.q, 4, hipMemcpyDeviceToHost, s));
        SPMV_TRY(hipStreamSynchronize(s));
    }
    // env SPMV_SLICE_ACC=32 (fp32 library): fp32 row accumulator, bitwise spmv_gold in fp32
    {
        const char *aenv = std::getenv("SPMV_SLICE_ACC");
        p.slice_acc_native = sizeof(ValueType) == 4 && aenv && std::atoi(aenv) == 32;
    }
    // env SPMV_SLICE_NARROW=0 keeps 32-bit columns
    const char *nenv = ablation_env("SPMV_SLICE_NARROW");
    const bool narrow = !(nenv && nenv[0] == '0');
    int ob = !narrow ? 4 : span < 256u ? 1 : span < 65536u ? 2 : 4;
    if (ob == 4 && narrow && n) {  // try up to 4 clusters of 16384 columns per slot
        uint32_t *sb4 = nullptr, bad = 1;
        SPMV_TRY(hipMalloc((void **)&sb4, std::max<uint64_t>(slots, 1) * 16));
        SPMV_TRY(hipMemsetAsync(tspan.q, 0, 4, s));
        hipLaunchKernelGGL(k_slices_clusters, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, s, p.d_slot_off,
                           (uint32_t)S, (const uint32_t *)tcol.q, sb4, (uint32_t *)tspan.q);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(&bad, tspan.q, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess)
            e = hipStreamSynchronize(s);
        if (e != hipSuccess || bad) {
            (void)hipFree(sb4);
            SPMV_TRY(e);
        } else {
            SPMV_TRY(hipFree(p.d_sbase));
            p.d_sbase = sb4;
            SPMV_TRY(hipMalloc(&p.d_colnar, std::max<uint64_t>(E, 2) * 2));
            hipLaunchKernelGGL(k_slices_off_cl, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, s, p.d_slot_off,
                               (uint32_t)S, (const uint32_t *)tcol.q, (const uint32_t *)p.d_sbase,
                               (uint16_t *)p.d_colnar);
            SPMV_TRY(hipGetLastError());
            SPMV_TRY(hipStreamSynchronize(s));
            p.slice_off_bytes = 2;
            p.slice_clustered = true;
            return 0;
        }
    }
    p.slice_off_bytes = ob;
    if (ob == 4) {  // absolute columns: padding lanes get column 0 (masked), bases 0
        if (E) {
            hipLaunchKernelGGL(k_slices_abs, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, (uint32_t *)tcol.q, E);
            SPMV_TRY(hipGetLastError());
        }
        SPMV_TRY(hipMemsetAsync(p.d_sbase, 0, std::max<uint64_t>(slots, 1) * 4, s));
        p.d_colnar = tcol.q;
        tcol.q = nullptr;
    } else {
        SPMV_TRY(hipMalloc(&p.d_colnar, std::max<uint64_t>(E, 2) * ob));
        if (n) {
            if (ob == 1)
                hipLaunchKernelGGL(k_slices_off<uint8_t>, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, s, p.d_slot_off,
                                   (uint32_t)S, (const uint32_t *)tcol.q, p.d_sbase, (uint8_t *)p.d_colnar);
            else
                hipLaunchKernelGGL(k_slices_off<uint16_t>, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, s, p.d_slot_off,
                                   (uint32_t)S, (const uint32_t *)tcol.q, p.d_sbase, (uint16_t *)p.d_colnar);
            SPMV_TRY(hipGetLastError());
        }
    }
    SPMV_TRY(hipStreamSynchronize(s));
    return 0;
}

}  // namespace spmvhw
