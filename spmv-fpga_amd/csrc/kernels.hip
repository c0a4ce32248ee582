// HIP kernels of the MI355X SpMV hot path (gfx950, wave64).
//
// Replaces the reference's per-column-block FPGA dataflow
//   read_data_submatrix (spmv.cpp:6-34) -> stream_data_col_ind / stream_data_values
//   (spmv.cpp:36-64) -> compute_results (spmv.cpp:66-104) -> write_back_results
//   (spmv.cpp:106-120), and the host scatter accum_results (csr_hw.cpp:1531-1565),
// with one flat, nnz-balanced pass over the matrix:
//
//   k_spmv_tiles: one wave per 512-entry tile. Coalesced 1-KiB dwordx4 wave loads of col/val
//     (read_data_submatrix + stream_data_*), a register gather of x, lane-local products and a
//     segmented inclusive scan across the 64 lanes keyed by the row-end bitmap
//     (compute_results: the reference emits a row sum when the row-end bit of a group is set,
//     spmv.cpp:99-102). Row sums are stored straight to y at their row (write_back_results +
//     accum_results); a row that crosses a tile boundary leaves its partial sums in head/tail.
//   k_fixup: one thread per tile completes every row that crossed a tile boundary, adding the
//     partials in tile order (deterministic, no atomics).
// Roofline: HBM-bound gather, no MFMA.
#include "spmv_internal.hpp"

namespace spmvhw {

__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Streamed (read-once) loads: NT=true marks them non-temporal so they do not displace the x
// vector from L2 / Infinity Cache (MI355X_MICROARCH.md "nt-weights").
template <bool NT, typename T>
__device__ __forceinline__ T ld(const T *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T *p, T v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// 4 consecutive logical entries [kb + 4*lane, +4) of a wave step.
template <bool NT>
__device__ __forceinline__ void load_vals(const double *__restrict__ val, uint64_t kb, int lane,
                                          double (&v)[4])
{
    // fp64 pair-interleaved layout: dev[kb + j*128 + 2*lane + i] = logical[kb + 4*lane + 2*j + i]
    const f64x2 a = ld<NT>(reinterpret_cast<const f64x2 *>(val + kb + 2 * lane));
    const f64x2 b = ld<NT>(reinterpret_cast<const f64x2 *>(val + kb + 128 + 2 * lane));
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}
template <bool NT>
__device__ __forceinline__ void load_vals(const float *__restrict__ val, uint64_t kb, int lane,
                                          float (&v)[4])
{
    const f32x4 a = ld<NT>(reinterpret_cast<const f32x4 *>(val + kb + 4 * lane));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}

template <bool NTY, typename V>
__device__ __forceinline__ void emit(V sum, uint32_t r, bool to_head, V *__restrict__ head,
                                     uint64_t t, const uint32_t *__restrict__ row_id,
                                     V *__restrict__ y)
{
    if (to_head)
        head[t] = sum;
    else
        st<NTY>(y + (row_id ? row_id[r] : r), sum);
}

// VAR bit 0: non-temporal streamed loads (col, val, row-end bits); bit 1: non-temporal y stores.
// CB = bytes per stored column: 4 = absolute (col), 2 / 1 = offsets (colnar) from the tile's
// base column (tile_cbase); CB = 3 = clustered 16-bit: (cluster << 14) | offset from one of the
// tile's four bases (tile_cbase[4 t + cluster]), for tiles whose columns fall into up to four
// narrow clusters (3-D stencils: one cluster per grid plane).
template <typename V, int U, int VAR, int CB>
__global__ __launch_bounds__(kBlockThreads) void k_spmv_tiles(
    const uint32_t *__restrict__ col, const void *__restrict__ colnar, const uint32_t *__restrict__ tile_cbase,
    const V *__restrict__ val, const uint32_t *__restrict__ rowend,
    const uint32_t *__restrict__ tile_info, const uint32_t *__restrict__ row_id,
    const V *__restrict__ x, V *__restrict__ y, V *__restrict__ head, V *__restrict__ tail,
    uint64_t nnz, uint64_t ntiles, uint32_t xcd_chunk)
{
    const int lane = threadIdx.x & (kWave - 1);
    // XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin, so workgroup b runs
    // on XCD b % 8; with xcd_chunk > 0 that XCD takes the contiguous block range
    // [(b % 8) * xcd_chunk, +xcd_chunk) in order, and rows that share x lines (neighbouring
    // tiles) meet in one XCD's L2 instead of being fetched by all eight
    const uint64_t blk = xcd_chunk ? (uint64_t)(blockIdx.x % 8u) * xcd_chunk + blockIdx.x / 8u : blockIdx.x;
    const uint64_t t = blk * (kBlockThreads / kWave) + (threadIdx.x >> 6);
    if (t >= ntiles)
        return;  // wave-uniform
    const uint64_t k0 = t * (uint64_t)(U * kStep);

    // ---- issue every streaming load of the tile first (memory-level parallelism) ----
    uint32_t c[U][4];
    V v[U][4];
    uint32_t fl[U];
    const uint32_t cbase = (CB == 1 || CB == 2) ? tile_cbase[t] : 0u;
    uint32_t cb4[4] = {0u, 0u, 0u, 0u};
    if constexpr (CB == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            cb4[k] = tile_cbase[4 * t + k];  // wave-uniform: scalar loads
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t kb = k0 + (uint64_t)u * kStep;
        if constexpr (CB == 2) {
            const u16x4 cc = ld<(VAR & 1) != 0>(reinterpret_cast<const u16x4 *>(colnar) + (kb / 4 + lane));
            c[u][0] = cbase + cc.x; c[u][1] = cbase + cc.y; c[u][2] = cbase + cc.z; c[u][3] = cbase + cc.w;
        } else if constexpr (CB == 3) {
            const u16x4 cc = ld<(VAR & 1) != 0>(reinterpret_cast<const u16x4 *>(colnar) + (kb / 4 + lane));
            const uint32_t w4[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = w4[j] >> 14;
                const uint32_t b = k == 0 ? cb4[0] : k == 1 ? cb4[1] : k == 2 ? cb4[2] : cb4[3];
                c[u][j] = b + (w4[j] & 0x3FFFu);
            }
        } else if constexpr (CB == 1) {
            const uint32_t cc = ld<(VAR & 1) != 0>(reinterpret_cast<const uint32_t *>(colnar) + (kb / 4 + lane));
            c[u][0] = cbase + (cc & 0xFFu); c[u][1] = cbase + ((cc >> 8) & 0xFFu);
            c[u][2] = cbase + ((cc >> 16) & 0xFFu); c[u][3] = cbase + (cc >> 24);
        } else {
            const u32x4 cc = ld<(VAR & 1) != 0>(reinterpret_cast<const u32x4 *>(col + kb + 4 * lane));
            c[u][0] = cc.x; c[u][1] = cc.y; c[u][2] = cc.z; c[u][3] = cc.w;
        }
        load_vals<(VAR & 1) != 0>(val, kb, lane, v[u]);
        fl[u] = (ld<(VAR & 1) != 0>(rowend + (kb >> 5) + (lane >> 3)) >> ((lane & 7) * 4)) & 0xFu;
    }
    V xv[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            xv[u][j] = x[c[u][j]];

    const uint32_t info = tile_info[t];
    uint32_t rowc = info >> 1;          // compact row of the tile's first entry
    bool pending = (info & 1u) != 0;    // first row end of the tile closes a row begun earlier
    bool last_is_end = false;
    V carry = V(0);

#pragma unroll
    for (int u = 0; u < U; ++u) {
        V p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            p[j] = v[u][j] * xv[u][j];
        const uint32_t f = fl[u];

        // lane-local sum of the entries after the lane's last row end
        V o = p[0];
        o = (f & 1u) ? p[1] : o + p[1];
        o = (f & 2u) ? p[2] : o + p[2];
        o = (f & 4u) ? p[3] : o + p[3];
        o = (f & 8u) ? V(0) : o;
        int closed = f != 0u;

        // segmented inclusive scan across the wave: (I,F) <- (I_prev,F_prev) (+) (I,F)
        V I = o;
        int F = closed;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const V In = __shfl_up(I, d, kWave);
            const int Fn = __shfl_up(F, d, kWave);
            if (lane >= d) {
                I = F ? I : In + I;
                F = F | Fn;
            }
        }
        V ex = __shfl_up(I, 1, kWave);
        int fx = __shfl_up(F, 1, kWave);
        if (lane == 0) {
            ex = V(0);
            fx = 0;
        }
        if (!fx)
            ex = carry + ex;

        const uint64_t b0 = __ballot(f & 1u), b1 = __ballot(f & 2u);
        const uint64_t b2 = __ballot(f & 4u), b3 = __ballot(f & 8u);
        const uint64_t bany = b0 | b1 | b2 | b3;
        uint32_t r = rowc + lanes_below(b0) + lanes_below(b1) + lanes_below(b2) + lanes_below(b3);
        bool to_head = pending && bany != 0 && lane == (int)(__ffsll((unsigned long long)bany) - 1);

        V run = ex;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            run = run + p[j];
            if (f & (1u << j)) {
                emit<(VAR & 2) != 0>(run, r, to_head, head, t, row_id, y);
                to_head = false;
                ++r;
                run = V(0);
            }
        }

        const V I63 = __shfl(I, kWave - 1, kWave);
        const int F63 = __shfl(F, kWave - 1, kWave);
        carry = F63 ? I63 : carry + I63;
        rowc += (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
        if (bany)
            pending = false;
        last_is_end = (b3 >> 63) & 1ull;
    }

    if (lane == 0 && !last_is_end && (k0 + (uint64_t)(U * kStep) < nnz))
        tail[t] = carry;  // the tile ends inside a row that continues in tile t+1
}

// Completes every row that crosses a tile boundary. The crossings are structural (known when
// the plan is built): crossing c covers tiles [first, last]; its sum is tail[first] + tail[first+1]
// + ... + tail[last-1] + head[last], added in tile order (deterministic, no atomics).
template <typename V>
__global__ __launch_bounds__(256) void k_fixup(const uint32_t *__restrict__ cross, uint64_t ncross,
                                               const V *__restrict__ head, const V *__restrict__ tail,
                                               const uint32_t *__restrict__ row_id, V *__restrict__ y)
{
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncross)
        return;
    const uint32_t row = cross[3 * c], first = cross[3 * c + 1], last = cross[3 * c + 2];
    V acc = tail[first];
    for (uint32_t j = first + 1; j < last; ++j)
        acc = acc + tail[j];
    acc = acc + head[last];
    y[row_id ? row_id[row] : row] = acc;
}

// Copies logical CSR col/val into the padded hw representation (fp64: pair-interleaved).
template <typename V>
__global__ void k_pack(const IndexType *__restrict__ col_src, const V *__restrict__ val_src,
                       uint64_t nnz, uint64_t nnz_pad, uint32_t ncols, uint32_t *__restrict__ col,
                       V *__restrict__ val, uint32_t *__restrict__ bad)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz_pad)
        return;
    const bool in = k < nnz;
    uint32_t c = in ? col_src[k] : 0u;
    if (c >= ncols)  // validated before packing; never let an out-of-range index reach a gather
        c = 0u;
    col[k] = c;
    uint64_t dst = k;
    if (sizeof(V) == 8) {
        const uint64_t base = k & ~(uint64_t)(kStep - 1);
        const uint32_t w = (uint32_t)(k & (kStep - 1));
        const uint32_t ln = w >> 2, e = w & 3u;
        dst = base + (e >> 1) * 128u + 2u * ln + (e & 1u);
    }
    val[dst] = in ? val_src[k] : V(0);
}

hipError_t launch_spmv(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.ntiles == 0)
        return hipSuccess;
    const uint64_t waves_per_block = kBlockThreads / kWave;
    const uint64_t nblk = (p.ntiles + waves_per_block - 1) / waves_per_block;
    const uint32_t xcd_chunk = p.tile_xcd ? (uint32_t)((nblk + 7) / 8) : 0u;
    const uint64_t blocks = xcd_chunk ? 8ull * xcd_chunk : nblk;
#define SPMV_LAUNCH(VAR, CB)                                                                      \
    launch_or_warm(warm, k_spmv_tiles<ValueType, kTileSteps, VAR, CB>, dim3((unsigned)blocks),       \
                       dim3(kBlockThreads), 0, s, p.d_col, p.d_colnar, p.d_tile_cbase, p.d_val,     \
                       p.d_rowend, p.d_tile_info, p.d_row_id, d_x, d_y, p.d_head, p.d_tail, p.nnz, \
                       p.ntiles, xcd_chunk)
#define SPMV_VARIANTS(CB)                    \
    switch (p.variant & 3) {                 \
    case 0: SPMV_LAUNCH(0, CB); break;       \
    case 1: SPMV_LAUNCH(1, CB); break;       \
    case 2: SPMV_LAUNCH(2, CB); break;       \
    default: SPMV_LAUNCH(3, CB); break;      \
    }
    if (p.tile_col_bytes == 1) {
        SPMV_VARIANTS(1)
    } else if (p.tile_col_bytes == 2 && p.tile_clustered) {
        SPMV_VARIANTS(3)
    } else if (p.tile_col_bytes == 2) {
        SPMV_VARIANTS(2)
    } else {
        SPMV_VARIANTS(4)
    }
#undef SPMV_VARIANTS
#undef SPMV_LAUNCH
    return hipGetLastError();
}

hipError_t launch_fixup(const spmv_plan &p, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.ncross == 0)
        return hipSuccess;
    const uint64_t blocks = (p.ncross + 255) / 256;
    launch_or_warm(warm, k_fixup<ValueType>, dim3((unsigned)blocks), dim3(256), 0, s, p.d_cross, p.ncross,
                       p.d_head, p.d_tail, p.d_row_id, d_y);
    return hipGetLastError();
}

__global__ void k_validate(const IndexType *__restrict__ col, uint64_t nnz, uint32_t ncols,
                           uint32_t *__restrict__ bad)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nnz && col[k] >= ncols)
        atomicOr(bad, 1u);
}

hipError_t launch_validate(const IndexType *d_col, uint64_t nnz, uint32_t ncols, uint32_t *d_bad, hipStream_t s)
{
    if (nnz == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_validate, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, d_col, nnz, ncols, d_bad);
    return hipGetLastError();
}

hipError_t launch_pack(const IndexType *d_col_src, const ValueType *d_val_src, uint64_t nnz,
                       uint64_t nnz_pad, uint32_t ncols, uint32_t *d_col, ValueType *d_val,
                       uint32_t *d_bad, hipStream_t s)
{
    if (nnz_pad == 0)
        return hipSuccess;
    const uint64_t blocks = (nnz_pad + 255) / 256;
    hipLaunchKernelGGL((k_pack<ValueType>), dim3((unsigned)blocks), dim3(256), 0, s, d_col_src,
                       d_val_src, nnz, nnz_pad, ncols, d_col, d_val, d_bad);
    return hipGetLastError();
}

// One wave per tile: min / max column of the tile's real entries (k < nnz).
__global__ __launch_bounds__(256) void k_tile_span(const uint32_t *__restrict__ col, uint64_t nnz, uint64_t ntiles,
                                                   uint32_t *__restrict__ cbase, uint32_t *__restrict__ maxspan)
{
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= ntiles)
        return;
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    for (int j = 0; j < kTileNnz / kWave; ++j) {
        const uint64_t k = t * kTileNnz + (uint64_t)j * kWave + lane;
        if (k < nnz) {
            const uint32_t c = col[k];
            lo = c < lo ? c : lo;
            hi = c > hi ? c : hi;
        }
    }
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t l2 = __shfl_xor(lo, d, kWave), h2 = __shfl_xor(hi, d, kWave);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if (lane == 0) {
        if (lo == 0xFFFFFFFFu)
            lo = hi = 0u;  // a tile of padding only
        cbase[t] = lo;
        atomicMax(maxspan, hi - lo);
    }
}

// One wave per tile: up to four cluster bases. base_0 = the tile's min column; base_k = the min
// column >= base_{k-1} + 16384. Every column then lies within 16384 of the largest base not
// above it, unless some column is >= base_3 + 16384 (*bad |= 1: the plan keeps 32-bit columns).
__global__ __launch_bounds__(256) void k_tile_clusters(const uint32_t *__restrict__ col, uint64_t nnz, uint64_t ntiles,
                                                       uint32_t *__restrict__ bases, uint32_t *__restrict__ bad)
{
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= ntiles)
        return;
    uint32_t cols[kTileNnz / kWave];
#pragma unroll
    for (int j = 0; j < kTileNnz / kWave; ++j) {
        const uint64_t k = t * kTileNnz + (uint64_t)j * kWave + lane;
        cols[j] = k < nnz ? col[k] : 0xFFFFFFFFu;  // padding: not a column
    }
    uint64_t lim = 0;  // next base = min column >= lim
    uint32_t base[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < kTileNnz / kWave; ++j)
            if (cols[j] != 0xFFFFFFFFu && cols[j] >= lim && cols[j] < m)
                m = cols[j];
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t o = __shfl_xor(m, d, kWave);
            m = o < m ? o : m;
        }
        base[b] = m == 0xFFFFFFFFu ? (b ? base[b - 1] : 0u) : m;
        lim = m == 0xFFFFFFFFu ? lim : uint64_t(m) + 16384u;
    }
    bool over = false;
#pragma unroll
    for (int j = 0; j < kTileNnz / kWave; ++j)
        over |= cols[j] != 0xFFFFFFFFu && uint64_t(cols[j]) >= lim;
    if (__ballot(over) && lane == 0)
        atomicOr(bad, 1u);
    if (lane < 4)
        bases[4 * t + lane] = base[lane];
}

__global__ void k_cluster_encode(const uint32_t *__restrict__ col, uint64_t nnz, uint64_t nnz_pad,
                                 const uint32_t *__restrict__ bases, uint16_t *__restrict__ out)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz_pad)
        return;
    const uint32_t *b = bases + 4 * (k / kTileNnz);
    if (k >= nnz) {
        out[k] = 0;  // padding: gathers x[base_0] with value 0 and no row end
        return;
    }
    const uint32_t c = col[k];
    uint32_t cl = 0;
#pragma unroll
    for (uint32_t j = 1; j < 4; ++j)
        if (b[j] <= c && b[j] > b[j - 1])
            cl = j;
    out[k] = (uint16_t)((cl << 14) | (c - b[cl]));
}

template <typename T>
__global__ void k_narrow(const uint32_t *__restrict__ col, uint64_t nnz, uint64_t nnz_pad,
                         const uint32_t *__restrict__ cbase, T *__restrict__ out)
{
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz_pad)
        return;
    // padding entries gather x[cbase] (a valid column) with value 0 and no row end
    out[k] = k < nnz ? (T)(col[k] - cbase[k / kTileNnz]) : (T)0;
}

hipError_t launch_tile_span(const uint32_t *d_col, uint64_t nnz, uint64_t ntiles, uint32_t *d_cbase,
                            uint32_t *d_maxspan, hipStream_t s)
{
    if (ntiles == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_tile_span, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, d_col, nnz, ntiles,
                       d_cbase, d_maxspan);
    return hipGetLastError();
}

hipError_t launch_tile_clusters(const uint32_t *d_col, uint64_t nnz, uint64_t ntiles, uint32_t *d_bases,
                                uint32_t *d_bad, hipStream_t s)
{
    if (ntiles == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_tile_clusters, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, d_col, nnz, ntiles,
                       d_bases, d_bad);
    return hipGetLastError();
}

hipError_t launch_cluster_encode(const uint32_t *d_col, uint64_t nnz, uint64_t nnz_pad, const uint32_t *d_bases,
                                 uint16_t *d_out, hipStream_t s)
{
    if (nnz_pad == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_cluster_encode, dim3((unsigned)((nnz_pad + 255) / 256)), dim3(256), 0, s, d_col, nnz,
                       nnz_pad, d_bases, d_out);
    return hipGetLastError();
}

hipError_t launch_narrow(const uint32_t *d_col, uint64_t nnz, uint64_t nnz_pad, const uint32_t *d_cbase,
                         void *d_out, int bytes, hipStream_t s)
{
    if (nnz_pad == 0)
        return hipSuccess;
    const dim3 grid((unsigned)((nnz_pad + 255) / 256)), block(256);
    if (bytes == 1)
        hipLaunchKernelGGL((k_narrow<uint8_t>), grid, block, 0, s, d_col, nnz, nnz_pad, d_cbase, (uint8_t *)d_out);
    else
        hipLaunchKernelGGL((k_narrow<uint16_t>), grid, block, 0, s, d_col, nnz, nnz_pad, d_cbase, (uint16_t *)d_out);
    return hipGetLastError();
}

}  // namespace spmvhw
