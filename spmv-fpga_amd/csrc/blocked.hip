// Kernel 4 — "blocked": the reference's FPGA dataflow on MI355X, x staged in LDS per column block.
//
// The reference splits the columns into blocks of COLS_DIV_BLOCKS (util.h:41-59); for every
// block it builds a compact CSR of the rows that have entries there (create_block_matrix,
// csr_hw.cpp:190-265), copies the block of x into on-chip BRAM (spmv.cpp:180,280-294), streams
// the block's packed entries through compute_results (spmv.cpp:66-104: VF-wide groups, 15-bit
// block-relative column + row-end bit), writes one partial sum per compact row
// (write_back_results, spmv.cpp:106-120) and the host adds the blocks' partials into y in block
// order (accum_results, csr_hw.cpp:1531-1565). Here:
//   phase 1 (k_blocked_partials): one workgroup per work unit = (block b, range of b's compact
//     rows). It loads x[b*W, (b+1)*W) into LDS once (coalesced), then every thread sums one
//     compact row at a time in the FPGA order (groups of VF from 0, the last group padded with
//     0 * x[b*W]) and writes the row's block partial.
//   phase 2 (k_blocked_merge): one workgroup per row chunk loads the chunk's partials into LDS
//     and every thread adds its row's partials in block order from 0 (accum_results into a
//     zeroed y), then stores y.
// y is bit for bit the same as kernel 3 (k_spmv_fpga) and oracle.spmv_fpga_order for
// (SPMV_FPGA_VF, SPMV_FPGA_BLOCK).
//
// Representation (built on the GPU in O(nnz): one 64-bit and two 32-bit radix sorts):
//   bval V[nnz], bcol u16[nnz]  entries ordered by (block, row), CSR order inside; bcol is the
//                               column relative to the block (the reference's 15-bit field)
//   kptr u32[K+1]               first entry of each compact row (K = (row, block) pairs)
//   kpos u32[K]                 where phase 1 stores the compact row's partial: partials are laid
//                               out per row chunk (contiguous), block-major inside a chunk, so
//                               a unit's consecutive compact rows store to consecutive words
//   part V[K]                   the partials (scratch, rewritten every SpMV)
//   rp2 u32[n+1]                row-major offsets of each row's partials (row r has rp2[r+1] -
//                               rp2[r] blocks)
//   rl u16[K]                   row-major: index of each (row, block) partial inside its chunk
//   chunk_row u32[C+1]          row ranges of the chunks (<= kBlockedChunk partials each)
//   unit_blk u32[U], unit_k u32[U+1]  block and compact-row range of each phase-1 unit
// Roofline (power-law 10M/160M): ~1 partial per entry, so the partials cost 2 x sizeof(V) per
// entry on top of the 10 (fp64) / 6 (fp32) B of the entry stream and ~10 B of kptr/kpos/rl:
// this layout moves ~2x the CSR bytes, and phase 1 waits on two dependent loads per compact row
// (kptr, then the entry). Measured 1.80 ms fp64 (16384-column blocks) / 1.27 ms fp32 against
// 0.80 / 0.61 ms for the panel sweep: the reference's dataflow, kept as the
// faster FPGA-order mode for scattered matrices, not the fast path.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "spmv_internal.hpp"

namespace spmvhw {

constexpr int kBlockedThreads = 1024;                // phase 1: 16 waves, one block of x per CU
constexpr int kBlockedUnroll = 8;                    // compact rows per thread in flight
constexpr int kMergeThreads = 512;                   // phase 2
constexpr uint32_t kBlockedChunkBytes = 32 * 1024;  // phase 2: partials of one row chunk in LDS
constexpr uint32_t kBlockedChunk = kBlockedChunkBytes / sizeof(ValueType);
constexpr uint64_t kBlockedXLdsBytes = 128 * 1024;  // phase 1: one block of x in LDS, when it fits

// lds[0, n) <- g[0, n) by NT threads, U loads in flight per thread before the LDS stores (a plain
// copy loop waits on every load before the next one)
template <int NT, int U, typename T>
__device__ __forceinline__ void stage_to_lds(T *lds, const T *__restrict__ g, uint32_t n)
{
    for (uint32_t base = 0; base < n; base += U * NT) {
        T t[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + j * NT + threadIdx.x;
            t[j] = i < n ? g[i] : T(0);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + j * NT + threadIdx.x;
            if (i < n)
                lds[i] = t[j];
        }
    }
}

// FPGA-order running sums of one compact row (compute_results, spmv.cpp:74-103)
template <typename V, int VF>
struct FpgaSum {
    V sum = V(0), group = V(0);
    uint32_t in_group = 0;
    __device__ __forceinline__ void add(V prd)
    {
        group = group + prd;
        if (++in_group == (uint32_t)VF) {
            sum = sum + group;
            group = V(0);
            in_group = 0;
        }
    }
    __device__ __forceinline__ V close(V z) const { return in_group != 0 ? sum + (group + z) : sum; }
};

// Each thread sums kBlockedUnroll compact rows at a time (all their kptr / kpos / first-entry
// loads in flight together: the compact rows of a scattered matrix hold ~1 entry, so the loads
// of one row alone would leave the CU waiting on two dependent round trips per entry).
template <typename V, int VF, bool XLDS, int ABL = 0>
__global__ __launch_bounds__(kBlockedThreads) void k_blocked_partials(
    const V *__restrict__ bval, const uint16_t *__restrict__ bcol, const uint32_t *__restrict__ kptr,
    const uint32_t *__restrict__ kpos, const uint32_t *__restrict__ unit_blk, const uint32_t *__restrict__ unit_k,
    const V *__restrict__ x, uint32_t ncols, uint32_t width, V *__restrict__ part)
{
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *xs = reinterpret_cast<V *>(smem);
    const uint64_t c0 = (uint64_t)unit_blk[blockIdx.x] * width;
    const V *__restrict__ xg = x + c0;
    if constexpr (XLDS) {
        const uint32_t wb = (uint32_t)min<uint64_t>(width, ncols - c0);  // columns of this block
        stage_to_lds<kBlockedThreads, 16>(xs, xg, wb);
        __syncthreads();
    }
    auto xat = [&](uint32_t c) -> V {
        if constexpr (XLDS)
            return xs[c];
        else
            return xg[c];
    };
    const V z = V(0) * xg[0];  // the pad product 0 * x[block start] (+0, -0 or NaN)
    const uint32_t k1 = unit_k[blockIdx.x + 1];
    constexpr uint32_t U = kBlockedUnroll;
    for (uint32_t k = unit_k[blockIdx.x] + threadIdx.x; k < k1; k += U * kBlockedThreads) {
        uint32_t eb[U], ee[U], kp[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            const uint32_t kk = k + j * kBlockedThreads;
            const bool ok = kk < k1;
            eb[j] = ok ? kptr[kk] : 0u;
            ee[j] = ok ? kptr[kk + 1] : 0u;
            kp[j] = ABL == 1 ? kk : ok ? kpos[kk] : 0u;  // ABL 1 (measurement only): store in compact order
        }
        V v0[U];
        uint32_t c0v[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {  // first entries (entry 0 stands in for empty slots)
            v0[j] = bval[eb[j]];
            c0v[j] = bcol[eb[j]];
        }
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            if (eb[j] < ee[j]) {  // false only for slots past the unit's end
                FpgaSum<V, VF> acc;
                acc.add(v0[j] * xat(c0v[j]));
                uint32_t e = eb[j] + 1;
                for (; e + 8 <= ee[j]; e += 8) {  // long compact rows: 8 entries' loads in flight
                    V v[8];
                    uint32_t c[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        v[i] = bval[e + i];
                        c[i] = bcol[e + i];
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        acc.add(v[i] * xat(c[i]));
                }
                for (; e < ee[j]; ++e)
                    acc.add(bval[e] * xat(bcol[e]));
                part[kp[j]] = acc.close(z);
            }
        }
    }
}

// The chunk's partials and their row-major slot indices are staged in LDS; then each thread
// adds its rows' partials in block order.
template <typename V>
__global__ __launch_bounds__(kMergeThreads) void k_blocked_merge(const V *__restrict__ part,
                                                                 const uint32_t *__restrict__ rp2,
                                                                 const uint16_t *__restrict__ rl,
                                                                 const uint32_t *__restrict__ chunk_row,
                                                                 V *__restrict__ y)
{
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *ps = reinterpret_cast<V *>(smem);
    uint16_t *rls = reinterpret_cast<uint16_t *>(ps + kBlockedChunk);
    const uint32_t r0 = chunk_row[blockIdx.x], r1 = chunk_row[blockIdx.x + 1];
    const uint32_t q0 = rp2[r0], nq = rp2[r1] - q0;
    stage_to_lds<kMergeThreads, 8>(ps, part + q0, nq);
    stage_to_lds<kMergeThreads, 8>(rls, rl + q0, nq);
    __syncthreads();
    for (uint32_t r = r0 + threadIdx.x; r < r1; r += kMergeThreads) {
        V acc = V(0);
        const uint32_t qe = rp2[r + 1] - q0;
        uint32_t q = rp2[r] - q0;
        for (; q + 8 <= qe; q += 8) {  // rows over many blocks: 8 LDS reads in flight, in-order adds
            V t[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                t[i] = ps[rls[q + i]];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc = acc + t[i];
        }
        for (; q < qe; ++q)
            acc = acc + ps[rls[q]];
        y[r] = acc;
    }
}

hipError_t launch_blocked(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    if (p.nunits) {
        const bool xlds = p.blocked_xlds;
        const size_t lds = xlds ? size_t(p.fpga_width) * sizeof(ValueType) : 0;
#define BK(VF)                                                                                                   \
    launch_or_warm(warm, xlds ? k_blocked_partials<ValueType, VF, true> : k_blocked_partials<ValueType, VF, false>, \
                   dim3((unsigned)p.nunits), dim3(kBlockedThreads), lds, s, (const ValueType *)p.d_val,             \
                   (const uint16_t *)p.d_colnar, (const uint32_t *)p.d_kptr, (const uint32_t *)p.d_kpos,           \
                   (const uint32_t *)p.d_unit_panel, (const uint32_t *)p.d_unit_ent, d_x, p.nr_cols, p.fpga_width,  \
                   p.d_bpart)
#ifdef SPMV_ABLATIONS
        if (p.variant == 1) {  // measurement-only ablation (tools library only): partials stored in compact-row order
            launch_or_warm(warm, k_blocked_partials<ValueType, 1, true, 1>, dim3((unsigned)p.nunits),
                           dim3(kBlockedThreads), lds, s, (const ValueType *)p.d_val, (const uint16_t *)p.d_colnar,
                           (const uint32_t *)p.d_kptr, (const uint32_t *)p.d_kpos, (const uint32_t *)p.d_unit_panel,
                           (const uint32_t *)p.d_unit_ent, d_x, p.nr_cols, p.fpga_width, p.d_bpart);
        } else
#endif
        switch (p.fpga_vf) {
        case 8: BK(8); break;
        case 4: BK(4); break;
        case 2: BK(2); break;
        default: BK(1); break;
        }
#undef BK
    }
    launch_or_warm(warm, k_blocked_merge<ValueType>, dim3((unsigned)p.nchunks), dim3(kMergeThreads),
                   size_t(kBlockedChunk) * (sizeof(ValueType) + 2), s,
                   (const ValueType *)p.d_bpart, (const uint32_t *)p.d_rp2, (const uint16_t *)p.d_rl,
                   (const uint32_t *)p.d_chunk_row, d_y);
    return hipGetLastError();
}

// ---- build ----

__global__ void k_blk_keys(const IndexType *__restrict__ rp, const IndexType *__restrict__ col, IndexType nrows,
                           uint32_t width, uint32_t rowbits, uint64_t *__restrict__ keys, uint32_t *__restrict__ idx)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows)
        return;
    for (IndexType j = rp[r]; j < rp[r + 1]; ++j) {
        keys[j] = ((uint64_t)(col[j] / width) << rowbits) | r;
        idx[j] = j;
    }
}

// sorted entry i: value, block-relative column, "starts a compact row" flag
__global__ void k_blk_gather(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ idx, uint64_t nnz,
                             const IndexType *__restrict__ col, const ValueType *__restrict__ val, uint32_t width,
                             uint32_t rowbits, ValueType *__restrict__ bval, uint16_t *__restrict__ bcol,
                             uint32_t *__restrict__ flag)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nnz)
        return;
    const uint32_t j = idx[i];
    const uint64_t key = keys[i];
    bval[i] = val[j];
    bcol[i] = (uint16_t)(col[j] - (uint32_t)(key >> rowbits) * width);
    flag[i] = (i == 0 || keys[i - 1] != key) ? 1u : 0u;
}

// compact row k = cidx[i] starts at sorted entry i
__global__ void k_blk_compact(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ flag,
                              const uint32_t *__restrict__ cidx, uint64_t nnz, uint32_t rowbits,
                              uint32_t *__restrict__ kptr, uint32_t *__restrict__ krow, uint32_t *__restrict__ kblk,
                              uint32_t *__restrict__ cnt)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nnz || !flag[i])
        return;
    const uint32_t k = cidx[i];
    const uint64_t key = keys[i];
    const uint32_t r = (uint32_t)(key & ((1ull << rowbits) - 1));
    kptr[k] = (uint32_t)i;
    krow[k] = r;
    kblk[k] = (uint32_t)(key >> rowbits);
    atomicAdd(&cnt[r], 1u);
}

// chunk of compact row k's row (keys for the by-chunk sort); first compact row of every block
__global__ void k_blk_chunk_keys(const uint32_t *__restrict__ krow, const uint32_t *__restrict__ kblk, uint32_t K,
                                 const uint32_t *__restrict__ chunk_row, uint32_t nchunks, uint32_t *__restrict__ ckey,
                                 uint32_t *__restrict__ iota, uint32_t *__restrict__ kb)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K)
        return;
    const uint32_t r = krow[k];
    uint32_t lo = 0, hi = nchunks;  // last c with chunk_row[c] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (chunk_row[mid] <= r)
            lo = mid;
        else
            hi = mid;
    }
    ckey[k] = lo;
    iota[k] = k;
    if (k == 0 || kblk[k - 1] != kblk[k])
        kb[kblk[k]] = k;
}

// by-chunk order: sorted position i is the bucket position of compact row order[i]
__global__ void k_blk_kpos(const uint32_t *__restrict__ order, uint32_t K, uint32_t *__restrict__ kpos)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < K)
        kpos[order[i]] = i;
}

// by-row order: sorted position q is the row-major slot of compact row order[q]
__global__ void k_blk_rl(const uint32_t *__restrict__ order, uint32_t K, const uint32_t *__restrict__ kpos,
                         const uint32_t *__restrict__ ckey, const uint32_t *__restrict__ chunk_row,
                         const uint32_t *__restrict__ rp2, uint16_t *__restrict__ rl)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= K)
        return;
    const uint32_t k = order[q];
    rl[q] = (uint16_t)(kpos[k] - rp2[chunk_row[ckey[k]]]);
}

__global__ void k_blk_take(const uint32_t *__restrict__ src, const uint32_t *__restrict__ at, uint32_t n,
                           uint32_t *__restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = src[at[i]];
}

int build_blocked(spmv_plan &p, const IndexType *h_rp, const IndexType *d_col_src, const ValueType *d_val_src,
                  hipStream_t s)
{
    const IndexType n = p.nr_rows;
    const uint64_t nnz = p.nnz;
    const uint32_t W = p.fpga_width;
    if (W > 65536) {
        set_error("blocked kernel: SPMV_FPGA_BLOCK above 65536 (columns are stored as 16-bit block offsets)");
        return 1;
    }
    if (nnz > 0x7FFFFFFFull || uint64_t(n) >= 0x7FFFFFFFull) {  // hipcub item counts are int
        set_error("blocked kernel: more than 2^31-1 non-zeros or rows in one slice");
        return 1;
    }
    const uint64_t B = (uint64_t(p.nr_cols) + W - 1) / W;
    if (B > kBlockedChunk) {
        set_error("blocked kernel: more column blocks than one row chunk holds");
        return 1;
    }
    p.blocked_xlds = uint64_t(W) * sizeof(ValueType) <= kBlockedXLdsBytes;
    uint32_t rowbits = 1;
    while (rowbits < 32 && (1ull << rowbits) < uint64_t(n))
        ++rowbits;
    uint32_t blkbits = 1;
    while ((1ull << blkbits) < B)
        ++blkbits;

    struct Bufs {
        std::vector<void *> v;
        void *get(size_t bytes)
        {
            void *q = nullptr;
            if (hipMalloc(&q, std::max<size_t>(bytes, 16)) != hipSuccess)
                return nullptr;
            v.push_back(q);
            return q;
        }
        ~Bufs()
        {
            for (void *q : v)
                (void)hipFree(q);
        }
    } tmp;
    auto need = [&](void *q) {
        if (!q)
            set_error("blocked kernel: device allocation failed");
        return q != nullptr;
    };
#define BK_TRY(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            set_error(std::string("build_blocked: ") + #x + ": " + hipGetErrorString(e_));     \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

    // row-major partial offsets and chunks need the per-row pair counts, so even an empty
    // matrix gets rp2 / chunk tables
    SPMV_TRY(hipMalloc((void **)&p.d_rp2, (size_t(n) + 1) * 4));
    uint32_t *cnt = (uint32_t *)tmp.get((size_t(n) + 1) * 4);
    if (!need(cnt))
        return 1;
    BK_TRY(hipMemsetAsync(cnt, 0, (size_t(n) + 1) * 4, s));
    uint32_t K = 0;
    uint32_t *krow = nullptr, *kblk = nullptr;
    if (nnz) {
        IndexType *d_rp = (IndexType *)tmp.get((size_t(n) + 1) * 4);
        uint64_t *k0 = (uint64_t *)tmp.get(nnz * 8), *k1 = (uint64_t *)tmp.get(nnz * 8);
        uint32_t *i0 = (uint32_t *)tmp.get(nnz * 4), *i1 = (uint32_t *)tmp.get(nnz * 4);
        if (!need(d_rp) || !need(k0) || !need(k1) || !need(i0) || !need(i1))
            return 1;
        BK_TRY(hipMemcpyAsync(d_rp, h_rp, (size_t(n) + 1) * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_blk_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_rp, d_col_src, n, W,
                           rowbits, k0, i0);
        BK_TRY(hipGetLastError());
        size_t tb = 0;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, i0, i1, (int)nnz, 0, (int)(rowbits + blkbits), s));
        void *t = tmp.get(tb);
        if (!need(t))
            return 1;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(t, tb, k0, k1, i0, i1, (int)nnz, 0, (int)(rowbits + blkbits), s));
        SPMV_TRY(hipMalloc((void **)&p.d_val, nnz * sizeof(ValueType)));
        SPMV_TRY(hipMalloc(&p.d_colnar, nnz * 2));
        uint32_t *flag = i0, *cidx = (uint32_t *)k0;  // reuse: i0 and k0 are free after the sort
        hipLaunchKernelGGL(k_blk_gather, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, k1, i1, nnz,
                           d_col_src, d_val_src, W, rowbits, p.d_val, (uint16_t *)p.d_colnar, flag);
        BK_TRY(hipGetLastError());
        tb = 0;
        BK_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, cidx, (int)nnz, s));
        t = tmp.get(tb);
        if (!need(t))
            return 1;
        BK_TRY(hipcub::DeviceScan::ExclusiveSum(t, tb, flag, cidx, (int)nnz, s));
        uint32_t last[2] = {0, 0};
        BK_TRY(hipMemcpyAsync(&last[0], cidx + nnz - 1, 4, hipMemcpyDeviceToHost, s));
        BK_TRY(hipMemcpyAsync(&last[1], flag + nnz - 1, 4, hipMemcpyDeviceToHost, s));
        BK_TRY(hipStreamSynchronize(s));
        K = last[0] + last[1];
        SPMV_TRY(hipMalloc((void **)&p.d_kptr, (size_t(K) + 1) * 4));
        krow = (uint32_t *)tmp.get(size_t(K) * 4);
        kblk = (uint32_t *)tmp.get(size_t(K) * 4);
        if (!need(krow) || !need(kblk))
            return 1;
        hipLaunchKernelGGL(k_blk_compact, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, k1, flag, cidx, nnz,
                           rowbits, p.d_kptr, krow, kblk, cnt);
        BK_TRY(hipGetLastError());
        const uint32_t nnz32 = (uint32_t)nnz;
        BK_TRY(hipMemcpyAsync(p.d_kptr + K, &nnz32, 4, hipMemcpyHostToDevice, s));
    }
    p.nkpairs = K;
    {  // rp2 = exclusive scan of the per-row pair counts
        size_t tb = 0;
        BK_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, p.d_rp2, (int)(n + 1), s));
        void *t = tmp.get(tb);
        if (!need(t))
            return 1;
        BK_TRY(hipcub::DeviceScan::ExclusiveSum(t, tb, cnt, p.d_rp2, (int)(n + 1), s));
    }
    // row chunks: consecutive rows with at most kBlockedChunk partials (host, one pass)
    std::vector<uint32_t> rp2((size_t)n + 1);
    BK_TRY(hipMemcpyAsync(rp2.data(), p.d_rp2, rp2.size() * 4, hipMemcpyDeviceToHost, s));
    BK_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> chunk_row(1, 0);
    for (IndexType r = 0; r < n;) {
        IndexType e = (IndexType)(std::upper_bound(rp2.begin() + r + 1, rp2.end(), rp2[r] + kBlockedChunk) -
                                  rp2.begin()) - 1;  // last row end with <= kBlockedChunk partials
        if (e <= r)
            e = r + 1;  // cannot happen: a row has at most B <= kBlockedChunk partials
        chunk_row.push_back(e);
        r = e;
    }
    if (n == 0)
        chunk_row.push_back(0);
    p.nchunks = chunk_row.size() - 1;
    SPMV_TRY(hipMalloc((void **)&p.d_chunk_row, chunk_row.size() * 4));
    BK_TRY(hipMemcpyAsync(p.d_chunk_row, chunk_row.data(), chunk_row.size() * 4, hipMemcpyHostToDevice, s));
    SPMV_TRY(hipMalloc((void **)&p.d_bpart, std::max<size_t>(K, 1) * sizeof(ValueType)));
    SPMV_TRY(hipMalloc((void **)&p.d_rl, std::max<size_t>(K, 1) * 2));
    SPMV_TRY(hipMalloc((void **)&p.d_kpos, std::max<size_t>(K, 1) * 4));
    std::vector<uint32_t> uent, ublk;
    if (K) {
        uint32_t *ckey = (uint32_t *)tmp.get(size_t(K) * 4), *iota = (uint32_t *)tmp.get(size_t(K) * 4);
        uint32_t *ck2 = (uint32_t *)tmp.get(size_t(K) * 4), *ord = (uint32_t *)tmp.get(size_t(K) * 4);
        uint32_t *kb = (uint32_t *)tmp.get((B + 1) * 4);
        if (!need(ckey) || !need(iota) || !need(ck2) || !need(ord) || !need(kb))
            return 1;
        BK_TRY(hipMemsetAsync(kb, 0xFF, (B + 1) * 4, s));
        hipLaunchKernelGGL(k_blk_chunk_keys, dim3((K + 255) / 256), dim3(256), 0, s, krow, kblk, K, p.d_chunk_row,
                           (uint32_t)p.nchunks, ckey, iota, kb);
        BK_TRY(hipGetLastError());
        uint32_t cbits = 1;
        while ((1ull << cbits) < p.nchunks)
            ++cbits;
        size_t tb = 0;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ckey, ck2, iota, ord, (int)K, 0, (int)cbits, s));
        void *t = tmp.get(tb);
        if (!need(t))
            return 1;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(t, tb, ckey, ck2, iota, ord, (int)K, 0, (int)cbits, s));
        hipLaunchKernelGGL(k_blk_kpos, dim3((K + 255) / 256), dim3(256), 0, s, ord, K, p.d_kpos);
        BK_TRY(hipGetLastError());
        // by row (stable: blocks ascending inside a row)
        tb = 0;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, krow, ck2, iota, ord, (int)K, 0, (int)rowbits, s));
        t = tmp.get(tb);
        if (!need(t))
            return 1;
        BK_TRY(hipcub::DeviceRadixSort::SortPairs(t, tb, krow, ck2, iota, ord, (int)K, 0, (int)rowbits, s));
        hipLaunchKernelGGL(k_blk_rl, dim3((K + 255) / 256), dim3(256), 0, s, ord, K, p.d_kpos, ckey, p.d_chunk_row,
                           p.d_rp2, (uint16_t *)p.d_rl);
        BK_TRY(hipGetLastError());
        // work units: each block's compact rows cut into pieces of about `target` entries
        std::vector<uint32_t> hkb(B + 1);
        BK_TRY(hipMemcpyAsync(hkb.data(), kb, B * 4, hipMemcpyDeviceToHost, s));
        BK_TRY(hipStreamSynchronize(s));
        hkb[B] = K;
        for (int64_t b = (int64_t)B - 1; b >= 0; --b)  // blocks without entries: empty ranges
            hkb[b] = std::min(hkb[b], hkb[b + 1]);
        uint32_t *d_at = (uint32_t *)tmp.get((B + 1) * 4), *d_ent = (uint32_t *)tmp.get((B + 1) * 4);
        if (!need(d_at) || !need(d_ent))
            return 1;
        BK_TRY(hipMemcpyAsync(d_at, hkb.data(), (B + 1) * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_blk_take, dim3((unsigned)((B + 1 + 255) / 256)), dim3(256), 0, s, p.d_kptr, d_at,
                           (uint32_t)(B + 1), d_ent);
        BK_TRY(hipGetLastError());
        std::vector<uint32_t> hent(B + 1);
        BK_TRY(hipMemcpyAsync(hent.data(), d_ent, (B + 1) * 4, hipMemcpyDeviceToHost, s));
        BK_TRY(hipStreamSynchronize(s));
        // at least ~4 units per CU in flight, and a block of x (<= 128 KiB) amortised over
        // >= 16K entries
        const uint64_t target = std::max<uint64_t>(16384, nnz / (4 * 256));
        // units are consecutive compact-row ranges in block order (blocks' ranges are adjacent)
        for (uint64_t b = 0; b < B; ++b) {
            const uint32_t ka = hkb[b], kz = hkb[b + 1];
            if (kz == ka)
                continue;
            const uint64_t ents = uint64_t(hent[b + 1]) - hent[b];
            const uint64_t pieces = std::max<uint64_t>(1, std::min<uint64_t>(kz - ka, (ents + target - 1) / target));
            for (uint64_t t2 = 0; t2 < pieces; ++t2) {
                ublk.push_back((uint32_t)b);
                uent.push_back((uint32_t)(ka + (uint64_t(kz - ka) * t2) / pieces));
            }
        }
        uent.push_back(K);
    }
    p.nunits = ublk.size();
    if (p.nunits) {
        SPMV_TRY(hipMalloc((void **)&p.d_unit_panel, ublk.size() * 4));
        SPMV_TRY(hipMalloc((void **)&p.d_unit_ent, uent.size() * 4));
        BK_TRY(hipMemcpyAsync(p.d_unit_panel, ublk.data(), ublk.size() * 4, hipMemcpyHostToDevice, s));
        BK_TRY(hipMemcpyAsync(p.d_unit_ent, uent.data(), uent.size() * 4, hipMemcpyHostToDevice, s));
    }
    BK_TRY(hipStreamSynchronize(s));
#undef BK_TRY
    return 0;
}

}  // namespace spmvhw
