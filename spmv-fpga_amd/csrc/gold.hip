// Kernel 1 — "gold order": y bitwise equal to the reference's CPU spmv_gold (csr.cpp:184-194).
//
// spmv_gold adds each row's products v_j * x[c_j] one after another, in CSR order, into an
// accumulator that starts at +0.0, with a separate multiply and add (the reference is built
// -O2 without -march, so no FMA). The tile and sweep kernels reassociate those sums (segmented
// scans, LDS atomics) and agree only to rounding; this kernel keeps the exact order, for
// callers that need results reproducible against the reference bit for bit
// (env SPMV_HW_KERNEL=gold).
// One wave per 64 consecutive rows (lane = row). The wave walks its rows' entry range in
// chunks of kGoldChunk: all 64 lanes load col/val and gather x for the chunk (coalesced,
// many gathers in flight) and store the products in LDS; then every lane adds its own row's
// products of the chunk in order. Multiplies and adds are kept separate (fp contract off), so
// every product and every partial sum is the one spmv_gold computes. Roofline: the x gathers
// of an unstructured matrix miss L2 (~55 G/s); a correctness mode, not the fast
// path.
#include "spmv_internal.hpp"

namespace spmvhw {

constexpr int kGoldChunk = 1024;  // entries per wave per chunk (8 KiB of fp64 products in LDS)

// the wave's LDS writes complete before any lane reads them (and reads before the next writes)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename V>
__global__ __launch_bounds__(256) void k_spmv_gold(const uint32_t *__restrict__ rp, const uint32_t *__restrict__ col,
                                                   const V *__restrict__ val, const V *__restrict__ x,
                                                   V *__restrict__ y, uint32_t nrows)
{
#pragma clang fp contract(off)
    __shared__ V prod[4][kGoldChunk];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t r0 = (blockIdx.x * 4 + w) * kWave;
    if (r0 >= nrows)
        return;  // wave-uniform
    const uint32_t r = r0 + lane;
    const bool valid = r < nrows;
    const uint32_t rb = valid ? rp[r] : 0u, re = valid ? rp[r + 1] : 0u;
    const uint32_t B = rp[r0], E = rp[min(r0 + (uint32_t)kWave, nrows)];
    V acc = V(0);
    for (uint32_t cs = B; cs < E; cs += kGoldChunk) {
        const uint32_t ce = min(cs + (uint32_t)kGoldChunk, E);
        for (uint32_t k = cs + lane; k < ce; k += kWave) {
            const V prd = val[k] * x[col[k]];
            prod[w][k - cs] = prd;
        }
        wave_lds_sync();
        const uint32_t a = max(rb, cs), b = min(re, ce);
        uint32_t k = a;
        for (; k + 16 <= b; k += 16) {  // 16 LDS reads in flight, then the in-order adds
            V t[16];
#pragma unroll
            for (int i = 0; i < 16; ++i)
                t[i] = prod[w][k + i - cs];
#pragma unroll
            for (int i = 0; i < 16; ++i)
                acc = acc + t[i];
        }
        for (; k < b; ++k)
            acc = acc + prod[w][k - cs];
        wave_lds_sync();
    }
    if (valid)
        y[r] = acc;
}

// FPGA order (SPMV_HW_KERNEL=fpga): the arithmetic of the reference's hardware path for a given
// vectorisation factor VF and column-block width W (util.h:31-59). Per row and per column block
// in order: the row's entries of the block in CSR order (create_block_matrix,
// csr_hw.cpp:209-243) are summed in groups of VF, each group from 0 left to right, the last
// group padded with 0 * x[block start] (csr_hw.cpp:228-238); each group is added to the block's
// running sum (compute_results, spmv.cpp:74-103); each block's sum is added to y in block order
// (accum_results, csr_hw.cpp:1543-1562). The entries of every row are stored block-ordered
// (stable), so one in-order pass per lane suffices.
template <typename V, int VF>
__global__ __launch_bounds__(256) void k_spmv_fpga(const uint32_t *__restrict__ rp, const uint32_t *__restrict__ col,
                                                   const V *__restrict__ val, const V *__restrict__ x,
                                                   V *__restrict__ y, uint32_t nrows, uint32_t width)
{
#pragma clang fp contract(off)
    constexpr uint32_t kChunk = 512;
    __shared__ V prod[4][kChunk];
    __shared__ V padz[4][kChunk];  // 0 * x[start of the entry's block]: the pad product's value
    __shared__ uint32_t blk[4][kChunk];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t r0 = (blockIdx.x * 4 + w) * kWave;
    if (r0 >= nrows)
        return;  // wave-uniform
    const uint32_t r = r0 + lane;
    const bool valid = r < nrows;
    const uint32_t rb = valid ? rp[r] : 0u, re = valid ? rp[r + 1] : 0u;
    const uint32_t B = rp[r0], E = rp[min(r0 + (uint32_t)kWave, nrows)];
    const bool pow2 = (width & (width - 1)) == 0;
    const uint32_t shift = __builtin_ctz(width);
    V acc = V(0), sum = V(0), group = V(0), z = V(0);
    uint32_t cur = 0xFFFFFFFFu, in_group = 0;
    // ends the current block: pads its last group to VF with the product 0 * x[block start]
    // (one add stands for the VF - in_group pad adds: g + z + z == g + z for z = 0 * x, which
    // is +0, -0 or NaN), adds the group to the block sum and the block sum to the row's result
    auto close_block = [&]() {
        if (in_group != 0)
            sum = sum + (group + z);
        acc = acc + sum;
    };
    auto step = [&](uint32_t bk, V prd, V pz) {
        if (bk != cur) {
            if (cur != 0xFFFFFFFFu)
                close_block();
            cur = bk;
            z = pz;
            sum = V(0);
            group = V(0);
            in_group = 0;
        }
        group = group + prd;
        if (++in_group == (uint32_t)VF) {
            sum = sum + group;
            group = V(0);
            in_group = 0;
        }
    };
    for (uint32_t cs = B; cs < E; cs += kChunk) {
        const uint32_t ce = min(cs + kChunk, E);
        for (uint32_t k = cs + lane; k < ce; k += kWave) {
            const uint32_t c = col[k];
            const uint32_t bk = pow2 ? c >> shift : c / width;
            prod[w][k - cs] = val[k] * x[c];
            padz[w][k - cs] = V(0) * x[bk * width];  // bk * width <= c
            blk[w][k - cs] = bk;
        }
        wave_lds_sync();
        const uint32_t a = max(rb, cs), b = min(re, ce);
        uint32_t k = a;
        for (; k + 8 <= b; k += 8) {  // 24 LDS reads in flight, then the in-order steps
            V t[8], tz[8];
            uint32_t tb[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                t[i] = prod[w][k + i - cs];
                tz[i] = padz[w][k + i - cs];
                tb[i] = blk[w][k + i - cs];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
                step(tb[i], t[i], tz[i]);
        }
        for (; k < b; ++k)
            step(blk[w][k - cs], prod[w][k - cs], padz[w][k - cs]);
        wave_lds_sync();
    }
    if (valid) {
        if (cur != 0xFFFFFFFFu)
            close_block();
        y[r] = acc;
    }
}

hipError_t launch_gold(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    const uint32_t waves = (p.nr_rows + kWave - 1) / kWave;
    if (p.kernel == kKernelFpga) {
        auto k = p.fpga_vf == 8   ? k_spmv_fpga<ValueType, 8>
                 : p.fpga_vf == 4 ? k_spmv_fpga<ValueType, 4>
                 : p.fpga_vf == 2 ? k_spmv_fpga<ValueType, 2>
                                  : k_spmv_fpga<ValueType, 1>;
        launch_or_warm(warm, k, dim3((waves + 3) / 4), dim3(256), 0, s, p.d_rp, p.d_col, p.d_val, d_x, d_y,
                       p.nr_rows, p.fpga_width);
    } else
        launch_or_warm(warm, k_spmv_gold<ValueType>, dim3((waves + 3) / 4), dim3(256), 0, s, p.d_rp, p.d_col,
                       p.d_val, d_x, d_y, p.nr_rows);
    return hipGetLastError();
}

}  // namespace spmvhw
