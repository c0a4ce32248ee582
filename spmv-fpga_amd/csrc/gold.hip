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

hipError_t launch_gold(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    const uint32_t waves = (p.nr_rows + kWave - 1) / kWave;
    launch_or_warm(warm, k_spmv_gold<ValueType>, dim3((waves + 3) / 4), dim3(256), 0, s, p.d_rp, p.d_col, p.d_val,
                   d_x, d_y, p.nr_rows);
    return hipGetLastError();
}

}  // namespace spmvhw
