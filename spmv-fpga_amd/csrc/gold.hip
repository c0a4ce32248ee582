// Kernel 1 — "gold order": y bitwise equal to the reference's CPU spmv_gold (csr.cpp:184-194).
//
// spmv_gold adds each row's products v_j * x[c_j] one after another, in CSR order, into an
// accumulator that starts at +0.0, with a separate multiply and add (the reference is built
// -O2 without -march, so no FMA). The tile and sweep kernels reassociate those sums (segmented
// scans, LDS atomics) and agree only to rounding; this kernel keeps the exact order, for
// callers that need results reproducible against the reference bit for bit
// (env SPMV_HW_KERNEL=gold).
//   * rows of <= kGoldLong entries: one lane per row walks its entries in order;
//   * longer rows: one wave per row; the 64 lanes load and multiply 64 consecutive entries at
//     once, then the products are added into the row's accumulator strictly in order
//     (v_readlane chain), so the long rows cost one dependent add per entry, not one
//     dependent load.
// Multiplies and adds are kept separate (fp contract off). Roofline: the x gathers of an
// unstructured matrix miss L2 (~55 G/s); this is a correctness mode, not the
// fast path.
#include "spmv_internal.hpp"

namespace spmvhw {

template <typename V>
__device__ __forceinline__ V read_lane(V v, int lane)
{
    if constexpr (sizeof(V) == 8) {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
        return __builtin_bit_cast(V, (uint64_t(hi) << 32) | lo);
    } else {
        return __builtin_bit_cast(V, __builtin_amdgcn_readlane(__builtin_bit_cast(uint32_t, v), lane));
    }
}

template <typename V>
__global__ __launch_bounds__(256) void k_spmv_gold_rows(const uint32_t *__restrict__ rp, const uint32_t *__restrict__ col,
                                                        const V *__restrict__ val, const V *__restrict__ x,
                                                        V *__restrict__ y, uint32_t nrows)
{
#pragma clang fp contract(off)
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrows)
        return;
    const uint32_t b = rp[r], e = rp[r + 1];
    if (e - b > (uint32_t)kGoldLong)
        return;  // k_spmv_gold_long
    V acc = V(0);
    for (uint32_t j = b; j < e; ++j) {
        const V prod = val[j] * x[col[j]];
        acc = acc + prod;
    }
    y[r] = acc;
}

template <typename V>
__global__ __launch_bounds__(256) void k_spmv_gold_long(const uint32_t *__restrict__ rp, const uint32_t *__restrict__ col,
                                                        const V *__restrict__ val, const V *__restrict__ x,
                                                        const uint32_t *__restrict__ long_rows, uint32_t nlong,
                                                        V *__restrict__ y)
{
#pragma clang fp contract(off)
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= nlong)
        return;  // wave-uniform
    const uint32_t r = long_rows[w];
    const uint32_t b = rp[r], e = rp[r + 1];
    V acc = V(0);
    for (uint32_t base = b; base < e; base += kWave) {
        const uint32_t k = base + lane;
        V prod = V(0);
        if (k < e)
            prod = val[k] * x[col[k]];
        const int cnt = (int)min((uint32_t)kWave, e - base);
        if (cnt == kWave) {
            // constant lanes: the readlanes do not depend on acc and issue ahead of the add
            // chain, which then costs one dependent v_add per entry
#pragma unroll
            for (int t = 0; t < kWave; ++t)
                acc = acc + read_lane(prod, t);
        } else {
            for (int t = 0; t < cnt; ++t)
                acc = acc + read_lane(prod, t);  // wave-uniform: every lane holds the same acc
        }
    }
    if (lane == 0)
        y[r] = acc;
}

hipError_t launch_gold(const spmv_plan &p, const ValueType *d_x, ValueType *d_y, hipStream_t s, bool warm)
{
    if (p.nr_rows == 0)
        return hipSuccess;
    launch_or_warm(warm, k_spmv_gold_rows<ValueType>, dim3((p.nr_rows + 255) / 256), dim3(256), 0, s, p.d_rp,
                       p.d_col, p.d_val, d_x, d_y, p.nr_rows);
    if (p.nlong)
        launch_or_warm(warm, k_spmv_gold_long<ValueType>, dim3((unsigned)((p.nlong + 3) / 4)), dim3(256), 0, s,
                           p.d_rp, p.d_col, p.d_val, d_x, p.d_long, (uint32_t)p.nlong, d_y);
    return hipGetLastError();
}

}  // namespace spmvhw
