// Synthetic inputs for the benchmark configurations of SURVEY.md §8(d) (bench/test
// infrastructure, not the hot path). Every value is a pure function of (seed, row, position),
// computed with integer splitmix64 hashing and exact conversions, so any row range can be
// generated independently (per rank, per partition) and identically on every run.
#include <cmath>

#include "spmv_internal.hpp"

namespace spmvhw {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// key of (row, position) streams; position < 2^20
__host__ __device__ __forceinline__ uint64_t hash3(uint64_t seed, uint64_t row, uint64_t pos)
{
    return splitmix64(splitmix64(seed) ^ ((row << 20) | pos));
}
// [0,1) with 53 random bits (exact)
__host__ __device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

__global__ void k_gen_banded(IndexType n, IndexType w, uint64_t seed, IndexType *row_ptr,
                             IndexType *col, ValueType *val)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n)
        return;
    row_ptr[i] = (IndexType)(i * w);
    if (i == n)
        return;
    int64_t start = (int64_t)i - (int64_t)(w / 2);
    if (start < 0)
        start = 0;
    if (start > (int64_t)n - (int64_t)w)
        start = (int64_t)n - (int64_t)w;
    for (IndexType j = 0; j < w; ++j) {
        col[i * w + j] = (IndexType)(start + j);
        val[i * w + j] = (ValueType)(2.0 * u01(hash3(seed, i, j)) - 1.0);
    }
}

// row i: l = row_ptr[i+1]-row_ptr[i]; entry j -> a uniform column of stratum j of l equal strata
__global__ void k_gen_fill(IndexType n, IndexType m, uint64_t seed, uint64_t row_offset,
                           const IndexType *row_ptr, IndexType *col, ValueType *val)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const IndexType b = row_ptr[i], l = row_ptr[i + 1] - b;
    const uint64_t gi = i + row_offset;
    for (IndexType j = 0; j < l; ++j) {
        const uint64_t h = hash3(seed, gi, j);
        // stratum j = [floor(j*m/l), floor((j+1)*m/l)): disjoint, so columns strictly increase
        const uint64_t lo = (uint64_t)j * m / l, hi = ((uint64_t)j + 1) * m / l;
        col[b + j] = (IndexType)(hi > lo ? lo + h % (hi - lo) : lo % m);
        val[b + j] = (ValueType)(2.0 * u01(splitmix64(h)) - 1.0);
    }
}

__global__ void k_gen_vector(IndexType n, uint64_t seed, uint64_t offset, double lo, double hi,
                             ValueType *x)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    x[i] = (ValueType)(lo + (hi - lo) * u01(hash3(seed, i + offset, 0xFFFFF)));
}

}  // namespace spmvhw

using namespace spmvhw;

extern "C" {

int spmv_gen_banded(IndexType n, IndexType width, uint64_t seed, IndexType *d_row_ptr,
                    IndexType *d_col, ValueType *d_val, void *stream)
{
    if (width == 0 || width > n || uint64_t(n) * width > 0xFFFFFFFFull) {
        set_error("spmv_gen_banded: need 0 < width <= n and n*width < 2^32");
        return 1;
    }
    const unsigned blocks = (unsigned)((uint64_t(n) + 1 + 255) / 256);
    hipLaunchKernelGGL(k_gen_banded, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, width, seed,
                       d_row_ptr, d_col, d_val);
    SPMV_TRY(hipGetLastError());
    return 0;
}

int spmv_gen_powerlaw_row_ptr(IndexType n, uint64_t nnz, IndexType max_len, uint64_t seed,
                              IndexType *h_row_ptr, double *scale_out)
{
    if (n == 0 || nnz < n || nnz > uint64_t(n) * max_len || nnz > 0xFFFFFFFFull || max_len == 0) {
        set_error("spmv_gen_powerlaw_row_ptr: need n <= nnz <= n*max_len and nnz < 2^32");
        return 1;
    }
    // g_i = u_i^-1/2 with u_i in (0,1]; l_i(s) = clamp(floor(s*g_i), 1, max_len), nondecreasing in s
    std::vector<double> g(n);
    for (IndexType i = 0; i < n; ++i)
        g[i] = 1.0 / std::sqrt(u01(hash3(seed, i, 0xFFFFE)) + 0x1.0p-53);
    auto total = [&](double s) {
        uint64_t t = 0;
        for (IndexType i = 0; i < n; ++i) {
            double l = std::floor(s * g[i]);
            t += (uint64_t)(l < 1.0 ? 1.0 : (l > max_len ? (double)max_len : l));
        }
        return t;
    };
    double lo = 0.0, hi = 1.0;
    while (total(hi) < nnz && hi < 1e12)
        hi *= 2.0;
    for (int it = 0; it < 200 && hi - lo > 1e-15 * hi; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (total(mid) <= nnz)
            lo = mid;
        else
            hi = mid;
    }
    const double s = lo;
    std::vector<IndexType> len(n);
    uint64_t t = 0;
    for (IndexType i = 0; i < n; ++i) {
        double l = std::floor(s * g[i]);
        len[i] = (IndexType)(l < 1.0 ? 1.0 : (l > max_len ? (double)max_len : l));
        t += len[i];
    }
    // spread the residual (0 <= nnz - t, small) as +1 over the last rows that can grow
    for (int64_t i = (int64_t)n - 1; t < nnz && i >= 0; --i) {
        if (len[i] < max_len) {
            ++len[i];
            ++t;
        }
    }
    if (t != nnz) {
        set_error("spmv_gen_powerlaw_row_ptr: could not reach the requested nnz");
        return 1;
    }
    h_row_ptr[0] = 0;
    for (IndexType i = 0; i < n; ++i)
        h_row_ptr[i + 1] = h_row_ptr[i] + len[i];
    if (scale_out)
        *scale_out = s;
    return 0;
}

int spmv_gen_fill(IndexType n, IndexType m, uint64_t seed, uint64_t row_offset,
                  const IndexType *d_row_ptr, IndexType *d_col, ValueType *d_val, void *stream)
{
    if (m == 0 && n > 0) {
        set_error("spmv_gen_fill: m must be > 0");
        return 1;
    }
    if (n == 0)
        return 0;
    const unsigned blocks = (unsigned)((uint64_t(n) + 255) / 256);
    hipLaunchKernelGGL(k_gen_fill, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, m, seed,
                       row_offset, d_row_ptr, d_col, d_val);
    SPMV_TRY(hipGetLastError());
    return 0;
}

int spmv_gen_vector(IndexType n, uint64_t seed, uint64_t offset, double lo, double hi, ValueType *d_x,
                    void *stream)
{
    if (n == 0)
        return 0;
    const unsigned blocks = (unsigned)((uint64_t(n) + 255) / 256);
    hipLaunchKernelGGL(k_gen_vector, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, seed, offset,
                       lo, hi, d_x);
    SPMV_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"
