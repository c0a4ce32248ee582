// hbm_calib — calibration micro-benchmarks for the SpMV roofline (not part of the product).
//
//  stream_read   : dwordx4 coalesced read of a 2 GiB buffer (achievable HBM read rate; the
//                  known byte count that calibrates FETCH_SIZE for wide streaming reads)
//  stream_copy   : dwordx4 copy of 1 GiB (achievable read+write rate)
//  gather_hbm    : 8-byte random gathers from a 2 GiB table (per-request HBM cost)
//  gather_mall   : 8-byte random gathers from an 80 MB table (the x vector of config 3: served
//                  by L2 / Infinity Cache) — the gather ceiling of the power-law SpMV
//  gather_mall_nt: the same gathers while a dwordx4 stream runs beside them (the SpMV mix)
// Prints one JSON line per test with GB/s and G-requests/s. Run it under rocprofv3 --pmc
// FETCH_SIZE (and separately WRITE_SIZE) to read bytes-per-request calibration factors.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__global__ void k_stream_read(const uint4 *__restrict__ a, size_t n, unsigned *__restrict__ sink)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

__global__ void k_stream_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// each thread: 8 independent random 8-byte gathers per iteration
__global__ void k_gather(const double *__restrict__ t, size_t tn, size_t per_thread, double *__restrict__ sink)
{
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (size_t it = 0; it < per_thread; it += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = t[mix(tid * 0x10000ull + it + j) % tn];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc += v[j];
    }
    if (acc == 1.2345)
        sink[0] = acc;
}

// the same L2-resident gather with other load flavours: 1 = sc1 (L1 bypass), 2 = nt
template <int KIND>
__global__ void k_gather_kind(const double *__restrict__ t, size_t tn, size_t per_thread, double *__restrict__ sink)
{
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (size_t it = 0; it < per_thread; it += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const double *p = t + mix(tid * 0x10000ull + it + j) % tn;
            if constexpr (KIND == 1)
                v[j] = __builtin_bit_cast(double, __hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT));
            else if constexpr (KIND == 2)
                v[j] = __builtin_nontemporal_load(p);
            else
                v[j] = *p;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc += v[j];
    }
    if (acc == 1.2345)
        sink[0] = acc;
}

// gathers confined to a window that sweeps the table (the column-sorted "x sweep" pattern):
// iteration `it` of every thread reads inside [it*step, it*step + win) mod tn
__global__ void k_gather_sweep(const double *__restrict__ t, size_t tn, size_t per_thread, size_t win,
                               size_t step, double *__restrict__ sink)
{
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (size_t it = 0; it < per_thread; it += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = t[((it + j) * step + mix(tid * 0x10000ull + it + j) % win) % tn];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc += v[j];
    }
    if (acc == 1.2345)
        sink[0] = acc;
}

// LDS fp64 atomic-add rate: every thread adds into random slots of a 16K-entry LDS array
__global__ void k_lds_add(size_t per_thread, double *__restrict__ sink)
{
    __shared__ double y[16384];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x)
        y[i] = 0.0;
    __syncthreads();
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (size_t it = 0; it < per_thread; ++it)
        atomicAdd(&y[mix(tid * 0x10000ull + it) & 16383], 1.0);
    __syncthreads();
    if (y[threadIdx.x] == 1.2345)
        sink[0] = y[threadIdx.x];
}

// SpMV-like mix: 12 streamed bytes (dwordx4 col/val-like) per random 8-byte gather
__global__ void k_mix(const uint4 *__restrict__ s, size_t sn, const double *__restrict__ t, size_t tn,
                      double *__restrict__ sink)
{
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < sn; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = s[i];
        acc += t[mix(v.x ^ (i << 1)) % tn] + t[mix(v.y ^ (i << 1) ^ 1) % tn];
    }
    if (acc == 1.2345)
        sink[0] = acc;
}

int main()
{
    const size_t big = 2ull << 30, small = 80ull << 20;
    uint4 *a = nullptr, *b = nullptr;
    double *sink = nullptr;
    unsigned *usink = nullptr;
    CHECK(hipMalloc(&a, big));
    CHECK(hipMalloc(&b, big / 2));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&usink, 64));
    CHECK(hipMemset(a, 1, big));
    CHECK(hipMemset(b, 0, big / 2));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = 256 * 8, block = 256;
    auto timed = [&](const char *name, auto launch, double bytes, double requests) -> int {
        for (int w = 0; w < 2; ++w)
            launch();
        CHECK(hipDeviceSynchronize());
        const int reps = 10;
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double s = ms / 1e3 / reps;
        std::printf("{\"test\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"Greq_per_s\": %.2f, \"bytes\": %.0f, "
                    "\"requests\": %.0f}\n", name, s * 1e3, bytes / s / 1e9, requests / s / 1e9, bytes, requests);
        std::fflush(stdout);
        return 0;
    };
    const size_t n4 = big / 16;
    if (timed("stream_read", [&] { hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(block), 0, 0, a, n4, usink); },
              (double)big, 0))
        return 1;
    if (timed("stream_copy", [&] { hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(block), 0, 0, a, b, n4 / 2); },
              (double)big, 0))
        return 1;
    const size_t per_thread = 256;
    const double nreq = (double)grid * block * per_thread;
    if (timed("gather_hbm", [&] {
            hipLaunchKernelGGL(k_gather, dim3(grid), dim3(block), 0, 0, (const double *)a, big / 8, per_thread, sink);
        }, nreq * 8, nreq))
        return 1;
    if (timed("gather_mall", [&] {
            hipLaunchKernelGGL(k_gather, dim3(grid), dim3(block), 0, 0, (const double *)a, small / 8, per_thread, sink);
        }, nreq * 8, nreq))
        return 1;
    for (size_t kb : {256ull, 1024ull, 2048ull, 4096ull, 16384ull}) {
        char name[64];
        std::snprintf(name, sizeof name, "gather_table_%zuKB", (size_t)kb);
        if (timed(name, [&] {
                hipLaunchKernelGGL(k_gather, dim3(grid), dim3(block), 0, 0, (const double *)a, kb * 1024 / 8,
                                   per_thread, sink);
            }, nreq * 8, nreq))
            return 1;
    }
    for (int kind = 0; kind < 3; ++kind) {
        char name[64];
        std::snprintf(name, sizeof name, "gather_2MB_kind%d", kind);
        auto go = [&] {
            const size_t tn = 2048 * 1024 / 8;
            if (kind == 0)
                hipLaunchKernelGGL(k_gather_kind<0>, dim3(grid), dim3(block), 0, 0, (const double *)a, tn, per_thread, sink);
            else if (kind == 1)
                hipLaunchKernelGGL(k_gather_kind<1>, dim3(grid), dim3(block), 0, 0, (const double *)a, tn, per_thread, sink);
            else
                hipLaunchKernelGGL(k_gather_kind<2>, dim3(grid), dim3(block), 0, 0, (const double *)a, tn, per_thread, sink);
        };
        if (timed(name, go, nreq * 8, nreq))
            return 1;
    }
    for (size_t win : {8192ull, 65536ull, 262144ull}) {
        char name[64];
        std::snprintf(name, sizeof name, "gather_sweep_win%zu", (size_t)win);
        if (timed(name, [&] {
                hipLaunchKernelGGL(k_gather_sweep, dim3(grid), dim3(block), 0, 0, (const double *)a, small / 8,
                                   per_thread, win, (small / 8) / per_thread, sink);
            }, nreq * 8, nreq))
            return 1;
    }
    if (timed("lds_add_f64", [&] {
            hipLaunchKernelGGL(k_lds_add, dim3(grid), dim3(block), 0, 0, per_thread, sink);
        }, nreq * 8, nreq))
        return 1;
    const size_t sn = (big / 2) / 16;
    if (timed("mix_stream_plus_mall_gather", [&] {
            hipLaunchKernelGGL(k_mix, dim3(grid), dim3(block), 0, 0, (const uint4 *)b, sn, (const double *)a,
                               small / 8, sink);
        }, (double)(big / 2) + 2.0 * sn * 8, 2.0 * sn))
        return 1;
    return 0;
}
