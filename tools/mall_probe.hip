// MALL (Infinity Cache, 256 MiB) probe: does a buffer written by one kernel and read back by the
// next come from MALL instead of HBM when it fits? For buffer sizes of 64 MiB .. 2 GiB: kernel W
// writes the buffer (16-B stores per lane, default or non-temporal policy), kernel R reads it back
// (16-B loads, default or non-temporal), five times in a row on the same buffer; HIP events time
// each kernel. A write-then-read rate well above the HBM stream ceiling (6.45 TB/s read,
// profiles/r01_hbm_calib.jsonl) at sizes below 256 MiB means the two-pass binned kernel's products
// (written by pass 1, read by pass 2) can live in MALL when a pass covers few enough of them.
// Prints one JSON line per (size, store policy, load policy). Measurement tool, not product code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_write(f4 *__restrict__ p, size_t n4, float v)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f4 w = {v, v + 1.f, v + 2.f, (float)(i & 1023)};
        if constexpr (NT)
            __builtin_nontemporal_store(w, p + i);
        else
            p[i] = w;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ p, size_t n4, float *__restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f4 w = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc += w.x + w.y + w.z + w.w;
    }
    if (acc == 12345.678f)  // keeps the loads; never true for the written values
        out[0] = acc;
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

int main()
{
    const size_t sizes_mb[] = {64, 128, 192, 256, 384, 512, 1024, 2048};
    f4 *buf = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&buf, (size_t)2048 << 20));
    CK(hipMalloc(&out, 4));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const dim3 grid(256 * 8), block(256);
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20, n4 = bytes / 16;
        for (int pol = 0; pol < 4; ++pol) {
            const bool ntw = pol & 1, ntr = pol & 2;
            double tw = 0, tr = 0;
            const int reps = 5;
            for (int r = 0; r < reps + 1; ++r) {
                CK(hipEventRecord(e0, nullptr));
                if (ntw)
                    hipLaunchKernelGGL(k_write<true>, grid, block, 0, nullptr, buf, n4, (float)r);
                else
                    hipLaunchKernelGGL(k_write<false>, grid, block, 0, nullptr, buf, n4, (float)r);
                CK(hipEventRecord(e1, nullptr));
                if (ntr)
                    hipLaunchKernelGGL(k_read<true>, grid, block, 0, nullptr, buf, n4, out);
                else
                    hipLaunchKernelGGL(k_read<false>, grid, block, 0, nullptr, buf, n4, out);
                CK(hipEventRecord(e2, nullptr));
                CK(hipEventSynchronize(e2));
                float a = 0, b = 0;
                CK(hipEventElapsedTime(&a, e0, e1));
                CK(hipEventElapsedTime(&b, e1, e2));
                if (r > 0) {  // the first pair warms the buffer's pages
                    tw += a;
                    tr += b;
                }
            }
            tw /= reps;
            tr /= reps;
            std::printf("{\"MiB\": %zu, \"store\": \"%s\", \"load\": \"%s\", \"write_ms\": %.4f, \"read_ms\": %.4f, "
                        "\"write_GBps\": %.1f, \"read_GBps\": %.1f}\n",
                        mb, ntw ? "nt" : "default", ntr ? "nt" : "default", tw, tr, bytes / (tw * 1e-3) / 1e9,
                        bytes / (tr * 1e-3) / 1e9);
            std::fflush(stdout);
        }
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
