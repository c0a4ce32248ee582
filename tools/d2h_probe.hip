// Device-to-host copy rate of an 80 MB y (10M fp64 rows) into host memory of each kind the merge
// of spmv_hw could stage into: hipHostMalloc with default / coherent / non-coherent flags, malloc
// + hipHostRegister, and pageable malloc. One copy or 64 pieces (the pieced copy of spmv_hw), 8
// timed repeats after one warm-up, wall clock around copy + stream sync. Prints one JSON line per
// (kind, pieces). Measurement tool, not product code.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : size_t(80) << 20;
    void *d = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const char *names[] = {"hipHostMalloc_default", "hipHostMalloc_coherent", "hipHostMalloc_noncoherent",
                           "malloc_hipHostRegister", "malloc_pageable"};
    for (int kind = 0; kind < 5; ++kind) {
        void *h = nullptr;
        if (kind == 0)
            CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
        else if (kind == 1)
            CK(hipHostMalloc(&h, bytes, hipHostMallocCoherent));
        else if (kind == 2)
            CK(hipHostMalloc(&h, bytes, hipHostMallocNonCoherent));
        else {
            h = std::aligned_alloc(4096, bytes);
            std::memset(h, 0, bytes);
            if (kind == 3)
                CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
        }
        for (int pieces : {1, 64}) {
            double best = 1e30, sum = 0;
            const int reps = 8;
            for (int r = 0; r <= reps; ++r) {
                const double t0 = now_ms();
                for (int p = 0; p < pieces; ++p) {
                    const size_t b = bytes * p / pieces, e = bytes * (p + 1) / pieces;
                    CK(hipMemcpyAsync((char *)h + b, (char *)d + b, e - b, hipMemcpyDeviceToHost, s));
                }
                CK(hipStreamSynchronize(s));
                const double t = now_ms() - t0;
                if (r) {
                    sum += t;
                    best = t < best ? t : best;
                }
            }
            std::printf("{\"kind\": \"%s\", \"pieces\": %d, \"MB\": %.1f, \"mean_ms\": %.4f, \"min_ms\": %.4f, "
                        "\"GBps\": %.1f}\n",
                        names[kind], pieces, bytes / 1e6, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9);
            std::fflush(stdout);
        }
        if (kind < 3)
            CK(hipHostFree(h));
        else {
            if (kind == 3)
                CK(hipHostUnregister(h));
            std::free(h);
        }
    }
    CK(hipFree(d));
    return 0;
}
