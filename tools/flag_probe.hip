// When does the host see a flag that a running kernel raises? (spmv_hw's streamed copy-back needs
// one workgroup's "my panel's y is in memory" to reach the host, or a copy engine, while the
// rest of the kernel still runs.) One workgroup raises the flag, then keeps the kernel alive for
// ~300 us (wall_clock64, 100 MHz); the host polls and records when it saw the flag and when the
// kernel ended. Modes:
//   0: pinned coherent host memory, release store at system scope   (host polls the word)
//   1: pinned coherent host memory, atomic add at system scope      (host polls the word)
//   2: pinned non-coherent host memory, release store at system scope
//   3: device memory, atomic add at system scope; a second stream waits on it with
//      hipStreamWaitValue32 and then copies 4 KiB device -> host; the host records when the
//      copy's event completed
// Output: one JSON line per mode and repetition. Measurement tool, not product code.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void k_raise(uint32_t *flag, int mode, uint64_t hold_ticks)
{
    if (threadIdx.x != 0)
        return;
    if (mode == 1 || mode == 3)
        __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    else
        __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < hold_ticks)
        __builtin_amdgcn_s_sleep(8);
}

// occupies every CU (one 1024-thread workgroup with 128 KiB of LDS each) for hold_ticks
__global__ __launch_bounds__(1024) void k_hog(uint64_t hold_ticks, float *sink)
{
    extern __shared__ float lds[];
    lds[threadIdx.x] = float(threadIdx.x);
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < hold_ticks)
        __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (lds[(threadIdx.x + 1) % 1024] < -1.0f)
        sink[0] = 1.0f;
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    const uint64_t hold = 30000;  // 300 us at 100 MHz
    hipStream_t ks, cs;
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("{\"can_use_stream_wait_value\": %d}\n", can_wait);
    uint32_t *h_coh = nullptr, *h_nc = nullptr, *d_flag = nullptr;
    CK(hipHostMalloc((void **)&h_coh, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void **)&h_nc, 4096, hipHostMallocNonCoherent | hipHostMallocMapped));
    CK(hipMalloc((void **)&d_flag, 4096));
    char *d_buf = nullptr, *h_buf = nullptr;
    CK(hipMalloc((void **)&d_buf, 4096));
    CK(hipHostMalloc((void **)&h_buf, 4096, hipHostMallocDefault));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    // warm the kernel and the copy path
    hipLaunchKernelGGL(k_raise, dim3(1), dim3(64), 0, ks, d_flag, 3, (uint64_t)10);
    CK(hipMemcpyAsync(h_buf, d_buf, 4096, hipMemcpyDeviceToHost, cs));
    CK(hipDeviceSynchronize());
    for (int mode = 0; mode < 4; ++mode) {
        if (mode == 3 && !can_wait)
            continue;
        for (int r = 0; r < reps; ++r) {
            uint32_t *host = mode == 2 ? h_nc : h_coh;
            uint32_t *dev = host;
            if (mode < 3) {
                std::memset(host, 0, 4096);
                CK(hipHostGetDevicePointer((void **)&dev, host, 0));
            } else {
                CK(hipMemset(d_flag, 0, 4096));
                dev = d_flag;
            }
            CK(hipDeviceSynchronize());
            const double t0 = now_us();
            hipLaunchKernelGGL(k_raise, dim3(1), dim3(64), 0, ks, dev, mode, hold);
            if (mode == 3) {
                CK(hipStreamWaitValue32(cs, d_flag, 1u, hipStreamWaitValueGte, 0xFFFFFFFFu));
                CK(hipMemcpyAsync(h_buf, d_buf, 4096, hipMemcpyDeviceToHost, cs));
                CK(hipEventRecord(ev, cs));
            }
            double seen = -1.0, end = -1.0;
            while (end < 0.0 || (seen < 0.0 && now_us() - t0 < 5e5)) {
                if (seen < 0.0) {
                    const bool up = mode < 3 ? __atomic_load_n(host, __ATOMIC_ACQUIRE) != 0
                                             : hipEventQuery(ev) == hipSuccess;
                    if (up)
                        seen = now_us() - t0;
                }
                if (end < 0.0 && hipStreamQuery(ks) == hipSuccess)
                    end = now_us() - t0;
            }
            CK(hipDeviceSynchronize());
            std::printf("{\"mode\": %d, \"rep\": %d, \"seen_us\": %.1f, \"kernel_end_us\": %.1f, \"seen_before_end\": %s}\n",
                        mode, r, seen, end, seen >= 0.0 && seen < end - 50.0 ? "true" : "false");
            std::fflush(stdout);
        }
    }
    // mode 4: a 40 MB device -> pinned host copy on a second stream while every CU is held by a
    // kernel for 1 ms: does the copy finish during the kernel (a copy engine) or after it (a
    // copy kernel that waits for CUs)? Copy alone for reference.
    {
        const size_t bytes = 40u << 20;
        char *d_big = nullptr, *h_big = nullptr;
        float *sink = nullptr;
        CK(hipMalloc((void **)&d_big, bytes));
        CK(hipMalloc((void **)&sink, 64));
        CK(hipHostMalloc((void **)&h_big, bytes, hipHostMallocDefault));
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        CK(hipMemcpyAsync(h_big, d_big, bytes, hipMemcpyDeviceToHost, cs));
        CK(hipDeviceSynchronize());
        for (int r = 0; r < reps; ++r) {
            double t0 = now_us();
            CK(hipMemcpyAsync(h_big, d_big, bytes, hipMemcpyDeviceToHost, cs));
            CK(hipStreamSynchronize(cs));
            const double alone = now_us() - t0;
            CK(hipDeviceSynchronize());
            t0 = now_us();
            hipLaunchKernelGGL(k_hog, dim3(cus), dim3(1024), 128 * 1024, ks, (uint64_t)100000, sink);
            CK(hipGetLastError());
            CK(hipMemcpyAsync(h_big, d_big, bytes, hipMemcpyDeviceToHost, cs));
            CK(hipEventRecord(ev, cs));
            double copy_done = -1.0, end = -1.0;
            while (copy_done < 0.0 || end < 0.0) {
                if (copy_done < 0.0 && hipEventQuery(ev) == hipSuccess)
                    copy_done = now_us() - t0;
                if (end < 0.0 && hipStreamQuery(ks) == hipSuccess)
                    end = now_us() - t0;
            }
            std::printf("{\"mode\": 4, \"rep\": %d, \"copy_alone_us\": %.1f, \"copy_done_us\": %.1f, "
                        "\"hog_end_us\": %.1f, \"copy_during_hog\": %s}\n",
                        r, alone, copy_done, end, copy_done < end ? "true" : "false");
            std::fflush(stdout);
        }
    }
    // mode 5: 80 MB device -> pinned host in 8 pieces on 1, 2 or 4 streams (copy engines in
    // parallel?), and as one copy; ms of the whole transfer
    {
        const size_t bytes = 80u << 20, piece = bytes / 8;
        char *d_big = nullptr, *h_big = nullptr;
        CK(hipMalloc((void **)&d_big, bytes));
        CK(hipHostMalloc((void **)&h_big, bytes, hipHostMallocDefault));
        hipStream_t ss[4];
        for (auto &x : ss)
            CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        for (int k = 0; k < 4; ++k)  // warm every stream's copy path
            CK(hipMemcpyAsync(h_big, d_big, bytes, hipMemcpyDeviceToHost, ss[k]));
        CK(hipDeviceSynchronize());
        for (int r = 0; r < reps; ++r) {
            for (int nst : {0, 1, 2, 4}) {
                const double t0 = now_us();
                if (nst == 0) {
                    CK(hipMemcpyAsync(h_big, d_big, bytes, hipMemcpyDeviceToHost, ss[0]));
                } else {
                    for (int k = 0; k < 8; ++k)
                        CK(hipMemcpyAsync(h_big + k * piece, d_big + k * piece, piece, hipMemcpyDeviceToHost, ss[k % nst]));
                }
                CK(hipDeviceSynchronize());
                std::printf("{\"mode\": 5, \"rep\": %d, \"streams\": %d, \"pieces\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n",
                            r, nst ? nst : 1, nst ? 8 : 1, (now_us() - t0) / 1000, bytes / (now_us() - t0) / 1000);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}
