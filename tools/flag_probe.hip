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
    return 0;
}
