// Device -> pinned host copy rate against the NUMA node the pinned pages sit on. The GPU's own
// node comes from sysfs (its PCI address); each online node's buffer is allocated under a bind
// policy (set_mempolicy + hipHostMallocNumaUser), and the default hipHostMalloc buffer is located
// with get_mempolicy. 80 MB of y copied as 8 back-to-back pieces on one stream (the form
// spmv_hw's copy-back issues), median of 7, HIP events. One JSON line per buffer.
// Measurement tool, not product code.
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static long set_policy(int mode, const unsigned long *mask, unsigned long maxnode)
{
    return syscall(SYS_set_mempolicy, mode, mask, maxnode);
}

static int node_of(void *p)
{
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, 3 /* MPOL_F_NODE | MPOL_F_ADDR */) != 0)
        return -1;
    return node;
}

static std::string read_file(const std::string &path)
{
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f)
        return "";
    char buf[256] = {0};
    size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    std::string s(buf, n);
    while (!s.empty() && (s.back() == '\n' || s.back() == ' '))
        s.pop_back();
    return s;
}

static float time_copy(void *h, const void *d, size_t bytes, hipStream_t s)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a, s));
        for (int k = 0; k < 8; ++k) {
            const size_t lo = bytes * k / 8, hi = bytes * (k + 1) / 8;
            CK(hipMemcpyAsync(static_cast<char *>(h) + lo, static_cast<const char *>(d) + lo, hi - lo,
                              hipMemcpyDeviceToHost, s));
        }
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main()
{
    const size_t bytes = size_t(80) << 20;
    char bus[64] = {0};
    CK(hipDeviceGetPCIBusId(bus, sizeof(bus), 0));
    std::string id(bus);
    for (char &c : id)
        c = (char)std::tolower((unsigned char)c);
    const std::string gpu_node = read_file("/sys/bus/pci/devices/" + id + "/numa_node");
    const std::string online = read_file("/sys/devices/system/node/online");
    std::printf("{\"pci\": \"%s\", \"gpu_numa_node\": \"%s\", \"online_nodes\": \"%s\", \"cpu\": %d}\n", id.c_str(),
                gpu_node.c_str(), online.c_str(), sched_getcpu());
    void *d = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    {  // default allocation
        void *h = nullptr;
        CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
        const float ms = time_copy(h, d, bytes, s);
        std::printf("{\"buffer\": \"hipHostMallocDefault\", \"node\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", node_of(h), ms,
                    bytes / ms / 1e6);
        CK(hipHostFree(h));
    }
    int maxn = 0;  // online nodes "0-1" or "0"
    {
        const size_t dash = online.find_last_of("-,");
        maxn = std::atoi(dash == std::string::npos ? online.c_str() : online.c_str() + dash + 1);
    }
    for (int n = 0; n <= maxn && n < 64; ++n) {
        unsigned long mask = 1ul << n;
        if (set_policy(2 /* MPOL_BIND */, &mask, 64) != 0) {
            std::printf("{\"buffer\": \"bind\", \"node_requested\": %d, \"error\": \"set_mempolicy failed\"}\n", n);
            continue;
        }
        void *h = nullptr;
        const hipError_t e = hipHostMalloc(&h, bytes, hipHostMallocNumaUser);
        set_policy(0 /* MPOL_DEFAULT */, nullptr, 0);
        if (e != hipSuccess) {
            std::printf("{\"buffer\": \"bind\", \"node_requested\": %d, \"error\": \"%s\"}\n", n, hipGetErrorString(e));
            continue;
        }
        const float ms = time_copy(h, d, bytes, s);
        std::printf("{\"buffer\": \"hipHostMallocNumaUser under MPOL_BIND\", \"node_requested\": %d, \"node\": %d, "
                    "\"ms\": %.4f, \"GBps\": %.1f}\n",
                    n, node_of(h), ms, bytes / ms / 1e6);
        CK(hipHostFree(h));
    }
    CK(hipFree(d));
    return 0;
}
