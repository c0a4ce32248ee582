// delta_probe — would 1-byte delta-coded row offsets make the binned kernel's pass 2 faster?
// Measurement tool, not part of the product.
//
// Pass 2 of kernel 6 (spmv-fpga_amd/csrc/binned.hip) streams 4 B (fp32 product) + 2 B (u16 row
// offset) per non-zero and adds into LDS. If each (window, panel) segment were sorted by row, the
// offsets could be 1-byte deltas (mean gap ~16 rows at the headline shape), decoded with a
// 64-lane DPP prefix sum per step: 5 B per non-zero instead of 6. This probe times both forms on
// synthetic segments of the 10M x 10M / 160M shape (256 windows x 512 panels x 1224 entries).
// Usage: delta_probe [check]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
            std::exit(1);                                                    \
        }                                                                    \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline uint32_t hash32(uint64_t a, uint32_t b)
{
    uint32_t h = (uint32_t)a * 0x9E3779B1u ^ (uint32_t)(a >> 32) * 0x61C88647u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    h *= 0x297A2D39u;
    return h ^ (h >> 15);
}

// 64-lane inclusive prefix sum (GCN DPP sequence: row_shr 1/2/3 on the source, row_shr 4/8 with
// bank masks, row_bcast 15/31 with row masks)
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v0)
{
    uint32_t v = v0;
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v0, 0x113, 0xf, 0xf, true);  // row_shr:3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xe, true);   // row_shr:4, banks 1-3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xc, true);   // row_shr:8, banks 2-3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15, rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31, rows 2, 3
    return v;
}

__global__ void k_init(uint64_t nnz, uint32_t L, uint32_t R, float *prod, uint16_t *rowp, uint8_t *delta)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * 256) {
        prod[i] = (float)((hash32(i, 3) & 0xFFFF) / 65536.0 - 0.5);
        rowp[i] = (uint16_t)(hash32(i, 2) % R);
        delta[i] = (i % L) == 0 ? 0 : (uint8_t)(hash32(i, 5) % 31);  // segment starts at row 0
    }
}

// MODE 0: u16 row offsets; MODE 1: u8 deltas decoded by a wave prefix sum (segments start at 0)
template <int MODE, int D>
__global__ __launch_bounds__(1024) void k_acc(const float *__restrict__ prod, const uint16_t *__restrict__ rowp,
                                              const uint8_t *__restrict__ delta, uint32_t nwin, uint32_t npan,
                                              uint32_t L, uint32_t R, float *__restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *ys = reinterpret_cast<double *>(smem);
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        ys[i] = 0.0;
    __syncthreads();
    const uint32_t p = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint32_t STEP = 256;
    for (uint32_t w = wv; w < nwin; w += 16) {
        const uint64_t b = ((uint64_t)w * npan + p) * L;
        uint32_t carry = 0;  // row of the segment's previous entry
        for (uint32_t s = 0; s < L; s += STEP * D) {
            f4 v[D];
            h4 r[D];
            uint32_t dl[D];
#pragma unroll
            for (int u = 0; u < D; ++u) {
                const uint32_t k = s + u * STEP + lane * 4;
                if (k < L) {
                    v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(prod + b + k));
                    if (MODE == 0)
                        r[u] = __builtin_nontemporal_load(reinterpret_cast<const h4 *>(rowp + b + k));
                    else
                        dl[u] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(delta + b + k));
                } else {
                    v[u] = f4{};
                    dl[u] = 0;
                }
            }
#pragma unroll
            for (int u = 0; u < D; ++u) {
                const uint32_t k = s + u * STEP + lane * 4;
                if (MODE == 1) {
                    const uint32_t d0 = dl[u] & 0xFF, d1 = (dl[u] >> 8) & 0xFF, d2 = (dl[u] >> 16) & 0xFF,
                                   d3 = dl[u] >> 24;
                    const uint32_t t = d0 + d1 + d2 + d3;
                    const uint32_t inc = wave_inclusive_sum(t);
                    const uint32_t base = carry + inc - t;
                    carry += __builtin_amdgcn_readlane(inc, 63);
                    r[u][0] = (uint16_t)min(base + d0, R - 1);
                    r[u][1] = (uint16_t)min(base + d0 + d1, R - 1);
                    r[u][2] = (uint16_t)min(base + d0 + d1 + d2, R - 1);
                    r[u][3] = (uint16_t)min(base + t, R - 1);
                }
                if (k < L) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        atomicAdd(&ys[r[u][q]], (double)v[u][q]);
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        y[(uint64_t)p * R + i] = (float)ys[i];
}

template <int MODE, int D>
static void run(const char *name, uint32_t nwin, uint32_t npan, uint32_t L, uint32_t R, bool check)
{
    const uint64_t nnz = (uint64_t)nwin * npan * L;
    float *prod, *y;
    uint16_t *rowp;
    uint8_t *delta;
    CHECK(hipMalloc(&prod, nnz * 4));
    CHECK(hipMalloc(&rowp, nnz * 2));
    CHECK(hipMalloc(&delta, nnz + 16));
    CHECK(hipMalloc(&y, (uint64_t)npan * R * 4));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, nnz, L, R, prod, rowp, delta);
    CHECK(hipDeviceSynchronize());
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_acc<MODE, D>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = check ? 1 : 10, warm = check ? 0 : 2;
    double t = 0;
    for (int it = 0; it < warm + reps; ++it) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((k_acc<MODE, D>), dim3(npan), dim3(1024), (size_t)R * 8, 0, prod, rowp, delta, nwin, npan, L,
                           R, y);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (it >= warm)
            t += ms;
    }
    t /= reps;
    double err = -1;
    if (check) {
        std::vector<float> hp(nnz), hy((uint64_t)npan * R);
        std::vector<uint16_t> hr(nnz);
        std::vector<uint8_t> hd(nnz);
        CHECK(hipMemcpy(hp.data(), prod, nnz * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hr.data(), rowp, nnz * 2, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hd.data(), delta, nnz, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hy.data(), y, hy.size() * 4, hipMemcpyDeviceToHost));
        std::vector<double> ref(hy.size(), 0.0), mag(hy.size(), 0.0);
        for (uint64_t w = 0; w < nwin; ++w)
            for (uint64_t p = 0; p < npan; ++p) {
                const uint64_t b0 = (w * npan + p) * L;
                uint32_t row = 0;
                for (uint32_t k = 0; k < L; ++k) {
                    row = MODE == 0 ? hr[b0 + k] : std::min<uint32_t>(row + hd[b0 + k], R - 1);
                    if (MODE == 1)
                        row = std::min<uint32_t>(row, R - 1);
                    ref[p * R + row] += hp[b0 + k];
                    mag[p * R + row] += std::fabs(hp[b0 + k]);
                }
            }
        err = 0;
        for (uint64_t i = 0; i < hy.size(); ++i)
            if (mag[i] > 0)
                err = std::fmax(err, std::fabs(ref[i] - hy[i]) / mag[i]);
    }
    const double bytes = nnz * (MODE == 0 ? 6.0 : 5.0);
    std::printf("{\"test\": \"%s\", \"mode\": %d, \"D\": %d, \"nnz\": %llu, \"ms\": %.4f, \"TBps\": %.2f, "
                "\"max_scaled_err\": %.3g}\n",
                name, MODE, D, (unsigned long long)nnz, t, bytes / t / 1e9, err);
    std::fflush(stdout);
    CHECK(hipFree(prod));
    CHECK(hipFree(rowp));
    CHECK(hipFree(delta));
    CHECK(hipFree(y));
}

int main(int argc, char **argv)
{
    if (argc > 1 && !std::strcmp(argv[1], "check")) {
        run<0, 4>("check_u16", 5, 7, 1224, 19532, true);
        run<1, 4>("check_delta", 5, 7, 1224, 19532, true);
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 4>("u16_rows", 256, 512, 1224, 19532, false);
        run<1, 4>("u8_deltas", 256, 512, 1224, 19532, false);
        run<0, 8>("u16_rows", 256, 512, 1224, 19532, false);
        run<1, 8>("u8_deltas", 256, 512, 1224, 19532, false);
    }
    return 0;
}
