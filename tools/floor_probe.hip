// floor_probe — what the memory system alone allows for the power-law SpMV (config 3), with no
// SpMV arithmetic. Measurement tool, not part of the product.
//
// The panel sweep (spmv-fpga_amd/csrc/sweep.hip) keeps a row panel's y in one CU's LDS and walks
// the panel's entries in column order. For 10M x 10M with 160M uniformly spread columns, a panel
// of 20,447 rows holds ~312K entries over x's 625K 128-byte lines, so a wave instruction of 64
// column-consecutive entries spans ~128 x lines and touches ~50 distinct ones: ~0.79 x-line
// requests per non-zero (126M per SpMV), on top of the 1.92 GB entry stream (12 B/entry). Any
// design that keeps y on chip per CU is held to this density by the 160 KiB LDS.
//
// This probe replays exactly that access pattern with synthetic data and times its parts:
//   lanes_*      : L2-resident 8-byte gathers with 1, 2 or 4 lanes per 128-B line, and 16-byte
//                  gathers: is the L2 bound requests or bytes, and what is a request
//   sweep_gather : 512 workgroups (one per CU, 2 rounds, 160 KiB LDS each) x 2441 chunks of 128
//                  entries; each gather instruction draws 64 uniform columns inside its 2048-column
//                  span (the Poisson statistics of the real matrix: ~0.79 lines per entry); the
//                  columns come from a hash, so nothing is streamed
//   sweep_stream : the same workgroups stream 12 B/entry (u32 + f64, non-temporal) = 1.92 GB
//   sweep_both   : both at once (the sweep's memory traffic)
//   sweep_full   : both + two LDS fp64 atomic adds per lane into a 20,447-slot y (the sweep
//                  minus the product and the y store)
//   *_l2x        : x gathers folded into a 2 MiB window (every gather an L2 hit, same count)
// One JSON line per test: ms (mean of 10 launches after 2 warm-ups), G requests/s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
            return 1;                                                        \
        }                                                                    \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t a, uint32_t b)
{
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    h *= 0x297A2D39u;
    return h ^ (h >> 15);
}

// L2-resident gathers, LPL lanes per 128-byte line: the lanes of a group hit one line, at words
// sub * STRIDE (STRIDE 8: the two 64-byte halves; 1: the same half); W bytes per lane (8 or 16)
template <int LPL, int STRIDE, int W>
__global__ __launch_bounds__(256) void k_lanes(const double *__restrict__ t, uint32_t lines, uint32_t iters,
                                               double *__restrict__ sink)
{
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t grp = tid / LPL, sub = tid % LPL;
    double acc = 0;
    for (uint32_t it = 0; it < iters; it += 4) {
        double v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t line = hash32(grp, it + j) % lines;
            const double *p = t + (uint64_t)line * 16 + sub * STRIDE;
            if constexpr (W == 16) {
                const double2 q = *reinterpret_cast<const double2 *>(p);
                v[j] = q.x + q.y;
            } else {
                v[j] = *p;
            }
        }
        acc += v[0] + v[1] + v[2] + v[3];
    }
    if (acc == 1.2345)
        sink[0] = acc;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kT = 1024;       // threads per workgroup (16 waves), as the sweep
constexpr uint32_t kChunk = 128;    // entries per chunk (one wave: 2 per lane)
constexpr uint32_t kRows = 20447;   // fp64 y slots in 160 KiB of LDS

typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

template <int MODE, bool L2X, int AUX = -1>
__device__ __forceinline__ void k_sweep_body(const uint32_t *__restrict__ rc, const double *__restrict__ val,
                                             const double *__restrict__ x, uint32_t m, uint32_t chunks_in,
                                             double *__restrict__ sink, uint32_t wg, uint32_t span_panels)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *y = reinterpret_cast<double *>(smem);
    for (uint32_t i = threadIdx.x; i <= kRows; i += kT)
        y[i] = 0;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t chunks = chunks_in * span_panels;
    const uint64_t pbase = (uint64_t)wg * chunks_in * kChunk;
    // columns per chunk: the panel's entries spread evenly over [0, m)
    const uint32_t cspan = m / chunks_in;
    double acc = 0;
    for (uint32_t c0 = 0; c0 < chunks; c0 += 2 * (kT / 64)) {
        uint2 w[2];
        double v[2][2];
        uint32_t col[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            uint32_t c = c0 + q * (kT / 64) + wave;
            c = c < chunks ? c : chunks - 1;
            if constexpr ((MODE & 2) && AUX >= 0) {
                // buffer loads with explicit cache-policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
                const uint32_t eo = c * kChunk + 2 * lane;
                const auto rrc = __builtin_amdgcn_make_buffer_rsrc((void *)(rc + pbase), (short)0, 0x7FFFFFFF, 0x00020000);
                const auto rvl = __builtin_amdgcn_make_buffer_rsrc((void *)(val + pbase), (short)0, 0x7FFFFFFF, 0x00020000);
                const u32x2v ww = __builtin_amdgcn_raw_buffer_load_b64(rrc, eo * 4, 0, AUX);
                const u32x4v vv = __builtin_amdgcn_raw_buffer_load_b128(rvl, eo * 8, 0, AUX);
                w[q] = make_uint2(ww.x, ww.y);
                v[q][0] = __builtin_bit_cast(double, ((uint64_t)vv.y << 32) | vv.x);
                v[q][1] = __builtin_bit_cast(double, ((uint64_t)vv.w << 32) | vv.z);
            } else if constexpr (MODE & 2) {
                const uint64_t e = pbase + (uint64_t)c * kChunk + 2 * lane;
                const u32x2 ww = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(rc + e));
                const f64x2 vv = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(val + e));
                w[q] = make_uint2(ww.x, ww.y);
                v[q][0] = vv.x;
                v[q][1] = vv.y;
            } else {
                w[q] = make_uint2(hash32(c, lane) % kRows, hash32(c, lane + 64) % kRows);
                v[q][0] = v[q][1] = 1.0;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                // gather instruction j covers the chunk's j-th half of its column span
                uint32_t cc = (c % chunks_in) * cspan + j * (cspan / 2) + hash32(wg * chunks_in + c, lane * 2 + j) % (cspan / 2);
                cc = cc < m ? cc : m - 1;
                if constexpr (L2X)
                    cc &= (1u << 18) - 1;  // 2 MiB window
                col[q][j] = cc;
            }
        }
        double xv[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                xv[q][j] = (MODE & 1) ? x[col[q][j]] : double(col[q][j] & 1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            // stream mode: the (constant) loaded word mixed with a hash, so rows stay random
            const uint32_t r0 = (MODE & 2) ? (w[q].x ^ hash32(c0 + q, lane)) % kRows : w[q].x;
            const uint32_t r1 = (MODE & 2) ? (w[q].y ^ hash32(c0 + q, lane + 64)) % kRows : w[q].y;
            if constexpr (MODE & 4) {
                atomicAdd(&y[r0], v[q][0] * xv[q][0]);
                atomicAdd(&y[r1], v[q][1] * xv[q][1]);
            } else {
                acc += v[q][0] * xv[q][0] + v[q][1] * xv[q][1] + double(r0 ^ r1);
            }
        }
    }
    __syncthreads();
    if (acc == 1.2345 || y[threadIdx.x] == 1.2345)
        sink[0] = acc + y[threadIdx.x];
}

// MODE bit 0: x gathers, bit 1: entry stream, bit 2: LDS adds; L2X: gathers folded into 2 MiB.
// SPLIT: workgroups split the roles -- even workgroups only stream, odd ones only gather, each
// over two panels' worth of chunks (same totals as MODE 3 on every workgroup)
template <int MODE, bool L2X, bool SPLIT = false, int AUX = -1>
__global__ __launch_bounds__(kT) void k_sweep(const uint32_t *__restrict__ rc, const double *__restrict__ val,
                                              const double *__restrict__ x, uint32_t m, uint32_t chunks_in,
                                              double *__restrict__ sink)
{
    if constexpr (SPLIT) {
        // one workgroup of each pair does the pair's stream, the other its gathers
        if (blockIdx.x & 1)
            return k_sweep_body<1, L2X>(rc, val, x, m, chunks_in, sink, blockIdx.x - 1, 2);
        return k_sweep_body<2, L2X>(rc, val, x, m, chunks_in, sink, blockIdx.x, 2);
    }
    return k_sweep_body<MODE, L2X, AUX>(rc, val, x, m, chunks_in, sink, blockIdx.x, 1);
}
int main()
{
    const uint32_t m = 10000000, panels = 512, chunks = 2441;  // 512 x 2441 x 128 = 160M entries
    const uint64_t ents = (uint64_t)panels * chunks * kChunk;
    uint32_t *rc = nullptr;
    double *val = nullptr, *x = nullptr, *sink = nullptr, *tab = nullptr;
    CHECK(hipMalloc(&rc, ents * 4));
    CHECK(hipMalloc(&val, ents * 8));
    CHECK(hipMalloc(&x, (uint64_t)m * 8));
    CHECK(hipMalloc(&tab, 4u << 20));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(rc, 0x11, ents * 4));
    CHECK(hipMemset(val, 0, ents * 8));
    CHECK(hipMemset(x, 0, (uint64_t)m * 8));
    CHECK(hipMemset(tab, 0, 4u << 20));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timed = [&](const char *name, auto launch, double requests, double bytes) -> int {
        for (int w = 0; w < 2; ++w)
            launch();
        CHECK(hipGetLastError());
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
        std::printf("{\"test\": \"%s\", \"ms\": %.4f, \"Greq_per_s\": %.2f, \"GBps\": %.1f, \"requests\": %.0f, "
                    "\"bytes\": %.0f}\n",
                    name, s * 1e3, requests / s / 1e9, bytes / s / 1e9, requests, bytes);
        std::fflush(stdout);
        return 0;
    };
    // L2-resident lane tests: 2 MiB table = 16384 lines, 2048 x 256 threads x 256 gathers
    {
        const uint32_t lines = 16384, iters = 256, grid = 2048;
        const double lanes = double(grid) * 256 * iters;
#define LANES(NAME, LPL, STRIDE, W)                                                                         \
    if (timed(NAME, [&] { hipLaunchKernelGGL((k_lanes<LPL, STRIDE, W>), dim3(grid), dim3(256), 0, 0, tab, lines, iters, sink); }, \
              lanes / LPL, lanes * W))                                                                       \
        return 1;
        LANES("lanes_1_per_line_8B", 1, 0, 8)
        LANES("lanes_2_per_line_8B_halves", 2, 8, 8)
        LANES("lanes_2_per_line_8B_same_half", 2, 1, 8)
        LANES("lanes_4_per_line_8B", 4, 4, 8)
        LANES("lanes_1_per_line_16B", 1, 0, 16)
#undef LANES
    }
    const size_t lds = (kRows + 1) * 8;
    CHECK(hipFuncSetAttribute((const void *)k_sweep<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const double greq = 0.79 * ents;  // x-line requests of the pattern (Poisson, 64 entries over 128 lines)
    const double sbytes = 12.0 * ents;
#define SWEEP(NAME, MODE, L2X) SWEEPS(NAME, MODE, L2X, false)
#define SWEEPS(NAME, MODE, L2X, SPL)                                                                                      \
    CHECK(hipFuncSetAttribute((const void *)k_sweep<MODE, L2X, SPL>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    if (timed(NAME, [&] { hipLaunchKernelGGL((k_sweep<MODE, L2X, SPL>), dim3(panels), dim3(kT), lds, 0, rc, val, x, m, chunks, sink); }, \
              (MODE & 1) ? greq : 0.0, (MODE & 2) ? sbytes : 0.0))                                                  \
        return 1;
    SWEEP("sweep_gather", 1, false)
    SWEEP("sweep_gather_l2x", 1, true)
    SWEEP("sweep_stream", 2, false)
    SWEEP("sweep_both", 3, false)
    SWEEP("sweep_both_l2x", 3, true)
    SWEEP("sweep_full", 7, false)
    SWEEP("sweep_full_l2x", 7, true)
    SWEEP("sweep_lds_only", 4, false)
#define SWEEPA(NAME, MODE, AUX)                                                                                      \
    CHECK(hipFuncSetAttribute((const void *)k_sweep<MODE, false, false, AUX>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    if (timed(NAME, [&] { hipLaunchKernelGGL((k_sweep<MODE, false, false, AUX>), dim3(panels), dim3(kT), lds, 0, rc, val, x, m, chunks, sink); }, \
              (MODE & 1) ? greq : 0.0, (MODE & 2) ? sbytes : 0.0))                                                  \
        return 1;
    // the entry stream with other cache-policy bits (buffer loads; 1 = sc0, 2 = nt, 16 = sc1)
    SWEEPA("stream_buf_aux0", 2, 0)
    SWEEPA("stream_buf_aux2_nt", 2, 2)
    SWEEPA("stream_buf_aux3_sc0nt", 2, 3)
    SWEEPA("stream_buf_aux18_sc1nt", 2, 18)
    SWEEPA("stream_buf_aux19_sc0sc1nt", 2, 19)
    SWEEPA("both_buf_aux2_nt", 3, 2)
    SWEEPA("both_buf_aux3_sc0nt", 3, 3)
    SWEEPA("both_buf_aux18_sc1nt", 3, 18)
    SWEEPA("both_buf_aux19_sc0sc1nt", 3, 19)
    SWEEPA("both_buf_aux17_sc0sc1", 3, 17)
#undef SWEEPA
    SWEEPS("sweep_split_roles", 3, false, true)
    SWEEPS("sweep_split_roles_l2x", 3, true, true)
#undef SWEEP
#undef SWEEPS
    // Where do the stream and the gathers collide? Half of the CUs (CU mask) stream half of the
    // entries while the other half gathers half of the x lines, each alone and then at the same
    // time on two streams. Concurrent ~ max(alone): the collision is inside a CU (in-order vector
    // memory pipe), and CUs that only pull entries into L2 could feed the sweeping ones.
    // Concurrent ~ sum: the collision is chip-level (L2 channels / fabric).
    {
        hipDeviceProp_t prop;
        CHECK(hipGetDeviceProperties(&prop, 0));
        const int cus = prop.multiProcessorCount;
        std::vector<uint32_t> ma((cus + 31) / 32, 0), mb((cus + 31) / 32, 0);
        for (int c = 0; c < cus; ++c)
            ((c & 1) ? mb : ma)[c / 32] |= 1u << (c % 32);
        hipStream_t sa, sb;
        CHECK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data()));
        CHECK(hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data()));
        const uint32_t half = panels / 2;
        auto launch_s = [&] { hipLaunchKernelGGL((k_sweep<2, false>), dim3(half), dim3(kT), lds, sa, rc, val, x, m, chunks, sink); };
        auto launch_g = [&] { hipLaunchKernelGGL((k_sweep<1, false>), dim3(half), dim3(kT), lds, sb, rc, val, x, m, chunks, sink); };
        CHECK(hipFuncSetAttribute((const void *)k_sweep<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        CHECK(hipFuncSetAttribute((const void *)k_sweep<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        auto wall = [&](const char *name, auto go, double req, double bytes) -> int {
            for (int w = 0; w < 2; ++w)
                go();
            CHECK(hipDeviceSynchronize());
            const int reps = 10;
            const auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; ++r)
                go();
            CHECK(hipDeviceSynchronize());
            const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
            std::printf("{\"test\": \"%s\", \"ms\": %.4f, \"Greq_per_s\": %.2f, \"GBps\": %.1f, \"requests\": %.0f, "
                        "\"bytes\": %.0f, \"cus_each\": %d}\n",
                        name, sec * 1e3, req / sec / 1e9, bytes / sec / 1e9, req, bytes, cus / 2);
            std::fflush(stdout);
            return 0;
        };
        const double hreq = greq / 2, hbytes = sbytes / 2;
        if (wall("halfcus_stream_alone", [&] { launch_s(); }, 0.0, hbytes))
            return 1;
        if (wall("halfcus_gather_alone", [&] { launch_g(); }, hreq, 0.0))
            return 1;
        if (wall("halfcus_stream_and_gather_concurrent", [&] { launch_s(); launch_g(); }, hreq, hbytes))
            return 1;
    }
    return 0;
}
