// binned_probe — two-pass "propagation blocking" SpMV timed on synthetic data of the headline
// shape (10M x 10M, 160M non-zeros uniformly spread). Measurement tool, not part of the product.
//
// The panel sweep (sweep.hip) gathers x through L2 (~0.79 x-line requests per non-zero) while it
// streams 12 B (fp64) / 8 B (fp32) per entry; both share the L2 channels, so the sweep costs about
// gather time + stream time. Propagation blocking replaces the gathers by a second
// stream (Beamer, Asanovic, Patterson, "Reducing PageRank communication via propagation
// blocking", IPDPS 2017):
//   pass 1 (k_mul): one workgroup per column window (W columns of x staged in LDS); it streams the
//                   window's entries (u16 column offset + value), multiplies by x from LDS and
//                   streams the products out in the same order;
//   pass 2 (k_acc): one workgroup per row panel (R row sums in LDS, fp64); it reads the panel's
//                   segment of every window (product + u16 row offset), adds into LDS and writes y.
// Entries are ordered (window, panel); a segment = the entries of one (window, panel) pair.
// Bytes per entry: fp32 4+2 read, 4 written, 4+2 read = 16 (sweep: 8 + gathers);
//                  fp64 8+2, 8, 8+2 = 28 (sweep: 12 + gathers).
// Usage: binned_probe [check]   (check: small sizes against a CPU loop, both precisions)
// One JSON line per test: pass 1, pass 2 and total ms (mean of 10 launches after 2 warm-ups).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
            std::exit(1);                                                    \
        }                                                                    \
    } while (0)

__host__ __device__ inline uint32_t hash32(uint64_t a, uint32_t b)
{
    uint32_t h = (uint32_t)a * 0x9E3779B1u ^ (uint32_t)(a >> 32) * 0x61C88647u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    h *= 0x297A2D39u;
    return h ^ (h >> 15);
}

template <typename V> struct Vec;
template <> struct Vec<float> { typedef float T __attribute__((ext_vector_type(4))); typedef uint16_t I __attribute__((ext_vector_type(4))); };
template <> struct Vec<double> { typedef double T __attribute__((ext_vector_type(2))); typedef uint16_t I __attribute__((ext_vector_type(2))); };

template <typename V>
__global__ void k_init(uint64_t nnz, uint32_t W, uint32_t R, uint16_t *colw, uint16_t *rowp, V *val)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * 256) {
        colw[i] = (uint16_t)(hash32(i, 1) % W);
        rowp[i] = (uint16_t)(hash32(i, 2) % R);
        val[i] = (V)((double)(hash32(i, 3) & 0xFFFFF) / 1048576.0 - 0.5);
    }
}

template <typename V>
__global__ void k_initx(uint32_t n, V *x)
{
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        x[i] = (V)((double)(hash32(i, 9) & 0xFFFFF) / 1048576.0 + 0.25);
}

// pass 1: blockIdx.x = window; entries [w EW, (w+1) EW), EW a multiple of PER
// ABL (measurement only, wrong products): 1 no LDS read (product = value * column offset), 2 no
// product stores (one sink store per lane), 3 no entry loads (stores of a lane-dependent constant)
template <typename V, int U, int G = 1, bool NTS = true, int ABL = 0>
__global__ __launch_bounds__(1024) void k_mul(const V *__restrict__ x, uint32_t ncols, uint32_t W, uint64_t EW,
                                              const uint16_t *__restrict__ colw, const V *__restrict__ val,
                                              V *__restrict__ prod)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *xs = reinterpret_cast<V *>(smem);
    typedef typename Vec<V>::T VT;
    typedef typename Vec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    const uint64_t c0 = (uint64_t)blockIdx.x * W;  // W a multiple of PER: 16-B aligned window
    {
        // stage the window with 16-B loads, 10 in flight per thread (W <= 40960 fp32 / 20480 fp64)
        constexpr int NR = 10;
        VT t[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t i = (r * 1024 + threadIdx.x) * PER;
            if (i < W) {
                if (c0 + i + PER <= ncols) {
                    t[r] = *reinterpret_cast<const VT *>(x + c0 + i);
                } else {
#pragma unroll
                    for (int k = 0; k < PER; ++k)
                        t[r][k] = c0 + i + k < ncols ? x[c0 + i + k] : V(0);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t i = (r * 1024 + threadIdx.x) * PER;
            if (i < W)
                *reinterpret_cast<VT *>(xs + i) = t[r];
        }
    }
    __syncthreads();
    const uint64_t e0 = (uint64_t)blockIdx.x * EW, e1 = e0 + EW;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint64_t STEP = 64 * PER * G;
    VT sink = {};
    for (uint64_t s = e0 + wv * STEP * U; s < e1; s += 16 * STEP * U) {
        VT v[U][G];
        IT c[U][G];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + u * STEP + lane * PER * G;
            if (i < e1) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if (ABL == 3) {
                        v[u][g] = VT{} + V(i & 7);
                        c[u][g] = IT{};
                    } else {
                        v[u][g] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(val + i + g * PER));
                        c[u][g] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(colw + i + g * PER));
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + u * STEP + lane * PER * G;
            if (i < e1) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    VT p;
#pragma unroll
                    for (int k = 0; k < PER; ++k)
                        p[k] = ABL == 1 ? v[u][g][k] * V(c[u][g][k]) : v[u][g][k] * xs[c[u][g][k]];
                    if (ABL == 2)
                        sink += p;
                    else if (NTS)
                        __builtin_nontemporal_store(p, reinterpret_cast<VT *>(prod + i + g * PER));
                    else
                        *reinterpret_cast<VT *>(prod + i + g * PER) = p;
                }
            }
        }
    }
    if (ABL == 2 && sink[0] == V(1.2345))
        prod[0] = sink[1];
}

// pass 2: blockIdx.x = panel; segment (w, p) = entries [(w P + p) L, +L), L a multiple of PER.
// Wave v takes windows v, v + 16, ...; its segments form one stream of 64 PER-entry steps (the last
// step of a segment masked), D steps of loads in flight before the adds.
template <typename V, int D, int G = 1>
__global__ __launch_bounds__(1024) void k_acc(const V *__restrict__ prod, const uint16_t *__restrict__ rowp,
                                              uint32_t nwin, uint32_t npan, uint32_t L, uint32_t R, uint32_t nrows,
                                              V *__restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *ys = reinterpret_cast<double *>(smem);
    typedef typename Vec<V>::T VT;
    typedef typename Vec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        ys[i] = 0.0;
    __syncthreads();
    const uint32_t p = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint32_t STEP = 64 * PER * G;
    uint32_t w = wv;
    uint64_t pos = ((uint64_t)w * npan + p) * L, end = pos + L;
    while (w < nwin) {
        VT v[D][G];
        IT r[D][G];
        uint64_t at[D], en[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
            if (pos >= end) {  // next segment of this wave (uniform)
                w += 16;
                pos = ((uint64_t)w * npan + p) * L;
                end = w < nwin ? pos + L : pos;
            }
            at[u] = pos + lane * PER * G;
            en[u] = end;
            if (at[u] < end) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    v[u][g] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(prod + at[u] + g * PER));
                    r[u][g] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(rowp + at[u] + g * PER));
                }
            }
            pos += STEP;
        }
#pragma unroll
        for (int u = 0; u < D; ++u) {
            if (at[u] < en[u]) {
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int q = 0; q < PER; ++q)
                        atomicAdd(&ys[r[u][g][q]], (double)v[u][g][q]);
            }
        }
        if (pos >= end) {
            w += 16;
            pos = ((uint64_t)w * npan + p) * L;
            end = pos + L;
        }
    }
    __syncthreads();
    const uint64_t r0 = (uint64_t)p * R;
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        if (r0 + i < nrows)
            y[r0 + i] = (V)ys[i];
}

// Software-pipelined forms: the loads of the next batch are issued before the current batch's
// products (pass 1) or adds (pass 2); pass 1 also issues its first batch before the x window is
// written to LDS.
template <typename V, int U>
__global__ __launch_bounds__(1024) void k_mul_pipe(const V *__restrict__ x, uint32_t ncols, uint32_t W, uint64_t EW,
                                                   const uint16_t *__restrict__ colw, const V *__restrict__ val,
                                                   V *__restrict__ prod)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    V *xs = reinterpret_cast<V *>(smem);
    typedef typename Vec<V>::T VT;
    typedef typename Vec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    constexpr uint64_t STEP = 64 * PER;
    constexpr uint64_t STRIDE = 16 * STEP * U;
    struct Batch { VT v[U]; IT c[U]; };
    const uint64_t e0 = (uint64_t)blockIdx.x * EW, e1 = e0 + EW;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    auto load = [&](uint64_t s, Batch &b) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint64_t i = s + k * STEP + lane * PER;
            if (i < e1) {
                b.v[k] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(val + i));
                b.c[k] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(colw + i));
            }
        }
    };
    auto comp = [&](uint64_t s, const Batch &b) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint64_t i = s + k * STEP + lane * PER;
            if (i < e1) {
                VT pr;
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    pr[q] = b.v[k][q] * xs[b.c[k][q]];
                __builtin_nontemporal_store(pr, reinterpret_cast<VT *>(prod + i));
            }
        }
    };
    const uint64_t c0 = (uint64_t)blockIdx.x * W;
    VT t[10];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t i = (r * 1024 + threadIdx.x) * PER;
        if (i < W) {
            if (c0 + i + PER <= ncols) {
                t[r] = *reinterpret_cast<const VT *>(x + c0 + i);
            } else {
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    t[r][q] = c0 + i + q < ncols ? x[c0 + i + q] : V(0);
            }
        }
    }
    uint64_t s = e0 + wv * STEP * U;
    Batch A, B;
    if (s < e1)
        load(s, A);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t i = (r * 1024 + threadIdx.x) * PER;
        if (i < W)
            *reinterpret_cast<VT *>(xs + i) = t[r];
    }
    __syncthreads();
    while (s < e1) {
        uint64_t s2 = s + STRIDE;
        if (s2 < e1)
            load(s2, B);
        comp(s, A);
        s = s2;
        if (s >= e1)
            break;
        s2 = s + STRIDE;
        if (s2 < e1)
            load(s2, A);
        comp(s, B);
        s = s2;
    }
}

template <typename V, int D>
__global__ __launch_bounds__(1024) void k_acc_pipe(const V *__restrict__ prod, const uint16_t *__restrict__ rowp,
                                                   uint32_t nwin, uint32_t npan, uint32_t L, uint32_t R,
                                                   uint32_t nrows, V *__restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *ys = reinterpret_cast<double *>(smem);
    typedef typename Vec<V>::T VT;
    typedef typename Vec<V>::I IT;
    constexpr int PER = 16 / sizeof(V);
    constexpr uint32_t STEP = 64 * PER;
    struct Batch { VT v[D]; IT r[D]; uint64_t at[D], en[D]; };
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        ys[i] = 0.0;
    __syncthreads();
    const uint32_t p = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t w = wv;
    uint64_t pos = ((uint64_t)w * npan + p) * L, end = w < nwin ? pos + L : pos;
    auto load = [&](Batch &b) -> bool {
        bool any = false;
#pragma unroll
        for (int u = 0; u < D; ++u) {
            while (pos >= end && w < nwin) {
                w += 16;
                pos = ((uint64_t)w * npan + p) * L;
                end = w < nwin ? pos + L : pos;
            }
            any |= w < nwin;
            b.at[u] = pos + lane * PER;
            b.en[u] = w < nwin ? end : 0;
            if (b.at[u] < b.en[u]) {
                b.v[u] = __builtin_nontemporal_load(reinterpret_cast<const VT *>(prod + b.at[u]));
                b.r[u] = __builtin_nontemporal_load(reinterpret_cast<const IT *>(rowp + b.at[u]));
            }
            pos += STEP;
        }
        return any;
    };
    auto add = [&](const Batch &b) {
#pragma unroll
        for (int u = 0; u < D; ++u)
            if (b.at[u] < b.en[u]) {
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    atomicAdd(&ys[b.r[u][q]], (double)b.v[u][q]);
            }
    };
    Batch A, B;
    bool ha = load(A);
    while (ha) {
        const bool hb = load(B);
        add(A);
        if (!hb)
            break;
        ha = load(A);
        add(B);
    }
    __syncthreads();
    const uint64_t r0 = (uint64_t)p * R;
    for (uint32_t i = threadIdx.x; i < R; i += 1024)
        if (r0 + i < nrows)
            y[r0 + i] = (V)ys[i];
}

template <typename V, int U, int D, int G1 = 1, int G2 = 1, bool NTS = true, bool PIPE = false, int ABL = 0>
static void run(const char *name, uint32_t n, uint32_t nwin, uint32_t npan, uint32_t L, bool check)
{
    constexpr int PER = 16 / sizeof(V);
    const uint32_t W = ((n + nwin - 1) / nwin + PER - 1) / PER * PER, R = (n + npan - 1) / npan;
    const uint64_t EW = (uint64_t)npan * L, nnz = EW * nwin;
    if (L % (PER * G2) || (uint64_t(npan) * L) % (PER * G1) || W * sizeof(V) > 160 * 1024 || R * 8 > 160 * 1024 || W > 65536 || R > 65536) {
        std::fprintf(stderr, "bad shape\n");
        std::exit(1);
    }
    uint16_t *colw, *rowp;
    V *val, *prod, *x, *y;
    CHECK(hipMalloc(&colw, nnz * 2));
    CHECK(hipMalloc(&rowp, nnz * 2));
    CHECK(hipMalloc(&val, nnz * sizeof(V)));
    CHECK(hipMalloc(&prod, nnz * sizeof(V)));
    CHECK(hipMalloc(&x, (uint64_t)nwin * W * sizeof(V)));
    CHECK(hipMalloc(&y, (uint64_t)n * sizeof(V)));
    hipLaunchKernelGGL(k_init<V>, dim3(4096), dim3(256), 0, 0, nnz, W, R, colw, rowp, val);
    hipLaunchKernelGGL(k_initx<V>, dim3(4096), dim3(256), 0, 0, n, x);
    CHECK(hipDeviceSynchronize());
    const size_t lds1 = W * sizeof(V), lds2 = R * 8;
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_mul<V, U, G1, NTS, ABL>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_mul_pipe<V, U>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_acc_pipe<V, D>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_acc<V, D, G2>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t ev[3];
    for (auto &evt : ev)
        CHECK(hipEventCreate(&evt));
    double t1 = 0, t2 = 0;
    const int reps = check ? 1 : 10, warm = check ? 0 : 2;
    for (int it = 0; it < warm + reps; ++it) {
        CHECK(hipEventRecord(ev[0], 0));
        if (PIPE)
            hipLaunchKernelGGL((k_mul_pipe<V, U>), dim3(nwin), dim3(1024), lds1, 0, x, n, W, EW, colw, val, prod);
        else
            hipLaunchKernelGGL((k_mul<V, U, G1, NTS, ABL>), dim3(nwin), dim3(1024), lds1, 0, x, n, W, EW, colw, val, prod);
        CHECK(hipEventRecord(ev[1], 0));
        if (PIPE)
            hipLaunchKernelGGL((k_acc_pipe<V, D>), dim3(npan), dim3(1024), lds2, 0, prod, rowp, nwin, npan, L, R, n, y);
        else
            hipLaunchKernelGGL((k_acc<V, D, G2>), dim3(npan), dim3(1024), lds2, 0, prod, rowp, nwin, npan, L, R, n, y);
        CHECK(hipEventRecord(ev[2], 0));
        CHECK(hipEventSynchronize(ev[2]));
        float a, b;
        CHECK(hipEventElapsedTime(&a, ev[0], ev[1]));
        CHECK(hipEventElapsedTime(&b, ev[1], ev[2]));
        if (it >= warm) {
            t1 += a;
            t2 += b;
        }
    }
    t1 /= reps;
    t2 /= reps;
    const double b1 = nnz * (2.0 + 2 * sizeof(V)), b2 = nnz * (2.0 + sizeof(V));
    double maxerr = -1;
    if (check) {
        std::vector<uint16_t> hc(nnz), hr(nnz);
        std::vector<V> hv(nnz), hx((uint64_t)nwin * W), hy(n);
        CHECK(hipMemcpy(hc.data(), colw, nnz * 2, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hr.data(), rowp, nnz * 2, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hv.data(), val, nnz * sizeof(V), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hx.data(), x, hx.size() * sizeof(V), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hy.data(), y, (uint64_t)n * sizeof(V), hipMemcpyDeviceToHost));
        std::vector<double> ref(n, 0.0), mag(n, 0.0);
        for (uint64_t i = 0; i < nnz; ++i) {
            const uint64_t w = i / EW, p = (i / L) % npan;
            const uint64_t row = p * R + hr[i], col = w * W + hc[i];
            if (row >= n)
                continue;
            const V xv = col < n ? hx[col] : V(0);
            ref[row] += (double)(V)(hv[i] * xv);
            mag[row] += std::fabs((double)hv[i] * (double)xv);
        }
        maxerr = 0;
        for (uint32_t r = 0; r < n; ++r)
            if (mag[r] > 0)
                maxerr = std::fmax(maxerr, std::fabs(ref[r] - (double)hy[r]) / mag[r]);
    }
    std::printf("{\"test\": \"%s\", \"n\": %u, \"nnz\": %llu, \"windows\": %u, \"W\": %u, \"panels\": %u, \"R\": %u, "
                "\"seg\": %u, \"U\": %d, \"D\": %d, \"G1\": %d, \"G2\": %d, \"nts\": %d, \"pass1_ms\": %.4f, \"pass2_ms\": %.4f, \"total_ms\": %.4f, \"total_ms_160M\": %.4f, "
                "\"pass1_TBps\": %.2f, \"pass2_TBps\": %.2f, \"max_scaled_err\": %.3g}\n",
                name, n, (unsigned long long)nnz, nwin, W, npan, R, L, U, D, G1, G2, (int)NTS, (int)PIPE, t1, t2, t1 + t2, (t1 + t2) * 160e6 / nnz,
                b1 / t1 / 1e9, b2 / t2 / 1e9, maxerr);
    std::fflush(stdout);
    CHECK(hipFree(colw));
    CHECK(hipFree(rowp));
    CHECK(hipFree(val));
    CHECK(hipFree(prod));
    CHECK(hipFree(x));
    CHECK(hipFree(y));
}

int main(int argc, char **argv)
{
    const bool check = argc > 1 && !std::strcmp(argv[1], "check");
    if (check) {
        run<float, 4, 8>("check_f32", 200000, 6, 12, 1224, true);
        return 0;
    }
    const uint32_t n = 10000000;
    // pass-1 ablations (pass 2 runs on whatever pass 1 wrote; only pass1_ms matters)
    for (int rep = 0; rep < 2; ++rep) {
        run<float, 4, 8>("f32_pass1", n, 256, 512, 1224, false);
        run<float, 4, 8, 1, 1, true, false, 1>("f32_pass1_noLDS", n, 256, 512, 1224, false);
        run<float, 4, 8, 1, 1, true, false, 2>("f32_pass1_nostore", n, 256, 512, 1224, false);
        run<float, 4, 8, 1, 1, true, false, 3>("f32_pass1_noload", n, 256, 512, 1224, false);
        run<double, 4, 8>("f64_pass1", n, 512, 512, 612, false);
        run<double, 4, 8, 1, 1, true, false, 1>("f64_pass1_noLDS", n, 512, 512, 612, false);
        run<double, 4, 8, 1, 1, true, false, 2>("f64_pass1_nostore", n, 512, 512, 612, false);
        run<double, 4, 8, 1, 1, true, false, 3>("f64_pass1_noload", n, 512, 512, 612, false);
    }
    return 0;
}
