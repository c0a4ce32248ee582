// LDS atomic throughput microbenchmark (random addresses per lane, 1024-thread workgroups, 1 per CU)
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomics.hip -o lds_atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int MODE>
__global__ __launch_bounds__(1024) void k(const uint32_t* __restrict__ idx, int iters, float* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* yf = (float*)smem; double* yd = (double*)smem; uint32_t* yu = (uint32_t*)smem;
  const int N = MODE == 1 ? 20000 : 40000;
  for (int i = threadIdx.x; i < N; i += 1024) { if (MODE == 1) yd[i] = 0; else yu[i] = 0; }
  __syncthreads();
  uint32_t h = idx[blockIdx.x * 1024 + threadIdx.x] ^ ((blockIdx.x * 1024u + threadIdx.x) * 2654435761u);
  float v = 1.0f + threadIdx.x * 1e-6f;
  for (int it = 0; it < iters; ++it) {
    h = h * 1664525u + 1013904223u;
    const uint32_t r = (h >> 8) % N;
    if (MODE == 0) atomicAdd(&yf[r], v);
    if (MODE == 1) atomicAdd(&yd[r], (double)v);
    if (MODE == 2) atomicAdd(&yu[r], (uint32_t)h);
    if (MODE == 3) { yf[r] = yf[r] + v; }   // racy RMW (throughput only)
    if (MODE == 4) __hip_atomic_fetch_add(&yf[r], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (MODE == 5) v += atomicAdd(&yf[r], v) * 1e-30f;  // returning form (ds_add_rtn_f32)
    if (MODE == 6) {  // compare-and-swap loop on the float's bits (ds_cmpst_rtn_b32)
      uint32_t old = yu[r], assumed;
      do {
        assumed = old;
        old = atomicCAS(&yu[r], assumed, __float_as_uint(__uint_as_float(assumed) + v));
      } while (old != assumed);
    }
  }
  __syncthreads();
  float s = 0; for (int i = threadIdx.x; i < N; i += 1024) s += (MODE == 1 ? (float)yd[i] : yf[i]);
  out[blockIdx.x * 1024 + threadIdx.x] = s;
}
int main() {
  uint32_t* idx; float* out; int B = 256 * 4;
  hipMalloc(&idx, B * 1024 * 4); hipMalloc(&out, B * 1024 * 4);
  hipMemset(idx, 7, B * 1024 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 2000;
  const char* names[] = {"ds_add_f32", "ds_add_f64", "ds_add_u32", "ds_read+write_f32", "ds_add_f32(relaxed,wg)",
                         "ds_add_rtn_f32", "cas_loop_f32"};
  for (int m = 0; m < 7; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(B), dim3(1024), 160000, 0, idx, iters, out); break;
      }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      double ops = (double)B * 1024 * iters;
      if (rep) printf("{\"test\": \"%s\", \"ms\": %.4f, \"Gops_per_s\": %.1f}\n", names[m], ms, ops / ms / 1e6);
    }
  }
  return 0;
}
