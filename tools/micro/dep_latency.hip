// Dependent-issue latency of v_add_f32 on one wave (a chain of 64 adds per iteration, registers
// only), and of the same with one LDS store per 4 adds: cycles per add via s_memtime.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ void k_dep(int iters, unsigned long long* out, float* sink) {
  __shared__ float lds[1024];
  float p = (float)threadIdx.x * 1e-7f;
  float x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = 1e-6f * (k + 1);
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      p = p + x[k & 15];
      if (MODE == 1 && (k & 3) == 3) lds[(k & 63) * 4 + (threadIdx.x & 3)] = p;
    }
    asm volatile("" : "+v"(p));
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = c1 - c0;
  sink[threadIdx.x] = p + lds[threadIdx.x & 255];
}

int main() {
  unsigned long long* out;
  float* sink;
  (void)hipMalloc(&out, 16);
  (void)hipMalloc(&sink, 4096);
  for (int mode = 0; mode < 2; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      const int iters = 1000;
      if (mode == 0) hipLaunchKernelGGL(k_dep<0>, dim3(1), dim3(64), 0, 0, iters, out, sink);
      else hipLaunchKernelGGL(k_dep<1>, dim3(1), dim3(64), 0, 0, iters, out, sink);
      unsigned long long h;
      (void)hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
      if (rep == 2) std::printf("{\"mode\": %d, \"cycles_per_add\": %.2f}\n", mode, (double)h / (iters * 64.0));
    }
  return 0;
}
