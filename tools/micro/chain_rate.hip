// Latency of the modulator's sequential phase chain on one lane: n dependent fp32 adds of
// values read ahead from LDS (k_mod_frame's chain loop shape), timed with s_memtime (shader
// clock) and s_memrealtime (100 MHz).  Prints cycles and ns per add and the clock, for one
// workgroup alone on the GPU and with the other waves of the workgroup busy.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(256) k_chain(int n, int busy, unsigned long long* out, float* sink) {
  __shared__ __attribute__((aligned(16))) float buf[4096 + 32];
  for (int i = threadIdx.x; i < 4096 + 32; i += 256) buf[i] = 1e-3f * (float)(i & 63);
  __syncthreads();
  if (threadIdx.x == 0) {
    float phase = 0.0f;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < n / 4096; ++rep) {
      float4 xa[4], xb[4], ra[4], rb[4];
      auto ld = [&](float4* x, int i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = reinterpret_cast<const float4*>(buf + i)[q];
      };
      auto run = [&](const float4* x, float4* r) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          r[q].x = phase = phase + x[q].x;
          r[q].y = phase = phase + x[q].y;
          r[q].z = phase = phase + x[q].z;
          r[q].w = phase = phase + x[q].w;
        }
      };
      auto st = [&](const float4* r, int i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) reinterpret_cast<float4*>(buf + i)[q] = r[q];
      };
      ld(xa, 0);
      ld(xb, 16);
      for (int i = 0; i < 4096; i += 32) {
        run(xa, ra);
        __builtin_amdgcn_sched_barrier(0);
        if (i > 0) st(rb, i - 16);
        ld(xa, i + 32);
        __builtin_amdgcn_sched_barrier(0);
        run(xb, rb);
        __builtin_amdgcn_sched_barrier(0);
        st(ra, i);
        ld(xb, i + 48);
        __builtin_amdgcn_sched_barrier(0);
      }
      st(rb, 4096 - 16);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[0] = c1 - c0;
    out[1] = r1 - r0;
    sink[0] = phase;
  } else if (busy) {
    // the other waves: sincos-like double work meanwhile
    double x = threadIdx.x;
    for (int k = 0; k < busy; ++k) x = __builtin_fma(x, 1.0000001, 1e-9);
    sink[threadIdx.x] = (float)x;
  }
}

int main() {
  unsigned long long* out;
  float* sink;
  hipMalloc(&out, 16);
  hipMalloc(&sink, 4096);
  for (int busy : {0, 20000}) {
    for (int n : {4096, 65536}) {
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(256), 0, 0, n, busy, out, sink);
        unsigned long long h[2];
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        if (rep == 2)
          std::printf("{\"busy\": %d, \"adds\": %d, \"cycles_per_add\": %.2f, \"ns_per_add\": %.3f, \"clock_mhz\": %.0f}\n",
                      busy, n, (double)h[0] / n, 10.0 * (double)h[1] / n, (double)h[0] / (10.0 * (double)h[1]) * 1e3);
      }
    }
  }
  return 0;
}
