// How the modulator's sequential phase chain (k_mod_frame's lane 0: one dependent fp32 add
// per sample) is best fed its operands: cycles per add on one lane for
//   0: operands already in VGPRs (the dependent-add floor),
//   1: 8 ds_read_b128 per 32 adds, one block ahead (k_mod_frame's chain as written),
//   2: 2 scalar loads of 16 dwords per 32 adds from global memory, one block ahead, the adds
//      taking their operands from SGPRs,
//   3: 8 global_load_dwordx4 per 32 adds, one block ahead,
//   4: as 2 with sets of 48 dwords (three loads),
//   5: as 2 with one LDS store per 32 adds.
// Timed with s_memtime (shader clock).  Prints one JSON line per mode.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f16v __attribute__((ext_vector_type(16)));
constexpr int kN = 65536;

// a 16-dword scalar load: the constant address space makes the compiler select s_load for a
// uniform address and track its counter itself
typedef __attribute__((address_space(4))) const f16v* cptr16;
__device__ __forceinline__ f16v sload16(const float* p) { return *(cptr16)p; }

template <int MODE>
__global__ void __launch_bounds__(64) k_feed(const float* __restrict__ g, unsigned long long* out, float* sink) {
  __shared__ __attribute__((aligned(16))) float buf[4096 + 64];
  for (int i = threadIdx.x; i < 4096 + 64; i += 64) buf[i] = 1e-3f * (float)(i & 63);
  __syncthreads();
  if (threadIdx.x != 0) return;
  float phase = 0.0f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  if constexpr (MODE == 0) {
    float x[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = buf[k];
    for (int i = 0; i < kN; i += 32) {
#pragma unroll
      for (int k = 0; k < 32; ++k) phase = phase + x[k];
      asm volatile("" : "+v"(phase));
    }
  } else if constexpr (MODE == 1) {
    float4 xa[8], xb[8];
    auto ld = [&](float4* x, int i) {
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = reinterpret_cast<const float4*>(buf + (i & 4095))[q];
    };
    auto run = [&](const float4* x) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        phase = phase + x[q].x;
        phase = phase + x[q].y;
        phase = phase + x[q].z;
        phase = phase + x[q].w;
      }
    };
    ld(xa, 0);
    ld(xb, 32);
    for (int i = 0; i < kN; i += 64) {
      run(xa);
      __builtin_amdgcn_sched_barrier(0);
      ld(xa, i + 64);
      __builtin_amdgcn_sched_barrier(0);
      run(xb);
      __builtin_amdgcn_sched_barrier(0);
      ld(xb, i + 96);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else if constexpr (MODE == 2 || MODE == 4 || MODE == 5) {
    // two sets of S dwords (MODE 4: 48, else 32): wait for set X, request set Y (the next
    // block), add set X.  Scalar loads return out of order, so a wait is always for all of
    // them: the explicit wait sits before the next requests (the compiler keeps a
    // preexisting s_waitcnt).  MODE 5: one LDS store per 32 adds (k_mod_frame's block starts).
    constexpr int NS = MODE == 4 ? 3 : 2, S = 16 * NS;
    f16v x[NS], y[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) x[k] = sload16(g + 16 * k);
    for (int i = 0; i < kN; i += 2 * S) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NS; ++k) y[k] = sload16(g + ((i + S + 16 * k) & (kN - 1)));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        if (MODE == 5) buf[(i >> 4) & 1023] = phase;
#pragma unroll
        for (int e = 0; e < 16; ++e) phase = phase + x[k][e];
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NS; ++k) x[k] = sload16(g + ((i + 2 * S + 16 * k) & (kN - 1)));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        if (MODE == 5) buf[((i >> 4) + 1) & 1023] = phase;
#pragma unroll
        for (int e = 0; e < 16; ++e) phase = phase + y[k][e];
      }
    }
  } else {
    float4 xa[8], xb[8];
    auto ld = [&](float4* x, int i) {
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = reinterpret_cast<const float4*>(g + (i & (kN - 1)))[q];
    };
    auto run = [&](const float4* x) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        phase = phase + x[q].x;
        phase = phase + x[q].y;
        phase = phase + x[q].z;
        phase = phase + x[q].w;
      }
    };
    ld(xa, 0);
    ld(xb, 32);
    for (int i = 0; i < kN; i += 64) {
      run(xa);
      __builtin_amdgcn_sched_barrier(0);
      ld(xa, i + 64);
      __builtin_amdgcn_sched_barrier(0);
      run(xb);
      __builtin_amdgcn_sched_barrier(0);
      ld(xb, i + 96);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  out[MODE] = c1 - c0;
  sink[MODE] = phase;
}

int main() {
  unsigned long long* out;
  float *sink, *g;
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&sink, 64);
  // (kN + 96 floats: the scalar modes read up to 96 past the wrapped index)
  (void)hipMalloc(&g, (kN + 128) * sizeof(float));
  (void)hipMemset(g, 0, (kN + 128) * sizeof(float));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_feed<0>, dim3(1), dim3(64), 0, 0, g, out, sink);
    hipLaunchKernelGGL(k_feed<1>, dim3(1), dim3(64), 0, 0, g, out, sink);
    hipLaunchKernelGGL(k_feed<2>, dim3(1), dim3(64), 0, 0, g, out, sink);
    hipLaunchKernelGGL(k_feed<3>, dim3(1), dim3(64), 0, 0, g, out, sink);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_feed<4>, dim3(1), dim3(64), 0, 0, g, out, sink);
    hipLaunchKernelGGL(k_feed<5>, dim3(1), dim3(64), 0, 0, g, out, sink);
  }
  unsigned long long h[6];
  (void)hipMemcpy(h, out, 48, hipMemcpyDeviceToHost);
  for (int m = 0; m < 6; ++m) std::printf("{\"mode\": %d, \"cycles_per_add\": %.2f}\n", m, (double)h[m] / kN);
  return 0;
}
