// Micro-benchmark: issue rate of packed vs scalar fp32 VALU ops and fp64 FMA on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
#define ITERS 4096
template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, float s) {
  float a[16]; f2v b[8]; double d[8];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int i = 0; i < 8; ++i) { b[i] = f2v{a[2*i], a[2*i+1]}; d[i] = a[i]; }
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(b[i]) : "v"(f2v{s, s}));
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(b[i]) : "v"(f2v{s, s}));
    } else if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"((double)s));
    } else if (MODE == 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "+v"(b[i]) : "v"(f2v{s, s}));
    } else if (MODE == 5) {  // packed FMA, 8 independent chains
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[i]) : "v"(f2v{s, s}));
    } else {  // scalar FMA, 16 independent chains
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
    }
  }
  float r = 0;
  for (int i = 0; i < 16; ++i) r += a[i];
  for (int i = 0; i < 8; ++i) r += b[i].x + b[i].y + (float)d[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int MODE>
float run(float* out, int blocks, int ninst) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double waves = blocks * 4.0, insts = waves * ITERS * ninst;
  int dev; hipGetDevice(&dev); int ncu; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  printf("mode %d: %.3f ms  %.3f wave-instr per CU per ns\n", MODE, ms, insts / ncu / (ms * 1e6));
  return ms;
}
int main() {
  float* out; hipMalloc(&out, 4096 * 256 * 4);
  run<0>(out, 4096, 16); run<1>(out, 4096, 8); run<2>(out, 4096, 8); run<3>(out, 4096, 8); run<4>(out, 4096, 8);
  run<5>(out, 4096, 8); run<6>(out, 4096, 16);
  return 0;
}
