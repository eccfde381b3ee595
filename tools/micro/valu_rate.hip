// Micro-benchmark: VALU issue cost per wave-instruction on gfx950, in shader-clock cycles
// (s_memtime around the loop, per wave) and in wave-instructions per CU per ns (HIP events),
// for the instruction forms the symbol pass is built from.  Independent chains, W waves per
// SIMD.  usage: valu_rate [waves_per_simd]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f2v __attribute__((ext_vector_type(2)));
#define ITERS 8192
#define OP_SCALAR(ins) for (int i = 0; i < 16; ++i) asm volatile(ins : "+v"(a[i]) : "v"(s), "v"(t));
#define OP_PACKED(ins) for (int i = 0; i < 8; ++i) asm volatile(ins : "+v"(b[i]) : "v"(f2v{s, t}), "v"(f2v{t, s}));
template <int MODE>
__global__ void __launch_bounds__(64) k(float* out, unsigned long long* cyc, float s, float t) {
  float a[16];
  f2v b[8];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int i = 0; i < 8; ++i) b[i] = f2v{a[2 * i], a[2 * i + 1]};
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < 1; ++r) {
      if (MODE == 0) { OP_SCALAR("v_fma_f32 %0, %0, %1, %2") }
      if (MODE == 1) { OP_SCALAR("v_add_f32 %0, %0, %1") }
      if (MODE == 2) { OP_PACKED("v_pk_fma_f32 %0, %0, %1, %2") }
      if (MODE == 3) { OP_PACKED("v_pk_add_f32 %0, %0, %1") }
      if (MODE == 4) { OP_PACKED("v_pk_fma_f32 %0, %0, %1, %2 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]") }
      if (MODE == 5) { OP_SCALAR("v_max_f32 %0, %0, %1") }
      if (MODE == 6) { OP_SCALAR("v_min_f32 %0, %0, %1") }
      if (MODE == 7) { OP_SCALAR("v_max3_f32 %0, %0, %1, %2") }
      if (MODE == 8) { OP_SCALAR("v_max3_f32 %0, %0, |%1|, |%2|") }
      if (MODE == 9) { OP_SCALAR("v_med3_f32 %0, %0, %1, %2") }
      if (MODE == 10) { OP_SCALAR("v_med3_u32 %0, %0, %1, %2") }
      if (MODE == 11) { OP_SCALAR("v_max_u32 %0, %0, %1") }
      if (MODE == 12) { OP_SCALAR("v_max3_u32 %0, %0, %1, %2") }
      if (MODE == 13) { OP_SCALAR("v_and_or_b32 %0, %0, %1, %2") }
      if (MODE == 14) { OP_SCALAR("v_and_b32 %0, %0, %1") }
      if (MODE == 15) { OP_SCALAR("v_add_u32 %0, %0, %1") }
      if (MODE == 16) { OP_SCALAR("v_lshlrev_b32 %0, 1, %0") }
      if (MODE == 17) { OP_SCALAR("v_cndmask_b32 %0, %0, %1, vcc") }
      if (MODE == 18) { OP_SCALAR("v_mov_b32 %0, %1") }
      if (MODE == 19) { OP_SCALAR("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") }
      if (MODE == 20) { OP_SCALAR("v_max_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") }
      if (MODE == 21) { OP_SCALAR("v_fma_f32 %0, -%0, |%1|, %2") }
      if (MODE == 22) { OP_SCALAR("v_sub_f32 %0, %0, %1") }
      if (MODE == 23) { OP_SCALAR("v_sin_f32 %0, %0") }
      if (MODE == 24) { OP_SCALAR("v_sqrt_f32 %0, %0") }
      if (MODE == 25) { OP_SCALAR("v_fract_f32 %0, %0") }
      if (MODE == 26) { OP_SCALAR("v_cvt_f32_u32 %0, %0") }
      if (MODE == 27) { OP_SCALAR("v_mul_hi_u32 %0, %0, %1") }
      if (MODE == 28) { for (int i = 0; i < 16; ++i) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); } }
      if (MODE == 29) { for (int i = 0; i < 16; ++i) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); } }
      if (MODE == 30) { for (int i = 0; i < 8; ++i) { asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(f2v{s, t}), "v"(f2v{t, s})); asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(t)); } }
    }
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float r = 0;
  for (int i = 0; i < 16; ++i) r += a[i];
  for (int i = 0; i < 8; ++i) r += b[i].x + b[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
static const char* names[] = {"v_fma_f32 %0, %0, %1, %2",
"v_add_f32 %0, %0, %1",
"v_pk_fma_f32 %0, %0, %1, %2",
"v_pk_add_f32 %0, %0, %1",
"v_pk_fma_f32 %0, %0, %1, %2 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]",
"v_max_f32 %0, %0, %1",
"v_min_f32 %0, %0, %1",
"v_max3_f32 %0, %0, %1, %2",
"v_max3_f32 %0, %0, |%1|, |%2|",
"v_med3_f32 %0, %0, %1, %2",
"v_med3_u32 %0, %0, %1, %2",
"v_max_u32 %0, %0, %1",
"v_max3_u32 %0, %0, %1, %2",
"v_and_or_b32 %0, %0, %1, %2",
"v_and_b32 %0, %0, %1",
"v_add_u32 %0, %0, %1",
"v_lshlrev_b32 %0, 1, %0",
"v_cndmask_b32 %0, %0, %1, vcc",
"v_mov_b32 %0, %1",
"v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
"v_max_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
"v_fma_f32 %0, -%0, |%1|, %2",
"v_sub_f32 %0, %0, %1",
"v_sin_f32 %0, %0",
"v_sqrt_f32 %0, %0",
"v_fract_f32 %0, %0",
"v_cvt_f32_u32 %0, %0",
"v_mul_hi_u32 %0, %0, %1",
"MIX v_fma_f32 %0, %0, %1, %2|v_max3_f32 %0, %0, %1, %2",
"MIX v_fma_f32 %0, %0, %1, %2|v_fma_f32 %0, %0, %1, %2|v_max3_f32 %0, %0, %1, %2",
"MIX v_pk_fma_f32 %0, %0, %1, %2|v_fma_f32 %0, %0, %1, %2"};

template <int MODE>
void run(float* out, unsigned long long* cyc, int wps, int ncu) {
  const int blocks = ncu * 4 * wps;
  static const int NI[] = {16,16,8,8,8,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,16,32,48,16};
  const int ninst = NI[MODE];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0000001f, 0.9999999f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0000001f, 0.9999999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * blocks);
  hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < blocks; ++i) sum += (double)h[i];
  const double per_wave = (double)ITERS * ninst;
  const double cyc_per_inst = sum / blocks / per_wave;  // per wave; W waves share a SIMD
  printf("%-36s W=%d  %.3f ms  %.3f wave-inst/CU/ns  %.2f cyc/inst per wave -> %.2f SIMD-cycles/inst\n",
         names[MODE], wps, ms, (double)blocks * per_wave / ncu / (ms * 1e6), cyc_per_inst, cyc_per_inst / wps);
  free(h);
}
int main(int argc, char** argv) {
  int dev;
  hipGetDevice(&dev);
  int ncu;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  printf("CUs %d, clock attribute %d kHz\n", ncu, clk);
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)ncu * 4 * 16 * 64 * 4);
  hipMalloc(&cyc, (size_t)ncu * 4 * 16 * 8);
  for (int w : {2, 4, 8}) {
    run<0>(out, cyc, w, ncu); run<1>(out, cyc, w, ncu); run<2>(out, cyc, w, ncu); run<3>(out, cyc, w, ncu); run<4>(out, cyc, w, ncu); run<5>(out, cyc, w, ncu); run<6>(out, cyc, w, ncu); run<7>(out, cyc, w, ncu); run<8>(out, cyc, w, ncu); run<9>(out, cyc, w, ncu); run<10>(out, cyc, w, ncu); run<11>(out, cyc, w, ncu); run<12>(out, cyc, w, ncu); run<13>(out, cyc, w, ncu); run<14>(out, cyc, w, ncu); run<15>(out, cyc, w, ncu); run<16>(out, cyc, w, ncu); run<17>(out, cyc, w, ncu); run<18>(out, cyc, w, ncu); run<19>(out, cyc, w, ncu); run<20>(out, cyc, w, ncu); run<21>(out, cyc, w, ncu); run<22>(out, cyc, w, ncu); run<23>(out, cyc, w, ncu); run<24>(out, cyc, w, ncu); run<25>(out, cyc, w, ncu); run<26>(out, cyc, w, ncu); run<27>(out, cyc, w, ncu); run<28>(out, cyc, w, ncu); run<29>(out, cyc, w, ncu); run<30>(out, cyc, w, ncu);
  }
  return 0;
}
