// The modulator's phase chain (ChirpGenerator.hpp:121, phase += f per sample, fp32) as a
// lane-shifted chain: lane i holds f_i of a 64-sample block, and 63 dependent DPP adds
// (v_add_f32_dpp wave_shr:1: lane i takes lane i-1's running phase plus its own f_i; lane 0,
// without a source lane, keeps its value) leave p_i in lane i - the same fl(p_{i-1} + f_i)
// as one lane adding serially.  Cycles per sample (s_memtime) for
//   0: one lane, operands in VGPRs (the serial floor, chain_feed.hip mode 0),
//   1: the DPP chain with s_nop 1 between steps (the VALU-write -> DPP-read wait states),
//   2: the same with s_nop 0,
//   3: row_shr:1 (16-lane rows) with s_nop 1, for the cost of the wave-wide shift,
// and whether mode 1's phases equal the serial chain's bit for bit.  One JSON line per mode.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kBlocks = 1024;

template <int MODE>
__global__ void __launch_bounds__(64) k_chain(const float* __restrict__ fin, unsigned long long* out, float* ph) {
  const int lane = threadIdx.x;
  float f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) f[k] = fin[k * 64 + lane];
  float carry = 0.0f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  if constexpr (MODE == 0) {
    // lane 0 adds the 64 values of a block serially (they sit in its own registers)
    float x[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) x[k] = __shfl(f[0], k, 64);
    for (int b = 0; b < kBlocks; ++b) {
#pragma unroll
      for (int k = 0; k < 64; ++k) carry = carry + x[k];
      asm volatile("" : "+v"(carry));
    }
  } else {
    for (int b = 0; b < kBlocks; ++b) {
      const float fb = f[b & 3];
      float v = carry + fb;  // lane 0: p_0; the other lanes are overwritten below
#define STEP1 "s_nop 1\n v_add_f32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define STEP0 "s_nop 0\n v_add_f32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define STEPR "s_nop 1\n v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define X8(s) s s s s s s s s
      if constexpr (MODE == 1) {
        asm volatile(X8(X8(STEP1)) : "+v"(v) : "v"(fb));
      } else if constexpr (MODE == 2) {
        asm volatile(X8(X8(STEP0)) : "+v"(v) : "v"(fb));
      } else {
        asm volatile(X8(X8(STEPR)) : "+v"(v) : "v"(fb));
      }
      // (64 steps where 63 suffice: the first extra one re-adds nothing for lane 0, whose lane
      // is disabled; every other lane's last write is its correct value)
      carry = __shfl(v, 63, 64);  // the block's last phase carries on
      if (b == 0) ph[MODE * 64 + lane] = v;
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[MODE] = c1 - c0;
  if (MODE == 0 && lane == 0) ph[0 * 64 + 0] = carry;
}

__global__ void k_ref(const float* __restrict__ fin, float* ref) {
  float p = 0.0f;
  for (int i = 0; i < 64; ++i) {
    p = p + fin[i];
    ref[i] = p;
  }
}

int main() {
  unsigned long long* out;
  float *fin, *ph, *ref;
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&fin, 256 * sizeof(float));
  (void)hipMalloc(&ph, 4 * 64 * sizeof(float));
  (void)hipMalloc(&ref, 64 * sizeof(float));
  float h[256];
  for (int i = 0; i < 256; ++i) h[i] = -3.14159f + 0.0491f * (float)(i % 128) + 1e-4f * (float)(i % 7);
  (void)hipMemcpy(fin, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, fin, out, ph);
    hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, fin, out, ph);
    hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, fin, out, ph);
    hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, fin, out, ph);
  }
  hipLaunchKernelGGL(k_ref, dim3(1), dim3(1), 0, 0, fin, ref);
  unsigned long long c[4];
  float got[4 * 64], want[64];
  (void)hipMemcpy(c, out, 32, hipMemcpyDeviceToHost);
  (void)hipMemcpy(got, ph, sizeof(got), hipMemcpyDeviceToHost);
  (void)hipMemcpy(want, ref, sizeof(want), hipMemcpyDeviceToHost);
  for (int m = 0; m < 4; ++m) {
    int bad = 0;
    if (m > 0)
      for (int i = 0; i < 64; ++i) bad += got[m * 64 + i] != want[i];
    std::printf("{\"mode\": %d, \"cycles_per_sample\": %.2f, \"mismatches_vs_serial\": %d}\n", m,
                (double)c[m] / (64.0 * kBlocks), m ? bad : -1);
  }
  return 0;
}
