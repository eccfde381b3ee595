// Cost of lora::chirp_segments (csrc/lora_chirp.h) on one lane: cycles per chirp and per run
// for SF 7 / 9 / 12 chirps, tables in LDS (as k_mod_frame builds them) or in registers' reach.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../lora-sdr-lightweight-standalone-library-_amd/csrc/lora_chirp.h"

__global__ void k_build(int sf, int reps, unsigned long long* out) {
  __shared__ lora::ChirpSeg seg[128];
  const int N = 1 << sf;
  lora::ChirpConst c;
  c.fMin = -M_PI;
  c.fMax = M_PI;
  c.fStep = (2 * M_PI) / N;
  c.span = c.fMax - c.fMin;
  int total = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0)
    for (int r = 0; r < reps; ++r) {
      const float f0 = (2.0f * float(M_PI) * (float)((r * 37) % N)) / (float)N;
      total += lora::chirp_segments(c.fMin + f0, N, c, seg, 128);
    }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = (unsigned long long)total;
  }
}

int main() {
  unsigned long long* out;
  (void)hipMalloc(&out, 16);
  for (int sf : {7, 9, 12}) {
    const int reps = 16;
    hipLaunchKernelGGL(k_build, dim3(1), dim3(64), 0, 0, sf, reps, out);
    hipLaunchKernelGGL(k_build, dim3(1), dim3(64), 0, 0, sf, reps, out);
    unsigned long long h[2];
    (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    std::printf("{\"sf\": %d, \"cycles_per_chirp\": %.0f, \"runs_per_chirp\": %.1f, \"cycles_per_run\": %.0f}\n", sf,
                (double)h[0] / reps, (double)h[1] / reps, (double)h[0] / (double)h[1]);
  }
  return 0;
}
