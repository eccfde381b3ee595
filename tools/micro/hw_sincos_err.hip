// Exhaustive error of the hardware sine/cosine (v_sin_f32 / v_cos_f32, argument in
// revolutions) over every fp32 input in [0, 1): max |hw(r) - sin/cos(2 pi r)| with the
// reference in double precision.  LORA_PRECISION_FAST's rotation evaluates exactly these
// instructions on fract(ph / 2pi); the certification bound of the speculative pipeline
// (lora_demod_fast.hip, k_est_fast<SPEC = 2>) uses the measured maximum.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/hw_sincos_err tools/micro/hw_sincos_err.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr unsigned kLast = 0x3f7fffffu;  // largest float < 1
constexpr int kBlocks = 8192, kThreads = 256;

__global__ void __launch_bounds__(kThreads) k_err(double* out_s, double* out_c, unsigned* worst) {
  __shared__ double rs[kThreads], rc[kThreads];
  __shared__ unsigned ws[kThreads], wc[kThreads];
  const unsigned tid = blockIdx.x * kThreads + threadIdx.x;
  const unsigned stride = kBlocks * kThreads;
  double es = 0.0, ec = 0.0;
  unsigned bs = 0, bc = 0;
  for (unsigned b = tid; b <= kLast; b += stride) {
    const float r = __uint_as_float(b);
    const double ang = 2.0 * M_PI * (double)r;
    const double ds = fabs((double)__builtin_amdgcn_sinf(r) - sin(ang));
    const double dc = fabs((double)__builtin_amdgcn_cosf(r) - cos(ang));
    if (ds > es) { es = ds; bs = b; }
    if (dc > ec) { ec = dc; bc = b; }
  }
  rs[threadIdx.x] = es;
  rc[threadIdx.x] = ec;
  ws[threadIdx.x] = bs;
  wc[threadIdx.x] = bc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      if (rs[threadIdx.x + o] > rs[threadIdx.x]) { rs[threadIdx.x] = rs[threadIdx.x + o]; ws[threadIdx.x] = ws[threadIdx.x + o]; }
      if (rc[threadIdx.x + o] > rc[threadIdx.x]) { rc[threadIdx.x] = rc[threadIdx.x + o]; wc[threadIdx.x] = wc[threadIdx.x + o]; }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out_s[blockIdx.x] = rs[0];
    out_c[blockIdx.x] = rc[0];
    worst[2 * blockIdx.x] = ws[0];
    worst[2 * blockIdx.x + 1] = wc[0];
  }
}

int main() {
  double *ds, *dc;
  unsigned* dw;
  if (hipMalloc(&ds, kBlocks * 8) != hipSuccess || hipMalloc(&dc, kBlocks * 8) != hipSuccess ||
      hipMalloc(&dw, kBlocks * 8) != hipSuccess)
    return 1;
  hipLaunchKernelGGL(k_err, dim3(kBlocks), dim3(kThreads), 0, 0, ds, dc, dw);
  std::vector<double> hs(kBlocks), hc(kBlocks);
  std::vector<unsigned> hw(2 * kBlocks);
  if (hipMemcpy(hs.data(), ds, kBlocks * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hc.data(), dc, kBlocks * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hw.data(), dw, kBlocks * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  double ms = 0, mc = 0;
  unsigned bs = 0, bc = 0;
  for (int i = 0; i < kBlocks; ++i) {
    if (hs[i] > ms) { ms = hs[i]; bs = hw[2 * i]; }
    if (hc[i] > mc) { mc = hc[i]; bc = hw[2 * i + 1]; }
  }
  float fs, fc;
  memcpy(&fs, &bs, 4);
  memcpy(&fc, &bc, 4);
  printf("{\"inputs\": \"every fp32 r in [0, 1)\", \"max_abs_err_sin\": %.6e, \"at_r_sin\": %.9g, "
         "\"max_abs_err_cos\": %.6e, \"at_r_cos\": %.9g}\n", ms, fs, mc, fc);
  return 0;
}
