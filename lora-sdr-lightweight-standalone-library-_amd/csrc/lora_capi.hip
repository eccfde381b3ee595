// lora_capi.hip — MI355X (gfx950) LoRa demodulator/modulator behind the C-ABI of
// include/lora_mi355x.h.
//
// Demodulation of F frames is three launches on one stream (generic path, any SF
// 2..12, any osr, any frame length):
//   k_frame_max  LEGACY only: per-frame max(|I|,|Q|) of the (dechirped) samples,
//                LoRaDemod.cpp:59-67, streamed with 16-byte loads; each block writes its
//                partial maximum to its own workspace slot (no atomics, no zeroing) and
//                the estimate reduces a frame's partials (k_frame_max_wave: one wave,
//                one partial per short frame).
//   k_estimate   one workgroup per frame: the 2-symbol x osr-phase offset estimate
//                (LoRaDemod.cpp:79-135 / phy.cpp:78-145) and the two sync symbols,
//                leaving cfo / t_off / rate / scale in the workspace.
//   k_demod      G = max(1, 1024/N) symbols per workgroup: (dechirp) -> (scale) ->
//                CFO rotation (glibc-faithful sincosf) -> (window) -> LDS radix-4/2
//                DIT FFT with kissfft's butterflies -> lowest-index argmax |X|^2
//                (LoRaDemod.cpp:141-174, LoRaDetector.hpp:39-58).
// The register-blocked fast kernels that replace k_estimate / k_demod wherever they
// cover the configuration live in lora_demod_fast.hip.
//
// All fp32 arithmetic follows the reference's operation order without contraction
// (compiled with -ffp-contract=off, see lora_device.h), so outputs are bit-identical
// to the reference's x86-64 build on the same inputs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lora_mi355x.h"
#include "lora_chirp.h"
#include "lora_device.h"
#include "lora_internal.h"

#pragma clang fp contract(off)

using lora::cf;
using lora::KArgs;

namespace lora {
thread_local LaunchRecord* t_launch_record = nullptr;
}  // namespace lora

namespace {

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return set_error(LORA_EIO, std::string(#expr) + ": " + hipGetErrorString(e_));      \
  } while (0)

using lora::PI_F;

// ---------------------------------------------------------------------------------
// Host-side table generation (runs once per plan, on the host, with the reference's
// exact formulas and the host libm, so the device sees the reference's constants).
// ---------------------------------------------------------------------------------

}  // namespace

// ChirpGenerator.hpp:105-132 (genChirp), float recurrence, std::polar -> sincosf.
void lora::host_gen_chirp(std::complex<float>* out, int N, int osr, int NN, float f0, bool down,
                          float ampl, float& phase, float bw_scale) {
  const float fMin = -M_PI * bw_scale / osr;
  const float fMax = M_PI * bw_scale / osr;
  const float fStep = (2 * M_PI * bw_scale) / (N * osr * osr);
  float f = fMin + f0;
  for (int i = 0; i < NN; i++) {
    f += fStep;
    if (f > fMax) f -= (fMax - fMin);
    if (down)
      phase -= f;
    else
      phase += f;
    float s, c;
    sincosf(phase, &s, &c);
    out[i] = std::complex<float>(ampl * c, ampl * s);
  }
  phase -= std::floor(phase / (2 * M_PI)) * 2 * M_PI;
}

namespace {
using lora::host_gen_chirp;

// kissfft.hh:81-97: radix plan; only 4/2 radices occur for powers of two.
std::vector<int> fft_radices(int nfft) {
  std::vector<int> r;
  int n = nfft, p = 4;
  do {
    while (n % p) {
      p = (p == 4) ? 2 : (p == 2) ? 3 : p + 2;
      if (p * p > n) p = n;
    }
    n /= p;
    r.push_back(p);
  } while (n > 1);
  return r;
}

// Leaf order of kf_work (kissfft.hh:106-131): out position -> input index.
void leaf_order(const std::vector<int>& radix, int stage, int out_pos, int in_idx, int fstride,
                int len, std::vector<uint16_t>& rev) {
  const int p = radix[stage];
  const int m = len / p;
  if (m == 1) {
    for (int j = 0; j < p; ++j) rev[in_idx + j * fstride] = (uint16_t)(out_pos + j);
    return;
  }
  for (int q = 0; q < p; ++q)
    leaf_order(radix, stage + 1, out_pos + q * m, in_idx + q * fstride, fstride * p, m, rev);
}

float bw_scale_of(unsigned bw_hz) { return static_cast<float>(bw_hz) / 125000.0f; }  // phy.hpp:47-49

bool bw_ok(unsigned bw) { return bw == 125000 || bw == 250000 || bw == 500000; }

// k_frame_max blocks per frame: rounded DOWN, so each block streams at least one full
// batch of 4096 samples (256 threads x 8 pairs): SF7 frames of 8448 samples as 2 x 4224
// rather than 3 x 2816 (partly idle batches); SF12 66 x 4096; at most kMaxBpf (longer
// frames use longer blocks).
constexpr int kMaxChunk = 4096;
int frame_max_blocks(int64_t frame_len) {
  return frame_len > 0 ? (int)std::min<int64_t>(lora::kMaxBpf, std::max<int64_t>(1, frame_len / kMaxChunk)) : 1;
}

// Workspace of one lora_demod_batch call, sized from the frames (no zeroing pass, no
// atomics on it): per-frame partial maxima (k_frame_max blocks; the speculative pipeline
// uses the first slot), the exact FrameParams, the pre-pass FrameParams, one 8-byte
// speculative entry per symbol and the certification's reject list.
struct WsLayout {
  size_t fp, fp_spec, marg, fix, total;
  int64_t fix_cap;  // entries per stripe of the reject list
};
WsLayout ws_layout(int64_t frames, int64_t frame_len, int step, int N) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const int64_t total = std::max<int64_t>(0, frame_len / step);
  const int64_t per = std::max<int64_t>(0, total - 2);
  WsLayout w;
  w.fp = al((size_t)frames * frame_max_blocks(frame_len) * sizeof(uint32_t));
  w.fp_spec = w.fp + al((size_t)frames * sizeof(lora::FrameParams));
  w.marg = w.fp_spec + al((size_t)frames * sizeof(lora::FrameParams));
  // one 8-byte entry per symbol (KArgs::spec_marg)
  w.fix = w.marg + al((size_t)frames * total * 2 * sizeof(float));
  // the certification's reject list: kFixStripes counts, then per stripe up to every data
  // symbol's (frame, j) and one sync-word entry per frame of its workgroups
  const int64_t spb = lora::est_frames_per_block(N);
  const int64_t wgs = (frames + spb - 1) / spb;
  w.fix_cap = (wgs + lora::kFixStripes - 1) / lora::kFixStripes * spb * (per + 1);
  // (LORA_MODE_RAW's certification lists from blocks of 256 symbols, every symbol an entry)
  const int64_t rblocks = (frames * total + 255) / 256;
  w.fix_cap = std::max<int64_t>(w.fix_cap, (rblocks + lora::kFixStripes - 1) / lora::kFixStripes * 256);
  w.total = w.fix + al(64 * lora::kFixStripes + (size_t)lora::kFixStripes * w.fix_cap * 2 * sizeof(uint32_t));
  return w;
}

// ---------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------

// Load sample j of a frame after the LEGACY caller-side dechirp and the
// normalisation of LoRaDemod.cpp:68-77 (z = y * (1/max) when max > 1).
__device__ __forceinline__ cf load_legacy(const cf* __restrict__ x, int64_t j,
                                          const cf* __restrict__ down, int step, int dechirp,
                                          int scaled, float scale) {
  cf v = x[j];
  if (dechirp) v = lora::cmul(v, down[j % step]);
  if (scaled) v = lora::cscale(v, scale);
  return v;
}


// Point i of symbol s of frame f, rotated/windowed, as fed to the detector
// (LoRaDemod.cpp:142-162; phy.cpp:205-225 for API mode).
__device__ __forceinline__ cf symbol_point(const KArgs& a, const cf* __restrict__ x,
                                           const lora::FrameParams& p, int s, int i) {
  int64_t base = (int64_t)s * a.step;
  if (p.t_off > 0) {
    if (base + p.t_off + a.step <= a.frame_len) base += p.t_off;
  } else if (p.t_off < 0) {
    const int64_t off = -(int64_t)p.t_off;
    if (off <= base) base -= off;
  }
  const float start = p.rate * ((float)((uint32_t)s * (uint32_t)a.N) +
                                (float)p.t_off / (float)a.osr);
  const int64_t j = base + (int64_t)i * a.osr;
  if (a.mode == LORA_MODE_RAW) {  // detector only: (dechirp) -> (window)
    cf v = load_legacy(x, j, a.down, a.step, a.dechirp, 0, 1.0f);
    if (a.hann) v = lora::cscale(v, a.win[i]);
    return v;
  }
  const float ph = start + p.rate * (float)i;
  float sn, cs;
  lm_sincosf(ph, &sn, &cs);
  cf v;
  if (a.mode == LORA_MODE_API) {
    v = lora::cmul(lora::cmul(x[j], a.down1[i]), cf{cs, sn});
  } else {
    v = lora::cmul(load_legacy(x, j, a.down, a.step, a.dechirp, p.scaled, p.scale), cf{cs, sn});
  }
  if (a.hann) v = lora::cscale(v, a.win[i]);
  return v;
}

// Workgroup argmax of one N-point spectrum in LDS (natural order).  Returns the
// key to every thread.
__device__ __forceinline__ uint64_t wg_argmax(const cf* A, int N, uint64_t* red) {
  uint64_t k = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) k = lora::umax64(k, lora::argmax_key(A[i], i));
  k = lora::group_max(k, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = k;
  __syncthreads();
  uint64_t r = red[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = lora::umax64(r, red[w]);
  __syncthreads();
  return r;
}

// Offset estimate (LoRaDemod.cpp:79-135 / phy.cpp:78-145) and the two sync symbols
// of frame f, by the whole workgroup (A: N-complex LDS FFT buffer).  `scaled`/`scale`
// carry the normalisation decision (LoRaDemod.cpp:68-77), `maxv` the frame max.
__device__ __forceinline__ void estimate_frame(const KArgs& a, int f, int scaled, float scale,
                                            float maxv, cf* A) {
  __shared__ uint64_t red[4];
  __shared__ lora::FrameParams sp;
  __shared__ uint16_t sw[2];
  const cf* x = a.iq + (int64_t)f * a.frame_stride;
  const int N = a.N;
  const bool raw = a.mode == LORA_MODE_API || a.est_only;
  const int est = a.est_only ? a.total : (a.mode == LORA_MODE_API) ? 2 : min(a.total, 2);
  const bool tie_rule = a.mode == LORA_MODE_LEGACY && !a.est_only;

  // Scalar estimator state lives in thread 0.
  float sum_index = 0.0f, phase_diff = 0.0f, prev_phase = 0.0f;
  bool have_prev = false;
  unsigned sum_t = 0;
  for (int s = 0; s < est; ++s) {
    float best_p = -1e30f, best_fi = 0.0f;
    uint32_t best_idx = 0;
    unsigned best_t = 0;
    cf best_bin = {0.0f, 0.0f};
    for (int t = 0; t < a.osr; ++t) {
      for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int64_t j = (int64_t)s * a.step + t + (int64_t)i * a.osr;
        cf v = raw ? x[j] : load_legacy(x, j, a.down, a.step, a.dechirp, scaled, scale);
        if (a.hann) v = lora::cscale(v, a.win[i]);
        A[a.rev[i]] = v;
      }
      __syncthreads();
      lora::fft_lds(A, a.sf, 1, a.tw, threadIdx.x, blockDim.x);
      const uint64_t key = wg_argmax(A, N, red);
      if (threadIdx.x == 0) {
        const uint32_t idx = lora::key_index(key);
        const float mv = lora::key_value(key);
        float p, fi;
        lora::detect_tail(mv, A[idx > 0 ? idx - 1 : N - 1], A[idx < (uint32_t)N - 1 ? idx + 1 : 0],
                          a.power_scale, &p, &fi);
        if (p > best_p || (tie_rule && p == best_p && idx < best_idx)) {
          best_p = p;
          best_idx = idx;
          best_fi = fi;
          best_t = t;
          best_bin = A[idx];
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      sum_t += best_t;
      sum_index += (float)best_idx + best_fi;
      const float phase = lm_atan2f(best_bin.im, best_bin.re);
      if (have_prev) {
        float d = phase - prev_phase;
        while (d > PI_F) d -= 2.0f * PI_F;
        while (d < -PI_F) d += 2.0f * PI_F;
        phase_diff += d;
      }
      prev_phase = phase;
      have_prev = true;
    }
  }
  if (a.est_only) {  // phy.cpp:87: no whole symbol -> metrics untouched
    if (threadIdx.x == 0 && est > 0) {
      const float avg_index = sum_index / (float)est;
      const float cfo_coarse = avg_index / (float)N;
      float cfo_fine = 0.0f;
      if (est > 1) cfo_fine = (phase_diff / (float)(est - 1)) / (2.0f * PI_F * (float)N);
      const float frac = avg_index - floorf(avg_index + 0.5f);
      const float avg_t = (float)sum_t / (float)est;
      if (a.cfo) a.cfo[f] = cfo_coarse + cfo_fine;
      if (a.toff) a.toff[f] = avg_t - frac * (float)N * (float)a.osr;
    }
    return;
  }
  if (threadIdx.x == 0) {
    const float avg_index = sum_index / (float)est;
    const float cfo_coarse = avg_index / (float)N;
    float cfo_fine = 0.0f;
    if (est > 1) cfo_fine = (phase_diff / (float)(est - 1)) / (2.0f * PI_F * (float)N);
    const float cfo = cfo_coarse + cfo_fine;
    const float frac = avg_index - floorf(avg_index + 0.5f);
    const float avg_t = (float)sum_t / (float)est;
    const float toff = avg_t - frac * (float)N * (float)a.osr;
    lora::FrameParams p;
    p.cfo = cfo;
    p.toff = toff;
    p.t_off = (int)roundf(toff);
    p.rate = -2.0f * PI_F * cfo / (float)N;
    p.scale = scale;
    p.scaled = scaled;
    p.pad0 = p.pad1 = 0;
    sp = p;
    a.fp[f] = p;
    if (a.cfo) a.cfo[f] = cfo;
    if (a.toff) a.toff[f] = toff;
    if (a.max_amp) a.max_amp[f] = maxv;
  }
  __syncthreads();

  // Sync symbols 0 and 1 (LoRaDemod.cpp:165-168, 177-192; phy.cpp:228-237).
  if (a.have_sync) {
    const lora::FrameParams p = sp;
    for (int s = 0; s < 2; ++s) {
      for (int i = threadIdx.x; i < N; i += blockDim.x) A[a.rev[i]] = symbol_point(a, x, p, s, i);
      __syncthreads();
      lora::fft_lds(A, a.sf, 1, a.tw, threadIdx.x, blockDim.x);
      const uint64_t key = wg_argmax(A, N, red);
      if (threadIdx.x == 0) sw[s] = (uint16_t)lora::key_index(key);
      __syncthreads();
    }
    if (threadIdx.x == 0 && a.sync) {
      const unsigned shift = a.sf > 4 ? a.sf - 4 : 0;
      a.sync[f] = (uint8_t)((((sw[0] >> shift) & 0x0f) << 4) | ((sw[1] >> shift) & 0x0f));
    }
  } else if (threadIdx.x == 0 && a.sync) {
    a.sync[f] = 0;
  }
}

// One workgroup per frame.  LEGACY: the normalisation decision from k_frame_max's
// per-frame maximum; API mode / lora_estimate_offsets_batch: raw samples.
__global__ void __launch_bounds__(256) k_estimate(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float maxv = 0.0f;
  if (a.mode == LORA_MODE_LEGACY && !a.est_only) maxv = lora::frame_maxv(a, blockIdx.x);
  const int scaled = maxv > 1.0f;
  estimate_frame(a, blockIdx.x, scaled, scaled ? 1.0f / maxv : 1.0f, maxv,
                 reinterpret_cast<cf*>(smem));
}

// LEGACY: per-frame max(|I|,|Q|) of the (dechirped) samples (LoRaDemod.cpp:59-67),
// streamed by `bpf` blocks per frame (`chunk` samples each, 16-byte loads); block c
// stores its partial maximum in maxbits[f*bpf + c] (the estimate reduces them).
__global__ void __launch_bounds__(256) k_frame_max(KArgs a, int bpf, int chunk,
                                                   uint32_t* __restrict__ maxbits) {
  __shared__ float wmax[4];
  const int64_t f = blockIdx.x / bpf;
  const int64_t c = blockIdx.x - f * bpf;
  const int64_t fb = f * a.frame_stride;
  const cf* x = a.iq + fb;
  const int step = a.step;
  const int64_t j0 = c * (int64_t)chunk;
  const int64_t j1 = min(j0 + (int64_t)chunk, a.frame_len);
  float m = 0.0f;
  if ((fb & 1) == 0) {  // 16-byte aligned frame (chunk starts are even)
    // Batches of KB pairs per thread: all IQ loads, then all table loads, then the
    // math, so each batch costs one memory round trip.
    constexpr int KB = 8;
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int64_t p0 = j0 >> 1, p1 = j1 >> 1;
    const int stride = (int)blockDim.x;
    int d = (int)((j0 + 2 * (int64_t)threadIdx.x) % step);
    const int inc = (2 * stride) % step;
    for (int64_t pb = p0 + threadIdx.x; pb < p1; pb += (int64_t)KB * stride) {
      f4v q[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const int64_t pr = pb + (int64_t)k * stride;
        // nontemporal: a once-read stream (the symbol pass re-reads it much later);
        // measured 8 % faster at SF7, 4 % at SF12 (tools/exp/maxpass_exp.sh)
        q[k] = pr < p1 ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x + 2 * pr))
                       : f4v{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (a.dechirp) {
        cf w0[KB], w1[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const int d1 = (d + 1 == step) ? 0 : d + 1;
          w0[k] = a.down[d];
          w1[k] = a.down[d1];
          d += inc;
          if (d >= step) d -= step;
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const cf v0 = lora::cmul(cf{q[k][0], q[k][1]}, w0[k]);
          const cf v1 = lora::cmul(cf{q[k][2], q[k][3]}, w1[k]);
          m = fmaxf(m, fmaxf(fmaxf(fabsf(v0.re), fabsf(v0.im)), fmaxf(fabsf(v1.re), fabsf(v1.im))));
        }
      } else {
#pragma unroll
        for (int k = 0; k < KB; ++k)
          m = fmaxf(m, fmaxf(fmaxf(fabsf(q[k][0]), fabsf(q[k][1])), fmaxf(fabsf(q[k][2]), fabsf(q[k][3]))));
      }
    }
    if ((j1 & 1) && threadIdx.x == 0) {  // odd end of the frame
      cf v = x[j1 - 1];
      if (a.dechirp) v = lora::cmul(v, a.down[(j1 - 1) % step]);
      m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
    }
  } else {
    for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
      cf v = x[j];
      if (a.dechirp) v = lora::cmul(v, a.down[j % step]);
      m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    maxbits[f * a.mx_bpf + c] = __float_as_uint(r);  // partial c of frame f
  }
}

// Short frames (one k_frame_max block per frame would stream less than two 4096-sample
// batches): one wave per frame, 4 frames per 256-thread block, the same 16-byte batched
// loads with the wave's 64 lanes striding the frame; the wave's maximum is the frame's
// single partial (mx_bpf = 1).  configs[4]'s 18-symbol SF7 frames (2304 samples): the
// block-per-frame pass ran at 4.9 TB/s.
__global__ void __launch_bounds__(256) k_frame_max_wave(KArgs a, int64_t frames,
                                                        uint32_t* __restrict__ maxbits) {
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= frames) return;  // whole waves exit together
  const int t = threadIdx.x & 63;
  const int64_t fb = f * a.frame_stride;
  const cf* x = a.iq + fb;
  const int step = a.step;
  const int64_t len = a.frame_len;
  float m = 0.0f;
  if ((fb & 1) == 0) {
    constexpr int KB = 8;
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int64_t p1 = len >> 1;
    int d = (2 * t) % step;
    const int inc = 128 % step;
    for (int64_t pb = t; pb < p1; pb += (int64_t)KB * 64) {
      f4v q[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const int64_t pr = pb + (int64_t)k * 64;
        q[k] = pr < p1 ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x + 2 * pr))
                       : f4v{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (a.dechirp) {
        cf w0[KB], w1[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const int d1 = (d + 1 == step) ? 0 : d + 1;
          w0[k] = a.down[d];
          w1[k] = a.down[d1];
          d += inc;
          if (d >= step) d -= step;
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const cf v0 = lora::cmul(cf{q[k][0], q[k][1]}, w0[k]);
          const cf v1 = lora::cmul(cf{q[k][2], q[k][3]}, w1[k]);
          m = fmaxf(m, fmaxf(fmaxf(fabsf(v0.re), fabsf(v0.im)), fmaxf(fabsf(v1.re), fabsf(v1.im))));
        }
      } else {
#pragma unroll
        for (int k = 0; k < KB; ++k)
          m = fmaxf(m, fmaxf(fmaxf(fabsf(q[k][0]), fabsf(q[k][1])), fmaxf(fabsf(q[k][2]), fabsf(q[k][3]))));
      }
    }
    if ((len & 1) && t == 0) {  // odd frame length: the last sample
      cf v = x[len - 1];
      if (a.dechirp) v = lora::cmul(v, a.down[(len - 1) % step]);
      m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
    }
  } else {
    for (int64_t j = t; j < len; j += 64) {
      cf v = x[j];
      if (a.dechirp) v = lora::cmul(v, a.down[j % step]);
      m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (t == 0) maxbits[f] = __float_as_uint(m);
}

// phy.cpp:147-176 (compensate_offsets), out of place: rotation by rate*n first,
// then the integer shift with zero fill.
__global__ void __launch_bounds__(256) k_compensate(const cf* __restrict__ in, cf* __restrict__ out,
                                                    int64_t frame_len, int64_t frame_stride,
                                                    int64_t frames, float Nosr,
                                                    const float* __restrict__ cfo,
                                                    const float* __restrict__ toff) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= frames * frame_len) return;
  const int64_t f = gid / frame_len;
  const int64_t n = gid - f * frame_len;
  const float rate = -2.0f * PI_F * cfo[f] / Nosr;
  const int offset = (int)roundf(toff[f]);
  int64_t src = n;
  bool zero = false;
  if (offset > 0 && (int64_t)offset < frame_len) {
    src = n - offset;
    zero = src < 0;
  } else if (offset < 0 && -(int64_t)offset < frame_len) {
    src = n - offset;
    zero = src >= frame_len;
  }
  cf v = {0.0f, 0.0f};
  if (!zero) {
    const float ph = rate * (float)(uint64_t)src;
    float sn, cs;
    lm_sincosf(ph, &sn, &cs);
    v = lora::cmul(in[f * frame_stride + src], cf{cs, sn});
  }
  out[f * frame_stride + n] = v;
}

// ---------------------------------------------------------------------------------
// Modulator (LoRaMod.cpp:8-43): chirp start phases by one lane per frame (the fp32
// phase recurrence is sequential), then one lane per chirp emits its samples.
// ---------------------------------------------------------------------------------
struct ModArgs {
  int N, osr, step, nchirp;
  int fpw;  // k_mod_phase: frames per 64-lane wave (lanes >= fpw idle)
  float fMin, fMax, fStep, ampl, bw_scale;
  uint16_t sw0, sw1;
  const uint16_t* syms;
  int64_t sym_count;
  cf* iq;
  int64_t frames;
  // k_mod_frame: the configuration's run tables (mod_run_table), runs of chirp value v at
  // seg[v * seg_cap], their count at cnt[v] (-1: over the cap), for v < seg_n; null: none
  const lora::ChirpSeg* seg;
  const int* cnt;
  int seg_n, seg_cap;
};

__device__ __forceinline__ unsigned chirp_value(const ModArgs& a, int64_t frame, int c) {
  return c == 0 ? a.sw0 : c == 1 ? a.sw1 : a.syms[frame * a.sym_count + (c - 2)];
}
__device__ __forceinline__ float chirp_f0(const ModArgs& a, int64_t frame, int c) {
  const unsigned v = chirp_value(a, frame, c);
  return (2.0f * PI_F * (float)(int)v * a.bw_scale) / ((float)a.N * (float)a.osr);
}

// glibc sincosf of one sample per lane, the reduction chosen per wave: the fast one when
// every active lane's |y| < 120, the Payne-Hanek one when every |y| is in [120, inf) (an
// SF12 chirp's phases, mid-chirp), else both evaluated and selected (lm_sincosf_bf).  The
// results are lm_sincosf's in every case (tests/native/libm_check: each form vs glibc).
__device__ __forceinline__ void mod_sincosf(float y, float* s, float* c) {
  if (__all(lm_sincosf_fast_ok(y)))
    lm_sincosf_fast(y, s, c);
  else if (__all(lm_sincosf_large_ok(y)))
    lm_sincosf_large(y, s, c);
  else
    lm_sincosf_bf(y, s, c);
}

// mod_sincosf of two samples per lane, the reduction chosen per wave for both
__device__ __forceinline__ void mod_sincosf2(float y0, float y1, float* s, float* c) {
  if (__all(lm_sincosf_fast_ok(y0) && lm_sincosf_fast_ok(y1))) {
    const float y[2] = {y0, y1};
    lm_sincosf_fast_k<2>(y, s, c);
  } else if (__all(lm_sincosf_large_ok(y0) && lm_sincosf_large_ok(y1))) {
    lm_sincosf_large(y0, &s[0], &c[0]);
    lm_sincosf_large(y1, &s[1], &c[1]);
  } else {
    lm_sincosf_bf(y0, &s[0], &c[0]);
    lm_sincosf_bf(y1, &s[1], &c[1]);
  }
}

// K steps of the genChirp recurrence (ChirpGenerator.hpp:118-128: f += fStep, wrap at
// fMax, phase += f, all fp32), speculatively without the wrap: fStep > 0, so f only grows
// between wraps and the K unwrapped steps are the recurrence's own exactly when the last
// f stays <= fMax; otherwise (once per chirp) the K steps are redone with the wrap.  Two
// VALU operations per step instead of five.  ph[k] (optional) receives the phases.
template <int K>
__device__ __forceinline__ void chirp_steps(float& f, float& phase, float fStep, float fMax, float span, float* ph) {
  float ft = f, pt = phase;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    ft += fStep;
    pt += ft;
    if (ph) ph[k] = pt;
  }
  if (ft > fMax) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      f += fStep;
      f = f > fMax ? f - span : f;
      phase += f;
      if (ph) ph[k] = phase;
    }
  } else {
    f = ft;
    phase = pt;
  }
}

// The start phase of every chirp of a frame: one lane per frame runs the frame's whole
// chain (sequential by construction: each chirp starts from the previous one's wrapped end
// phase).  For long chirps the chain's length, not the work, sets the kernel's time, so the
// frames are spread a.fpw per wave over about a thousand waves (at most one per SIMD), which
// also keeps chirp_steps' redo (a lane's wrap in a block) rare per wave (SF12, 15,625 frames:
// 3.47 -> 1.99 ms).
__global__ void k_mod_phase(ModArgs a) {
  if ((int)threadIdx.x >= a.fpw) return;
  const int64_t fr = (int64_t)blockIdx.x * a.fpw + threadIdx.x;
  if (fr >= a.frames) return;
  cf* out = a.iq + fr * (int64_t)a.nchirp * a.step;
  float phase = 0.0f;
  const float span = a.fMax - a.fMin;
  for (int c = 0; c < a.nchirp; ++c) {
    out[(int64_t)c * a.step].re = phase;  // start phase, consumed by k_mod_samples
    float f = a.fMin + chirp_f0(a, fr, c);
    // (a wave redoes a block when any of its fpw lanes wraps in it: one block in step / 16
    // per lane, so only long chirps gain)
    if (a.step >= 1024 && a.step % 16 == 0) {
      for (int i = 0; i < a.step; i += 16) chirp_steps<16>(f, phase, a.fStep, a.fMax, span, nullptr);
    } else {
      // unrolled: 5 VALU per sample, no scalar loop overhead (SF7: 0.29 -> 0.14 ms)
#pragma unroll 16
      for (int i = 0; i < a.step; ++i) {
        f += a.fStep;
        f = f > a.fMax ? f - span : f;
        phase += f;
      }
    }
    phase = (float)((double)phase - floor((double)phase / (2 * M_PI)) * 2 * M_PI);
  }
}

// One wave per 64 chirps, four waves per workgroup.  The genChirp recurrence
// (ChirpGenerator.hpp:118-128: f += fStep, wrap, phase += f, all fp32) is inherently
// sequential, so each lane advances its own chirp kModBatch samples at a time into the
// wave's LDS tile; the wave then evaluates sincosf over the transposed tile, four chirps
// x 16 consecutive samples per store instruction (128-B segments).  The narrow tile
// (64 x 17 floats per wave) keeps up to 8 waves per SIMD resident, which is what hides
// the recurrence's dependent-add latency (the former 64 x 65 tile allowed ~2).
constexpr int kModLanes = 64;
constexpr int kModBatch = 16;
constexpr int kModWaves = 4;
__global__ void __launch_bounds__(kModLanes * kModWaves) k_mod_samples(ModArgs a) {
  __shared__ float tiles[kModWaves][kModLanes][kModBatch + 1];  // [wave][chirp][sample]
  const int lane = threadIdx.x & (kModLanes - 1);
  const int wv = threadIdx.x / kModLanes;
  float(*tile)[kModBatch + 1] = tiles[wv];
  const int64_t nch = a.frames * (int64_t)a.nchirp;
  const int64_t w0 = ((int64_t)blockIdx.x * kModWaves + wv) * kModLanes;
  if (w0 >= nch) return;  // whole waves exit together; no workgroup barrier below
  const int64_t w = w0 + lane;
  const bool valid = w < nch;
  const int64_t wc = valid ? w : nch - 1;
  const int64_t fr = wc / a.nchirp;
  const int c = (int)(wc - fr * a.nchirp);
  float phase = a.iq[wc * a.step].re;  // start phase from k_mod_phase
  float f = a.fMin + chirp_f0(a, fr, c);
  const float span = a.fMax - a.fMin;
  const int nvalid = (int)min((int64_t)kModLanes, nch - w0);
  // store role of this lane: chirp sub-row (lane >> 4) and sample (lane & 15)
  const int sub = lane >> 4, j = lane & (kModBatch - 1);
  for (int i0 = 0; i0 < a.step; i0 += kModBatch) {
    const int cnt = min(kModBatch, a.step - i0);
    // (64 chirps per wave: the speculation pays only when a wave's blocks rarely hold a wrap)
    if (cnt == kModBatch && a.step >= 4096) {
      chirp_steps<kModBatch>(f, phase, a.fStep, a.fMax, span, tile[lane]);
    } else {
      for (int k = 0; k < cnt; ++k) {
        f += a.fStep;
        if (f > a.fMax) f -= span;
        phase += f;
        tile[lane][k] = phase;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (j < cnt) {
      for (int ch = sub; ch < nvalid; ch += kModLanes / kModBatch) {
        float sn, cs;
        mod_sincosf(tile[ch][j], &sn, &cs);
        a.iq[(w0 + ch) * a.step + i0 + j] = cf{a.ampl * cs, a.ampl * sn};
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}


// ---- few frames: one workgroup per frame (k_mod_frame) ------------------------------
// With few frames the bulk kernels above leave the chip idle while one lane per frame
// walks the whole frame's recurrence at five dependent operations per sample (SF7, one
// frame: ~180 us).  Here a frame's samples go through windows of <= 2048 samples in a
// four-stage pipeline over one workgroup:
//   * waves 1-3 fill window t+1 with its frequencies - short chirps (< kMfTabMin samples)
//     by one lane per chirp running the frequency recurrence, long ones from the runs of
//     lora_chirp.h (built one window ahead by a few lanes, then evaluated in parallel);
//   * lane 0 of wave 0 runs window t's phase additions (ChirpGenerator.hpp:121), the one
//     truly sequential part - one dependent fp32 add per sample, the frequencies read two
//     blocks ahead - and records the phase at the start of each 32-sample block (and the
//     per-chirp wrap, :130);
//   * waves 1-3 recompute window t-1's phases block by block from those starts (the same
//     additions, in parallel), then evaluate window t-2's samples (glibc-exact sincosf,
//     :122) with coalesced stores.
// A dependent add issues every ~4.6 cycles on one wave; a DS store per sample in the chain
// lane cost 14-15 cycles per sample (tools/micro/chain_rate.hip), hence the block starts.
// Results are the recurrence's own, bit for bit (the runs are exact, chirp_seg_check).
constexpr int kMfWin = 2048;     // samples per window (whole chirps, or an exact fraction of one)
constexpr int kMfBlk = 32;       // samples per recorded block start
constexpr int kMfPad = 2 * kMfBlk;  // the chain's read-ahead past a window
constexpr int kMfTabMin = 512;   // chirps of at least this many samples take runs
constexpr int kMfTabChirps = kMfWin / kMfTabMin;  // long chirps per window
constexpr int kMfSegMax = 92;    // runs per chirp: lora::chirp_seg_cap(12)
static_assert(kMfSegMax >= lora::chirp_seg_cap(12), "run table per chirp");
constexpr int kMfThreads = 256;
constexpr int kMfWorkers = kMfThreads - 64;
constexpr int64_t kMfMaxFrames = 512;  // at most this many frames take k_mod_frame

// The runs of every chirp value v < n of one configuration (one lane per value), for
// k_mod_frame's long chirps: built once per (device, sf, osr, bandwidth) by mod_run_table,
// so the frame kernel copies a chirp's table instead of deriving it (one lane, ~650 cycles
// per run: 44 k cycles per SF12 chirp - more than the chirp's whole phase chain).
__global__ void __launch_bounds__(64) k_mod_runs(ModArgs a, int n, int cap, lora::ChirpSeg* seg, int* cnt) {
  const int v = blockIdx.x * 64 + threadIdx.x;
  if (v >= n) return;
  const lora::ChirpConst cc{a.fMin, a.fMax, a.fStep, a.fMax - a.fMin};
  const float f0 = (2.0f * PI_F * (float)v * a.bw_scale) / ((float)a.N * (float)a.osr);  // chirp_f0's
  cnt[v] = lora::chirp_segments(a.fMin + f0, a.step, cc, seg + (size_t)v * cap, cap);
}

// window t's table group: a window of whole chirps is its own group, the windows of one
// long chirp share the chirp's
__device__ __forceinline__ int mf_group(int t, int W, int step) { return step <= W ? t : (int)((int64_t)t * W / step); }

// ChirpGenerator.hpp:130, after a chirp's last sample
__device__ __forceinline__ float mf_wrap(float phase) {
  return (float)((double)phase - floor((double)phase / (2 * M_PI)) * 2 * M_PI);
}

__global__ void __launch_bounds__(kMfThreads) k_mod_frame(ModArgs a, int W, int nwin) {
  __shared__ __attribute__((aligned(16))) float buf[4][kMfWin + kMfPad];
  __shared__ float pst[4][kMfWin / kMfBlk];  // phase before each block's first sample
  __shared__ lora::ChirpSeg tab[2][kMfTabChirps][kMfSegMax];
  __shared__ int tcnt[2][kMfTabChirps];
  const int64_t fr = blockIdx.x;
  cf* out = a.iq + fr * (int64_t)a.nchirp * a.step;
  const int tid = threadIdx.x;
  const int wk = tid - 64;  // worker index (waves 1-3), < 0 in wave 0
  const lora::ChirpConst cc{a.fMin, a.fMax, a.fStep, a.fMax - a.fMin};
  const int64_t total = (int64_t)a.nchirp * a.step;
  const bool runs = a.step >= kMfTabMin;
  const int cap = lora::chirp_seg_cap(31 - __builtin_clz((unsigned)a.N));
  // runs of the long chirps starting in window t, into slot group(t) % 2, by the last
  // workers (the others fill and evaluate meanwhile)
  const int nbuild = runs ? (a.step <= W ? W / a.step : 1) : 0;
  const int nwk = kMfWorkers - nbuild;  // workers that fill and evaluate
  auto wlen = [&](int t) { return (int)min((int64_t)W, total - (int64_t)t * W); };
  auto build = [&](int t) {
    const int j = wk - nwk;
    if (!runs || j < 0 || t >= nwin) return;
    if (t > 0 && mf_group(t, W, a.step) == mf_group(t - 1, W, a.step)) return;  // same chirp
    const int64_t s0 = (int64_t)t * W;
    const int c = (int)(s0 / a.step) + j;
    if (c >= a.nchirp || (int64_t)c * a.step >= s0 + W) return;
    const int slot = mf_group(t, W, a.step) & 1;
    const unsigned v = chirp_value(a, fr, c);
    if (a.seg && (int)v < a.seg_n) {
      // the precomputed runs of this chirp value (mod_run_table): a copy, 16 bytes per load
      const int nr = min(a.cnt[v], kMfSegMax);  // (< 0: the runs overflowed, the recurrence below)
      tcnt[slot][j] = nr;
      const uint4* src = reinterpret_cast<const uint4*>(a.seg + (size_t)v * a.seg_cap);
      uint4* dst = reinterpret_cast<uint4*>(tab[slot][j]);
      for (int r = 0; r < nr; ++r) dst[r] = src[r];
    } else {
      tcnt[slot][j] = lora::chirp_segments(a.fMin + chirp_f0(a, fr, c), a.step, cc, tab[slot][j], cap);
    }
  };
  // window t's frequencies into buf[t % 4]
  auto fill = [&](int t) {
    if (wk < 0 || wk >= nwk || t >= nwin) return;
    const int64_t s0 = (int64_t)t * W;
    const int n = wlen(t);
    float* b = buf[t % 4];
    if (!runs) {
      // whole short chirps, one lane each: the recurrence itself
      // (four values per store: a DS store reads its data after issue, so one store per step
      // made each step wait for the previous store)
      // (and two quads per round in registers of their own: a quad's registers are rewritten
      // only after the other quad's store has been issued)
      for (int c = wk; c < n / a.step; c += nwk) {
        float f = a.fMin + chirp_f0(a, fr, (int)(s0 / a.step) + c);
        float4* bc = reinterpret_cast<float4*>(b + c * a.step);  // step % 4 == 0, 16-byte aligned
        auto quad = [&](float4& v) {
          v.x = f = lora::chirp_fstep(f, cc);
          v.y = f = lora::chirp_fstep(f, cc);
          v.z = f = lora::chirp_fstep(f, cc);
          v.w = f = lora::chirp_fstep(f, cc);
        };
        int k = 0;
        for (; k + 2 <= a.step / 4; k += 2) {
          float4 va, vb;
          quad(va);
          bc[k] = va;
          quad(vb);
          bc[k + 1] = vb;
        }
        if (k < a.step / 4) {
          float4 va;
          quad(va);
          bc[k] = va;
        }
      }
      return;
    }
    const int slot = mf_group(t, W, a.step) & 1;
    const int per = (n + nwk - 1) / nwk;
    int i = wk * per;
    const int i1 = min(n, i + per);
    while (i < i1) {
      const int64_t g = s0 + i;
      const int c = (int)(g / a.step);
      const int j = c - (int)(s0 / a.step);  // the chirp's table in the slot
      int k = (int)(g - (int64_t)c * a.step) + 1;
      const int iend = min(i1, i + (a.step - k + 1));
      const int ns = tcnt[slot][j];
      if (ns < 0) {
        // (runs overflowed their cap - a start frequency far outside [fMin, fMax], a
        // symbol >= N: the recurrence from the chirp's start)
        float f = a.fMin + chirp_f0(a, fr, c);
        for (int q = 0; q < k - 1; ++q) f = lora::chirp_fstep(f, cc);
        for (; i < iend; ++i) {
          f = lora::chirp_fstep(f, cc);
          b[i] = f;
        }
        continue;
      }
      const lora::ChirpSeg* S = tab[slot][j];
      int lo = 0, hi = ns - 1;  // the last run with k0 <= k
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S[mid].k0 <= k) lo = mid;
        else hi = mid - 1;
      }
      for (; i < iend; ++i, ++k) {
        while (k >= S[lo].k0 + S[lo].len) ++lo;
        b[i] = lora::chirp_seg_f(S[lo], k);
      }
    }
  };
  // window t's phase additions (lane 0 only): the block starts into pst[t % 4]
  auto chain = [&](int t, float& phase) {
    const int64_t s0 = (int64_t)t * W;
    const int n = wlen(t);
    const float* b = buf[t % 4];
    float* ps = pst[t % 4];
    if (a.step % kMfBlk == 0) {
      // chirp ends fall on block ends; two blocks in flight, each block's frequencies
      // requested a block ahead (the loads past the window read its pad: unused); the
      // scheduling barriers keep the requests where they are
      float4 xa[kMfBlk / 4], xb[kMfBlk / 4];
      auto ld = [&](float4* x, int i) {
#pragma unroll
        for (int q = 0; q < kMfBlk / 4; ++q) x[q] = reinterpret_cast<const float4*>(b + i)[q];
      };
      int left = a.step - (int)(s0 % a.step);  // samples to the next chirp end (one division per window)
      auto run = [&](const float4* x, int i) {
        ps[i / kMfBlk] = phase;
#pragma unroll
        for (int q = 0; q < kMfBlk / 4; ++q) {
          phase = phase + x[q].x;
          phase = phase + x[q].y;
          phase = phase + x[q].z;
          phase = phase + x[q].w;
        }
        left -= kMfBlk;
        if (left == 0) {
          phase = mf_wrap(phase);
          left = a.step;
        }
      };
      ld(xa, 0);
      ld(xb, kMfBlk);
      int i = 0;
      for (; i + 2 * kMfBlk <= n; i += 2 * kMfBlk) {
        run(xa, i);
        __builtin_amdgcn_sched_barrier(0);
        ld(xa, i + 2 * kMfBlk);
        __builtin_amdgcn_sched_barrier(0);
        run(xb, i + kMfBlk);
        __builtin_amdgcn_sched_barrier(0);
        ld(xb, i + 3 * kMfBlk);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (i < n) run(xa, i);  // (n an odd number of blocks)
    } else {
      int left = a.step - (int)(s0 % a.step);
      for (int i = 0; i < n; ++i) {
        if (i % kMfBlk == 0) ps[i / kMfBlk] = phase;
        phase += b[i];
        if (--left == 0) {
          phase = mf_wrap(phase);
          left = a.step;
        }
      }
    }
  };
  // window t's phases, block by block from the recorded starts, in place of the frequencies
  auto recompute = [&](int t) {
    if (wk < 0 || wk >= nwk) return;
    const int64_t s0 = (int64_t)t * W;
    const int n = wlen(t);
    float* b = buf[t % 4];
    const float* ps = pst[t % 4];
    const bool aligned = a.step % kMfBlk == 0;  // chirp ends only at block ends
    for (int blk = wk; blk * kMfBlk < n; blk += nwk) {
      float phase = ps[blk];
      const int i0 = blk * kMfBlk, i1 = min(n, i0 + kMfBlk);
      if (aligned) {
        // a whole block: its frequencies in, 32 additions in registers, its phases out
        float4 x[kMfBlk / 4];
#pragma unroll
        for (int q = 0; q < kMfBlk / 4; ++q) x[q] = reinterpret_cast<const float4*>(b + i0)[q];
#pragma unroll
        for (int q = 0; q < kMfBlk / 4; ++q) {
          x[q].x = phase = phase + x[q].x;
          x[q].y = phase = phase + x[q].y;
          x[q].z = phase = phase + x[q].z;
          x[q].w = phase = phase + x[q].w;
        }
#pragma unroll
        for (int q = 0; q < kMfBlk / 4; ++q) reinterpret_cast<float4*>(b + i0)[q] = x[q];
      } else {
        int left = a.step - (int)((s0 + i0) % a.step);
        for (int i = i0; i < i1; ++i) {
          phase = phase + b[i];
          b[i] = phase;
          if (--left == 0) {
            phase = mf_wrap(phase);
            left = a.step;
          }
        }
      }
    }
  };
  // window t's samples (ChirpGenerator.hpp:122: polar(ampl, phase)), coalesced
  auto emit = [&](int t) {
    if (wk < 0 || wk >= nwk) return;
    const int64_t s0 = (int64_t)t * W;
    const int n = wlen(t);
    const float* b = buf[t % 4];
    // two samples per lane at a time: two independent double-precision chains in flight
    int i = wk;
    for (; i + nwk < n; i += 2 * nwk) {
      float sn[2], cs[2];
      mod_sincosf2(b[i], b[i + nwk], sn, cs);
      out[s0 + i] = cf{a.ampl * cs[0], a.ampl * sn[0]};
      out[s0 + i + nwk] = cf{a.ampl * cs[1], a.ampl * sn[1]};
    }
    if (i < n) {
      float sn, cs;
      mod_sincosf(b[i], &sn, &cs);
      out[s0 + i] = cf{a.ampl * cs, a.ampl * sn};
    }
  };
  float phase = 0.0f;
  // the chain's wave first in the CU's arbitration (its LDS reads queue behind the workers'):
  // one SF12 frame 1.124 -> 1.090 ms, SF7 unchanged (tools/exp/mod_ab.py --few)
  if (wk < 0) __builtin_amdgcn_s_setprio(3);
  build(0);
  __syncthreads();
#ifdef LORA_MF_PROF
  // diagnostics (results invalid): per iteration, shader cycles of the chain (lane 0) and of
  // the fill / build / recompute / emit stages and the barrier (the first and the last
  // worker lane), written over the frame's first samples at the end
  __shared__ uint32_t prof[64][8];
#endif
  for (int t = 0; t < nwin + 3; ++t) {
#ifdef LORA_MF_PROF
    const uint64_t p0 = __builtin_amdgcn_s_memtime();
    uint64_t p1 = p0, p2 = p0, p3 = p0, p4 = p0;
#endif
    if (wk < 0) {
      if (tid == 0 && t >= 1 && t - 1 < nwin) chain(t - 1, phase);
#ifdef LORA_MF_PROF
      p1 = __builtin_amdgcn_s_memtime();
#endif
    } else {
      fill(t);
#ifdef LORA_MF_PROF
      p1 = __builtin_amdgcn_s_memtime();
#endif
      build(t + 1);
#ifdef LORA_MF_PROF
      p2 = __builtin_amdgcn_s_memtime();
#endif
      if (t >= 2 && t - 2 < nwin) recompute(t - 2);
#ifdef LORA_MF_PROF
      p3 = __builtin_amdgcn_s_memtime();
#endif
      if (t >= 3) emit(t - 3);
#ifdef LORA_MF_PROF
      p4 = __builtin_amdgcn_s_memtime();
#endif
    }
    __syncthreads();
#ifdef LORA_MF_PROF
    const uint64_t p5 = __builtin_amdgcn_s_memtime();
    if (t < 64) {
      if (tid == 0) {
        prof[t][0] = (uint32_t)(p1 - p0);
        prof[t][7] = (uint32_t)(p5 - p0);
      }
      if (wk == 0) {
        prof[t][1] = (uint32_t)(p1 - p0);
        prof[t][2] = (uint32_t)(p2 - p1);
        prof[t][3] = (uint32_t)(p3 - p2);
        prof[t][4] = (uint32_t)(p4 - p3);
      }
      if (wk == kMfWorkers - 1) {
        prof[t][5] = (uint32_t)(p2 - p1);  // the last lane: a builder when there are runs
        prof[t][6] = (uint32_t)(p4 - p0);
      }
    }
#endif
  }
#ifdef LORA_MF_PROF
  __syncthreads();
  for (int i = tid; i < 64 * 8; i += kMfThreads) reinterpret_cast<uint32_t*>(out)[i] = prof[i / 8][i % 8];
#endif
}

}  // namespace

// ===================================================================================
// Plan
// ===================================================================================
struct lora_demod_plan {
  lora_demod_params prm;
  int N, step;
  float power_scale;
  void* dev_tables;  // one allocation: tw | down | down1 | win | rev
  cf* tw;
  cf* down;
  cf* down1;
  float* win;
  uint16_t* rev;
  cf* twTA = nullptr;  // pass-A twiddles, slot-major (lora::twT_index), or null
  cf* twTB = nullptr;  // pass-B twiddles, slot-major, or null
  cf* twTB2 = nullptr; // the same in slot pairs (16-byte loads), or null
  cf* downP = nullptr;  // dechirp-table pairs of the speculative demod (osr 1), or null
  int spec;              // speculative single-read pipeline enabled (LORA_MI355X_SPEC, default 1)
  unsigned int* spec_fix = nullptr;  // device counter of symbols the pipeline recomputed
  int last_kernels = 0;  // LORA_KERNEL_* mask of the last lora_demod_batch call
  // measurement hooks (lora_demod_profile_enable): per kernel launch (stage, begin, end)
  struct ProfRec {
    int stage;
    hipEvent_t b, e;
  };
  std::vector<hipEvent_t> prof_pool;
  std::vector<ProfRec> prof_recs;
  int prof_max = 0, prof_calls = 0;
  bool prof_short = false;  // the event pool ran out: the stage sums would be short
};

namespace {

// Event pair around one kernel launch (profiling only; no-op when disabled).
struct ProfScope {
  lora_demod_plan* plan;
  hipStream_t st;
  int stage;
  bool on;
  hipEvent_t e = nullptr;
  ProfScope(lora_demod_plan* p, int s, hipStream_t stream) : plan(p), st(stream), stage(s) {
    on = plan->prof_calls < plan->prof_max && plan->prof_pool.size() >= 2;
    if (plan->prof_calls < plan->prof_max && !on) plan->prof_short = true;  // a launch went untimed
    if (on) {
      hipEvent_t b = plan->prof_pool.back();
      plan->prof_pool.pop_back();
      e = plan->prof_pool.back();
      plan->prof_pool.pop_back();
      hipEventRecord(b, st);
      plan->prof_recs.push_back({stage, b, e});
    }
  }
  ~ProfScope() {
    if (on) hipEventRecord(e, st);
  }
};
}  // namespace

extern "C" {

#ifndef LORA_SRC_HASH
#define LORA_SRC_HASH "unknown"
#endif
#ifndef LORA_GIT_HASH
#define LORA_GIT_HASH "unknown"
#endif
// "src=" is the sha256 (first 16 hex digits) of the library's sources as the Makefile
// hashed them at build time; smoke() recomputes it from the tree it runs in, so a stale
// prebuilt library cannot pass for the current sources.
const char* lora_version(void) {
  return "lora_mi355x 0.2 (gfx950) src=" LORA_SRC_HASH " git=" LORA_GIT_HASH;
}

const char* lora_last_error(void) { return g_last_error.c_str(); }

int lora_demod_last_kernels(const lora_demod_plan* plan) { return plan ? plan->last_kernels : 0; }

int lora_demod_plan_create(const lora_demod_params* params, lora_demod_plan** out) {
  if (!params || !out) return set_error(LORA_EINVAL, "null argument");
  lora_demod_params p = *params;
  if (p.sf < 2 || p.sf > 12) return set_error(LORA_EINVAL, "sf must be in 2..12");
  if (p.osr == 0) p.osr = 1;  // phy.cpp:32
  if (p.osr > 64) return set_error(LORA_EINVAL, "osr must be <= 64");
  if (!bw_ok(p.bw_hz)) return set_error(LORA_EINVAL, "bw_hz must be 125000, 250000 or 500000");
  if (p.window != LORA_WINDOW_NONE && p.window != LORA_WINDOW_HANN)
    return set_error(LORA_EINVAL, "bad window");
  if (p.mode != LORA_MODE_LEGACY && p.mode != LORA_MODE_API && p.mode != LORA_MODE_RAW)
    return set_error(LORA_EINVAL, "bad mode");
  if (p.precision != LORA_PRECISION_EXACT && p.precision != LORA_PRECISION_FAST)
    return set_error(LORA_EINVAL, "bad precision");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (p.device < 0 || p.device >= ndev) return set_error(LORA_EINVAL, "bad device ordinal");

  const int N = 1 << p.sf;
  const int step = N * (int)p.osr;
  const float bws = bw_scale_of(p.bw_hz);
  // kissfft.hh:24-29 twiddles; LoRaDemod.cpp:17-25 window; genChirp down-chirps.
  // The dechirp table holds two periods (2 * step entries) so that a symbol window
  // starting at table phase cg reads down[cg + i*osr] without a per-sample wrap.
  std::vector<std::complex<float>> tw(N), down(2 * (size_t)step), down1(N);
  const float phinc = -2 * std::acos((float)-1) / N;
  for (int i = 0; i < N; ++i) tw[i] = std::exp(std::complex<float>(0, i * phinc));
  float ph = 0.0f;
  host_gen_chirp(down.data(), N, (int)p.osr, step, 0.0f, true, 1.0f, ph, bws);
  for (int i = 0; i < step; ++i) down[step + i] = down[i];
  ph = 0.0f;
  host_gen_chirp(down1.data(), N, 1, N, 0.0f, true, 1.0f, ph, bws);
  std::vector<float> win(N);
  for (int i = 0; i < N; ++i)
    win[i] = p.window == LORA_WINDOW_HANN
                 ? 0.5f - 0.5f * std::cos(2.0f * PI_F * static_cast<float>(i) /
                                          (static_cast<float>(N) - 1.0f))
                 : 1.0f;
  std::vector<uint16_t> rev(N);
  leaf_order(fft_radices(N), 0, 0, 0, 1, N, rev);
  for (int r : fft_radices(N))
    if (r != 2 && r != 4) return set_error(LORA_EINVAL, "unexpected FFT radix");

  // The fast kernels' LDS passes (radix 16 or 4 over butterfly groups k < MA): the
  // twiddles each group uses, stored slot-major (twT[j*MA + k] = tw[index of slot j for
  // group k]) so a wave instruction reads contiguous entries instead of a k-strided
  // gather.  Copies of the same table values: results unchanged (lora::twT_index).
  std::vector<std::complex<float>> twT;
  int twTA_off = -1, twTB_off = -1, twTB2_off = -1;
  if (p.sf >= 6) {
    lora::PassShape ps = lora::pass_shape((int)p.sf);
    auto add = [&](int R, int MA) {
      const int off = (int)twT.size();
      const int slots = R == 16 ? 15 : 3;
      for (int j = 0; j < slots; ++j)
        for (int k = 0; k < MA; ++k) twT.push_back(tw[lora::twT_index(N, MA, j, k)]);
      return off;
    };
    if (ps.RA > 1) twTA_off = add(ps.RA, ps.MA_A);
    if (ps.RB > 1) twTB_off = add(ps.RB, ps.MA_B);
    if (ps.RB > 1) {  // pass B again in slot pairs (lora::KArgs::twTB2), 16-byte aligned
      if (twT.size() & 1) twT.push_back(std::complex<float>(0.0f, 0.0f));
      twTB2_off = (int)twT.size();
      const int slots = ps.RB == 16 ? 15 : 3, MA = ps.MA_B;
      for (int pp = 0; pp < slots / 2; ++pp)
        for (int k = 0; k < MA; ++k) {
          twT.push_back(tw[lora::twT_index(N, MA, 2 * pp, k)]);
          twT.push_back(tw[lora::twT_index(N, MA, 2 * pp + 1, k)]);
        }
      if (slots & 1)
        for (int k = 0; k < MA; ++k) twT.push_back(tw[lora::twT_index(N, MA, slots - 1, k)]);
    }
  }
  // The speculative demod's dechirp-table pairs (lora::KArgs::downP, osr 1): lane l of a
  // window at table phase cg multiplies its points q = 2p, 2p+1 by down[cg + l + T*q];
  // stored as one 16-byte entry per (p, c = cg + l), c < N + T, so a wave instruction reads
  // 64 consecutive entries.  Copies of the same values (the doubled table needs no wrap).
  int downP_off = -1;
  if (p.sf >= 6 && p.osr == 1) {
    if (twT.size() & 1) twT.push_back(std::complex<float>(0.0f, 0.0f));
    downP_off = (int)twT.size();
    const int T = N / 16, C = N + T;
    for (int pp = 0; pp < 8; ++pp)
      for (int c = 0; c < C; ++c) {
        twT.push_back(down[c + T * 2 * pp]);
        twT.push_back(down[c + T * (2 * pp + 1)]);
      }
  }
  const size_t b_tw = sizeof(cf) * N, b_down = sizeof(cf) * 2 * step, b_down1 = sizeof(cf) * N,
               b_win = sizeof(float) * N, b_rev = sizeof(uint16_t) * N, b_twT = sizeof(cf) * twT.size();
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t total = al(b_tw) + al(b_down) + al(b_down1) + al(b_win) + al(b_rev) + al(b_twT) + 256;

  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(p.device));
  void* mem = nullptr;
  if (hipMalloc(&mem, total) != hipSuccess) {
    hipSetDevice(prev);
    return set_error(LORA_ENOMEM, "hipMalloc of plan tables failed");
  }
  unsigned char* b = static_cast<unsigned char*>(mem);
  lora_demod_plan* plan = new lora_demod_plan();
  plan->prm = p;
  plan->N = N;
  plan->step = step;
  plan->power_scale = 20 * std::log10(static_cast<size_t>(N));  // LoRaDetector.hpp:29
  {
    // The one diagnostic knob: LORA_MI355X_SPEC=0 runs the three-launch path (frame max,
    // estimate, demod) instead of the speculative single-read pipeline.
    const char* sp = std::getenv("LORA_MI355X_SPEC");
    plan->spec = !(sp && sp[0] == '0');
  }
  plan->dev_tables = mem;
  plan->tw = reinterpret_cast<cf*>(b);
  b += al(b_tw);
  plan->down = reinterpret_cast<cf*>(b);
  b += al(b_down);
  plan->down1 = reinterpret_cast<cf*>(b);
  b += al(b_down1);
  plan->win = reinterpret_cast<float*>(b);
  b += al(b_win);
  plan->rev = reinterpret_cast<uint16_t*>(b);
  b += al(b_rev);
  cf* twT_dev = twT.empty() ? nullptr : reinterpret_cast<cf*>(b);
  plan->twTA = twTA_off >= 0 ? twT_dev + twTA_off : nullptr;
  plan->twTB = twTB_off >= 0 ? twT_dev + twTB_off : nullptr;
  plan->twTB2 = twTB2_off >= 0 ? twT_dev + twTB2_off : nullptr;
  plan->downP = downP_off >= 0 ? twT_dev + downP_off : nullptr;
  b += al(b_twT);
  plan->spec_fix = reinterpret_cast<unsigned int*>(b);
  hipError_t e = hipMemcpy(plan->tw, tw.data(), b_tw, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->down, down.data(), b_down, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->down1, down1.data(), b_down1, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->win, win.data(), b_win, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->rev, rev.data(), b_rev, hipMemcpyHostToDevice);
  if (e == hipSuccess && !twT.empty()) e = hipMemcpy(twT_dev, twT.data(), b_twT, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(plan->spec_fix, 0, sizeof(unsigned int));
  hipSetDevice(prev);
  if (e != hipSuccess) {
    const std::string msg = std::string("plan setup: ") + hipGetErrorString(e);
    lora_demod_plan_destroy(plan);  // the tables
    return set_error(LORA_EIO, msg);
  }
  *out = plan;
  return LORA_OK;
}

int lora_demod_plan_set_pipeline(lora_demod_plan* plan, int speculative) {
  if (!plan || (speculative != 0 && speculative != 1)) return set_error(LORA_EINVAL, "bad argument");
  plan->spec = speculative;
  return LORA_OK;
}

int lora_demod_profile_enable(lora_demod_plan* plan, int max_calls) {
  if (!plan || max_calls < 0) return set_error(LORA_EINVAL, "bad argument");
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(plan->prm.device));
  for (auto& r : plan->prof_recs) {
    hipEventDestroy(r.b);
    hipEventDestroy(r.e);
  }
  for (hipEvent_t e : plan->prof_pool) hipEventDestroy(e);
  plan->prof_recs.clear();
  plan->prof_pool.assign((size_t)max_calls * 4 * 2, nullptr);  // up to four launches per call
  for (auto& e : plan->prof_pool) HIP_TRY(hipEventCreate(&e));
  plan->prof_max = max_calls;
  plan->prof_calls = 0;
  plan->prof_short = false;
  HIP_TRY(hipSetDevice(prev));
  return LORA_OK;
}

int lora_demod_profile_read(lora_demod_plan* plan, float* stage_ms, int* calls) {
  if (!plan || !stage_ms || !calls) return set_error(LORA_EINVAL, "bad argument");
  for (int k = 0; k < 3; ++k) stage_ms[k] = 0.0f;
  *calls = plan->prof_calls;
  if (plan->prof_short) return set_error(LORA_ERANGE, "profile event pool exhausted: stage times incomplete");
  for (auto& r : plan->prof_recs) {
    HIP_TRY(hipEventSynchronize(r.e));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, r.b, r.e));
    if (r.stage >= 0 && r.stage < 3) stage_ms[r.stage] += ms;
  }
  return LORA_OK;
}

int lora_demod_plan_destroy(lora_demod_plan* plan) {
  if (!plan) return LORA_OK;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(plan->prm.device);
  for (auto& r : plan->prof_recs) {
    hipEventDestroy(r.b);
    hipEventDestroy(r.e);
  }
  for (hipEvent_t e : plan->prof_pool) hipEventDestroy(e);
  hipFree(plan->dev_tables);
  hipSetDevice(prev);
  delete plan;
  return LORA_OK;
}

int64_t lora_demod_symbols_per_frame(const lora_demod_plan* plan, int64_t frame_len) {
  if (!plan || frame_len < 0) return set_error(LORA_EINVAL, "bad argument");
  const int64_t total = frame_len / plan->step;
  if (plan->prm.mode == LORA_MODE_API) {
    if (frame_len % plan->step != 0)  // phy.cpp:186
      return set_error(LORA_EINVAL, "API mode: frame_len must be a multiple of N*osr");
    if (total < 2) return set_error(LORA_EINVAL, "API mode: frame needs >= 2 symbols");  // phy.cpp:188
    return total - 2;
  }
  if (plan->prm.mode == LORA_MODE_RAW) return total;
  return total >= 2 ? total - 2 : total;  // LoRaDemod.cpp:194
}

size_t lora_demod_workspace_bytes(const lora_demod_plan* plan, int64_t frames, int64_t frame_len) {
  if (!plan || frames <= 0 || frame_len < 0) return 0;
  return ws_layout(frames, frame_len, plan->step, plan->N).total;
}

int64_t lora_demod_spec_recomputed(lora_demod_plan* plan) {
  if (!plan) return set_error(LORA_EINVAL, "null plan");
  unsigned int v = 0;
  HIP_TRY(hipMemcpy(&v, plan->spec_fix, sizeof(v), hipMemcpyDeviceToHost));
  return (int64_t)v;
}

int64_t lora_demod_batch(lora_demod_plan* plan, const float* iq, int64_t frames, int64_t frame_len,
                         int64_t frame_stride, const lora_demod_outputs* out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  if (!plan || !out) return set_error(LORA_EINVAL, "null argument");
  if (frames < 0 || frame_len < 0 || frame_stride < frame_len)
    return set_error(LORA_EINVAL, "bad frames / frame_len / frame_stride");
  if (frame_len >= (int64_t(1) << 31)) return set_error(LORA_EINVAL, "frame_len must be < 2^31");
  const int64_t nsym = lora_demod_symbols_per_frame(plan, frame_len);
  if (nsym < 0) return nsym;
  if (frames == 0) return nsym;
  if (!iq) return set_error(LORA_EINVAL, "null iq");
  if (out->symbols && out->sym_stride < nsym)
    return set_error(LORA_ERANGE, "sym_stride smaller than symbols per frame");  // phy.cpp:190
  const WsLayout wl = ws_layout(frames, frame_len, plan->step, plan->N);
  const size_t need = wl.total;
  if (!workspace || workspace_bytes < need)
    return set_error(LORA_ERANGE, "workspace too small");

  const lora_demod_params& p = plan->prm;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  if (prev != p.device) HIP_TRY(hipSetDevice(p.device));

  const int64_t total = frame_len / plan->step;
  KArgs a;
  a.iq = reinterpret_cast<const cf*>(iq);
  a.frame_len = frame_len;
  a.frame_stride = frame_stride;
  a.sf = (int)p.sf;
  a.N = plan->N;
  a.osr = (int)p.osr;
  a.step = plan->step;
  a.total = (int)total;
  a.mode = p.mode;
  a.have_sync = (p.mode == LORA_MODE_API) ? 1 : (p.mode == LORA_MODE_LEGACY && total >= 2 ? 1 : 0);
  a.dechirp = (p.mode != LORA_MODE_API && p.dechirp) ? 1 : 0;
  a.hann = p.window == LORA_WINDOW_HANN;
  a.power_scale = plan->power_scale;
  a.tw = plan->tw;
  a.rev = plan->rev;
  a.win = plan->win;
  a.down = plan->down;
  a.down1 = plan->down1;
  a.twTA = plan->twTA;
  a.twTB = plan->twTB;
  a.twTB2 = plan->twTB2;
  a.downP = plan->downP;
  unsigned char* wsb = static_cast<unsigned char*>(workspace);
  uint32_t* maxbits = reinterpret_cast<uint32_t*>(wsb);
  a.maxbits = maxbits;
  a.fp = reinterpret_cast<lora::FrameParams*>(wsb + wl.fp);
  a.fp_spec = reinterpret_cast<lora::FrameParams*>(wsb + wl.fp_spec);
  a.spec_marg = reinterpret_cast<float*>(wsb + wl.marg);
  a.spec_max = maxbits;
  a.spec_fix = plan->spec_fix;
  a.fix_count = reinterpret_cast<unsigned int*>(wsb + wl.fix);
  a.fix_list = reinterpret_cast<uint32_t*>(wsb + wl.fix + 64 * lora::kFixStripes);
  a.fix_cap = wl.fix_cap;
  a.syms = out->symbols;
  a.sym_stride = out->sym_stride;
  a.sync = out->sync;
  a.cfo = out->cfo;
  a.toff = out->time_offset;
  a.max_amp = out->max_amp;
  a.est_only = 0;
  a.fast_rot = (p.precision == LORA_PRECISION_FAST && p.mode != LORA_MODE_RAW) ? 1 : 0;

  const int s0 = a.have_sync ? 2 : 0;
  const int64_t per = total - s0;
  // k_frame_max: frames shorter than two batches take one wave each (k_frame_max_wave)
  const int bpf = frame_max_blocks(frame_len);
  const bool max_wave = bpf == 1;
  a.mx_bpf = (p.mode == LORA_MODE_LEGACY && frame_len > 0) ? bpf : 0;
  // split evenly over the frame's blocks
  const int chunk = (int)((((frame_len + bpf - 1) / bpf) + 1) & ~int64_t(1));
  if (frames * bpf >= (int64_t(1) << 31)) {
    if (prev != p.device) hipSetDevice(prev);
    return set_error(LORA_EINVAL, "batch too large");
  }
  int kernels = 0;
  int rc = LORA_OK;
  if (p.mode == LORA_MODE_RAW && lora::t_launch_record) lora::t_launch_record->bad = true;
  if (p.mode == LORA_MODE_RAW) {
    // detector only: per-frame outputs are defined as 0
    hipError_t e = hipSuccess;
    if (a.sync) e = hipMemsetAsync(a.sync, 0, (size_t)frames, st);
    if (a.cfo && e == hipSuccess) e = hipMemsetAsync(a.cfo, 0, sizeof(float) * (size_t)frames, st);
    if (a.toff && e == hipSuccess) e = hipMemsetAsync(a.toff, 0, sizeof(float) * (size_t)frames, st);
    if (a.max_amp && e == hipSuccess) e = hipMemsetAsync(a.max_amp, 0, sizeof(float) * (size_t)frames, st);
    if (e != hipSuccess) rc = set_error(LORA_EIO, "hipMemsetAsync failed");
  }
  // Speculative single-read pipeline (LoRaDemod.cpp:59-192 reordered, results identical;
  // LEGACY frames at osr 1-4, either window; API frames at osr 1, below):
  //   1. offset estimate on UNSCALED samples (k_est_split / k_est_fast<SPEC=1>), plus the
  //      maximum of the samples outside the data-symbol windows it implies;
  //   2. every symbol with those offsets on unscaled samples (k_spec_demod), which also
  //      reduces each data window's max(|I|,|Q|) - the frame-max pass's work, from the same
  //      read - and records each symbol's argmax margin;
  //   3. the exact estimate from the assembled maximum (k_est_fast<SPEC=2>; SF 6-9
  //      k_cert_split): outputs, and each speculative symbol - sync symbols included -
  //      either certified (its margin exceeds the rounding bound, so the reference's argmax
  //      is the same bin) or listed;
  //   4. the listed symbols and sync words recomputed exactly (k_spec_fix).
  // The IQ is read once plus symbols 0/1 twice; lora_demod_spec_recomputed() counts
  // recomputations.  The symbol demod rotates with the hardware sine/cosine under either
  // precision; the certification holds it to the EXACT reference.  A sync block of
  // k_spec_demod spans 512/N frames (N < 1024): their byte offsets must fit 31 bits.
  const int64_t sync_frames = plan->N < 1024 ? 512 / plan->N : 1;
  // Oversampled frames (osr 2-4) take it too: the symbol pass reads every sample of each
  // window (the frame maximum) and transforms every osr-th one; its buffer offsets need the
  // frame's bytes below 2^31.
  // LORA_MODE_API frames at osr 1 take it too (phy.cpp:178-239): no normalisation, so the
  // exact estimate runs first and the symbol pass speculates only on the rotation (the
  // hardware sine/cosine and fused multiply-adds), certified with no rate difference.
  const bool api = p.mode == LORA_MODE_API;
  const bool spec_ok = plan->spec && (p.mode == LORA_MODE_LEGACY || (api && p.osr == 1)) && p.osr >= 1 &&
                       p.osr <= 4 && p.sf >= 6 && total >= 3 && total - 2 <= lora::kSpecChunks * (plan->N / 16) &&
                       sync_frames * frame_stride * 8 < (int64_t(1) << 31) && frame_len * 8 < (int64_t(1) << 31);
  // LORA_MODE_RAW at osr 1, SF 6-9 (the detector alone, awgn_sweep.py:262-273): every symbol through
  // the symbol pass with no offsets and no rotation, certified against the transforms'
  // rounding alone (k_cert_raw) or recomputed exactly (k_spec_fix)
  const bool spec_raw = plan->spec && p.mode == LORA_MODE_RAW && p.osr == 1 && p.sf >= 6 && p.sf <= 9 && total >= 1 &&
                        total <= lora::kSpecChunks * (plan->N / 16) && frame_len * 8 < (int64_t(1) << 31);
  if (rc == LORA_OK && spec_raw) {
    KArgs as = a;
    hipError_t e = hipMemsetAsync(a.fp, 0, sizeof(lora::FrameParams) * (size_t)frames, st);  // no offsets
    bool ok = e == hipSuccess;
    if (ok) {
      ProfScope ps(plan, 2, st);
      ok = lora::launch_spec(as, frames, 1, st);
    }
    if (ok) {
      ProfScope ps(plan, 1, st);
      ok = lora::launch_spec(as, frames, 2, st);
    }
    if (ok) {
      ProfScope ps(plan, 1, st);
      ok = lora::launch_spec(as, frames, 3, st);
    }
    if (!ok) rc = set_error(LORA_EIO, "RAW pipeline launch failed");
    kernels |= LORA_KERNEL_SPEC | LORA_KERNEL_DEMOD;
  } else if (rc == LORA_OK && spec_ok) {
    KArgs as = a;
    as.mx_bpf = 1;  // one slot per frame: the pre-pass's max outside the data windows
    if (api) {
      as.fp_spec = as.fp;  // the offsets the symbol pass uses are the exact ones
      as.dechirp = 1;      // each window times the down-chirp (table phase 0, k_spec_demod API)
    }
    bool ok;
    {
      ProfScope ps(plan, 1, st);
      ok = lora::launch_spec(as, frames, 0, st);
    }
    if (ok) {
      ProfScope ps(plan, 2, st);
      ok = lora::launch_spec(as, frames, 1, st);
    }
    if (ok) {
      ProfScope ps(plan, 1, st);
      ok = lora::launch_spec(as, frames, 2, st);
    }
    if (ok) {
      ProfScope ps(plan, 1, st);
      ok = lora::launch_spec(as, frames, 3, st);
    }
    if (!ok) rc = set_error(LORA_EIO, "speculative pipeline launch failed");
    kernels |= LORA_KERNEL_SPEC | LORA_KERNEL_ESTIMATE | LORA_KERNEL_DEMOD;
  } else if (rc == LORA_OK) {
    // three launches: (LEGACY) frame max, estimate + sync symbols, symbol demod
    if (p.mode == LORA_MODE_LEGACY && frame_len > 0) {
      kernels |= LORA_KERNEL_FRAME_MAX | (max_wave ? LORA_KERNEL_FRAME_MAX_WAVE : 0);
      ProfScope ps(plan, 0, st);
      if (max_wave)
        lora::launch(k_frame_max_wave, dim3((unsigned)((frames + 3) / 4)), dim3(256), 0, st, a, frames,
                           maxbits);
      else
        lora::launch(k_frame_max, dim3((unsigned)(frames * bpf)), dim3(256), 0, st, a, bpf, chunk, maxbits);
    }
    if (p.mode != LORA_MODE_RAW) {
      ProfScope ps(plan, 1, st);
      kernels |= LORA_KERNEL_ESTIMATE;
      if (!lora::launch_est_fast(a, frames, st)) {
        kernels |= LORA_KERNEL_GENERIC;
        lora::launch(k_estimate, dim3((unsigned)frames), dim3(256), sizeof(cf) * plan->N, st, a);
      }
    }
    const int64_t work = frames * per;
    if (work > 0) {
      ProfScope ps(plan, 2, st);
      kernels |= LORA_KERNEL_DEMOD;
      if (!lora::launch_demod_fast(a, s0, work, st)) rc = set_error(LORA_EIO, "symbol demod launch failed");
    }
  }
  if (plan->prof_calls < plan->prof_max) ++plan->prof_calls;
  plan->last_kernels = kernels;
  if (rc == LORA_OK) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) rc = set_error(LORA_EIO, std::string("kernel launch: ") + hipGetErrorString(e));
  }
  if (prev != p.device) hipSetDevice(prev);
  return rc < 0 ? rc : nsym;
}

namespace {
// The run tables of k_mod_runs per (device, sf, osr, bandwidth), kept for the process's
// lifetime: chirp values below max(N, 256) (symbols, sync nibbles, lora_encode's 8-bit
// codewords); a larger value's chirp is derived in the frame kernel itself.  SF12 osr 1:
// 4,096 x 92 runs x 16 B = 6 MB.
struct ModRunTable {
  int device, sf, osr;
  float bw_scale;
  int n, cap;
  lora::ChirpSeg* seg;
  int* cnt;
};
std::mutex g_mrt_mu;
std::vector<ModRunTable> g_mrt;

// fills a.seg / cnt / seg_n / seg_cap; false (g_last_error set) if the tables could not be made
bool mod_run_table(ModArgs& a, int sf, hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(LORA_EIO, "hipGetDevice"), false;
  std::lock_guard<std::mutex> lk(g_mrt_mu);
  for (const ModRunTable& t : g_mrt)
    if (t.device == dev && t.sf == sf && t.osr == a.osr && t.bw_scale == a.bw_scale) {
      a.seg = t.seg;
      a.cnt = t.cnt;
      a.seg_n = t.n;
      a.seg_cap = t.cap;
      return true;
    }
  ModRunTable t{dev, sf, a.osr, a.bw_scale, std::max(a.N, 256), lora::chirp_seg_cap(sf), nullptr, nullptr};
  if (hipMalloc(&t.seg, sizeof(lora::ChirpSeg) * (size_t)t.n * t.cap) != hipSuccess ||
      hipMalloc(&t.cnt, sizeof(int) * (size_t)t.n) != hipSuccess) {
    if (t.seg) hipFree(t.seg);
    return set_error(LORA_EIO, "hipMalloc"), false;
  }
  // Built and waited for here, once, always through HIP - also while the C++ drop-in records
  // launches for its AQL queue (then on the null stream): an entry enters g_mrt only once its
  // tables are complete, so no caller (another thread's lora_mod_batch, or this one after the
  // queue refused its record) can find a table that was never filled.
  hipStream_t bst = lora::t_launch_record ? nullptr : st;
  hipLaunchKernelGGL(k_mod_runs, dim3((unsigned)((t.n + 63) / 64)), dim3(64), 0, bst, a, t.n, t.cap, t.seg, t.cnt);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(bst) != hipSuccess) {
    hipFree(t.seg);
    hipFree(t.cnt);
    return set_error(LORA_EIO, "k_mod_runs"), false;
  }
  g_mrt.push_back(t);
  a.seg = t.seg;
  a.cnt = t.cnt;
  a.seg_n = t.n;
  a.seg_cap = t.cap;
  return true;
}
}  // namespace

int64_t lora_mod_batch(unsigned sf, unsigned osr, unsigned bw_hz, float amplitude, uint8_t sync,
                       const uint16_t* symbols, int64_t frames, int64_t sym_count, float* iq,
                       int device, void* stream) {
  if (sf < 2 || sf > 12) return set_error(LORA_EINVAL, "sf must be in 2..12");
  if (osr == 0) osr = 1;
  if (!bw_ok(bw_hz)) return set_error(LORA_EINVAL, "bad bw_hz");
  if (frames < 0 || sym_count < 0) return set_error(LORA_EINVAL, "bad sizes");
  const int N = 1 << sf;
  const int step = N * (int)osr;
  const int64_t per_frame = (sym_count + 2) * (int64_t)step;
  if (frames == 0) return per_frame;
  if (!iq || (sym_count > 0 && !symbols)) return set_error(LORA_EINVAL, "null buffer");
  const float bws = bw_scale_of(bw_hz);
  ModArgs a;
  a.N = N;
  a.osr = (int)osr;
  a.step = step;
  a.nchirp = (int)(sym_count + 2);
  a.fMin = -M_PI * bws / osr;  // ChirpGenerator.hpp:107-109 (double -> float)
  a.fMax = M_PI * bws / osr;
  a.fStep = (2 * M_PI * bws) / (N * osr * osr);
  a.ampl = std::max(-1.0f, std::min(1.0f, amplitude));  // LoRaMod.cpp:16
  a.bw_scale = bws;
  const unsigned shift = sf > 4 ? sf - 4 : 0;
  a.sw0 = (uint16_t)((sync >> 4) << shift);
  a.sw1 = (uint16_t)((sync & 0x0f) << shift);
  a.syms = symbols;
  a.sym_count = sym_count;
  a.iq = reinterpret_cast<cf*>(iq);
  a.frames = frames;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  if (prev != device) HIP_TRY(hipSetDevice(device));
  // (lora::launch: recorded instead when the C++ drop-in dispatches on its AQL queue)
  // k_mod_phase: long chirps (the speculative blocks, step >= 1024) over about 1024 waves
  // (frames per wave a power of two <= 64: fewer lanes per wave, fewer redone blocks);
  // short ones 64 frames per wave (their chains are short: the lanes' issue count matters)
  a.fpw = step >= 1024 ? 1 : 64;
  while (a.fpw < 64 && (int64_t)a.fpw * 1024 < frames) a.fpw *= 2;
  a.seg = nullptr;
  a.cnt = nullptr;
  a.seg_n = a.seg_cap = 0;
  // k_mod_frame's windows hold whole chirps or an exact fraction of one (a window never
  // crosses a chirp boundary inside it), and with chirps of whole 32-sample blocks whole
  // blocks: osr values that break either (SF10 osr 5: 5,120-sample chirps, 1,706-sample
  // windows) take the bulk kernels
  const int W = step <= kMfWin ? step * (kMfWin / step) : step / ((step + kMfWin - 1) / kMfWin);
  const bool mf_ok = (step <= W ? W % step == 0 : step % W == 0) && (step % kMfBlk != 0 || W % kMfBlk == 0);
  if (frames <= kMfMaxFrames && mf_ok) {
    // few frames: a workgroup per frame, windows of whole chirps or exact chirp fractions;
    // long chirps from the configuration's run tables (built here on first use)
    if (step >= kMfTabMin && !mod_run_table(a, (int)sf, st)) {
      if (prev != device) hipSetDevice(prev);
      return set_error(LORA_EIO, "modulator run tables: " + g_last_error);
    }
    const int64_t nwin = (per_frame + W - 1) / W;
    lora::launch(k_mod_frame, dim3((unsigned)frames), dim3(kMfThreads), 0, st, a, W, (int)nwin);
  } else {
    lora::launch(k_mod_phase, dim3((unsigned)((frames + a.fpw - 1) / a.fpw)), dim3(64), 0, st, a);
    const int64_t chirps = frames * a.nchirp;
    const int64_t per_block = (int64_t)kModLanes * kModWaves;
    lora::launch(k_mod_samples, dim3((unsigned)((chirps + per_block - 1) / per_block)), dim3(per_block), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (prev != device) hipSetDevice(prev);
  if (e != hipSuccess) return set_error(LORA_EIO, std::string("mod launch: ") + hipGetErrorString(e));
  return per_frame;
}

int64_t lora_estimate_offsets_batch(lora_demod_plan* plan, const float* iq, int64_t frames,
                                    int64_t frame_len, int64_t frame_stride, float* cfo,
                                    float* time_offset, void* stream) {
  if (!plan) return set_error(LORA_EINVAL, "null plan");
  if (frames < 0 || frame_len < 0 || frame_stride < frame_len)
    return set_error(LORA_EINVAL, "bad frames / frame_len / frame_stride");
  if (frame_len >= (int64_t(1) << 31)) return set_error(LORA_EINVAL, "frame_len must be < 2^31");
  const int64_t total = frame_len / plan->step;
  if (frames == 0 || total == 0) return total;
  if (!iq) return set_error(LORA_EINVAL, "null iq");
  const lora_demod_params& p = plan->prm;
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  if (prev != p.device) HIP_TRY(hipSetDevice(p.device));
  KArgs a;
  std::memset(&a, 0, sizeof(a));
  a.iq = reinterpret_cast<const cf*>(iq);
  a.frame_len = frame_len;
  a.frame_stride = frame_stride;
  a.sf = (int)p.sf;
  a.N = plan->N;
  a.osr = (int)p.osr;
  a.step = plan->step;
  a.total = (int)total;
  a.mode = LORA_MODE_API;
  a.hann = p.window == LORA_WINDOW_HANN;
  a.power_scale = plan->power_scale;
  a.tw = plan->tw;
  a.rev = plan->rev;
  a.win = plan->win;
  a.down = plan->down;
  a.down1 = plan->down1;
  a.cfo = cfo;
  a.toff = time_offset;
  a.mx_bpf = 0;
  a.est_only = 1;
  hipLaunchKernelGGL(k_estimate, dim3((unsigned)frames), dim3(256), sizeof(cf) * plan->N,
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  if (prev != p.device) hipSetDevice(prev);
  if (e != hipSuccess) return set_error(LORA_EIO, std::string("estimate launch: ") + hipGetErrorString(e));
  return total;
}

int64_t lora_compensate_offsets_batch(unsigned sf, unsigned osr, const float* in, int64_t frames,
                                      int64_t frame_len, int64_t frame_stride, const float* cfo,
                                      const float* time_offset, int device, void* stream,
                                      float* out) {
  if (sf < 2 || sf > 12) return set_error(LORA_EINVAL, "sf must be in 2..12");
  if (osr == 0) osr = 1;
  if (frames < 0 || frame_len < 0 || frame_stride < frame_len)
    return set_error(LORA_EINVAL, "bad frames / frame_len / frame_stride");
  if (frames == 0 || frame_len == 0) return frame_len;
  if (!in || !out || !cfo || !time_offset) return set_error(LORA_EINVAL, "null buffer");
  if (in == out) return set_error(LORA_EINVAL, "in and out must not overlap");
  const float Nosr = static_cast<float>(1u << sf) * static_cast<float>(osr);  // phy.cpp:156
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  if (prev != device) HIP_TRY(hipSetDevice(device));
  const int64_t n = frames * frame_len;
  hipLaunchKernelGGL(k_compensate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<const cf*>(in),
                     reinterpret_cast<cf*>(out), frame_len, frame_stride, frames, Nosr, cfo,
                     time_offset);
  hipError_t e = hipGetLastError();
  if (prev != device) hipSetDevice(prev);
  if (e != hipSuccess) return set_error(LORA_EIO, std::string("compensate launch: ") + hipGetErrorString(e));
  return frame_len;
}

}  // extern "C"

