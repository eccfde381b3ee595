// lora_demod_fast.hip — per-symbol demodulator with a register-blocked FFT (gfx950).
//
// Geometry: each symbol (N = 2^SF points) is handled by T = N/16 lanes holding 16
// points each (SF <= 5: one lane holds the whole symbol).  A 256-thread workgroup
// handles SPW = 256/T symbols.  When T <= 64 every symbol lives inside one wave and
// the wave works alone (wave-local LDS rows, no workgroup barrier).
//   phase 0  slot table: (frame, symbol) of every slot, window base with the t_off
//            rule (LoRaDemod.cpp:142-149), rotation start phase (:151-152).
//   phase 1  coalesced 16-byte loads of each symbol window; LEGACY caller-side
//            dechirp (e2e_chain_test.cpp:88-93) and normalisation (LoRaDemod.cpp:
//            68-77) are applied here, once per sample, into an LDS row.
//   pass 1   each lane gathers its 16 points (stride T), applies the CFO rotation
//            with glibc-faithful sincosf (LoRaDemod.cpp:153-157) and the window, and
//            runs the innermost FFT stages (radix-2 for odd SF, then radix-4) in
//            registers.
//   pass A/B the remaining radix-4 stages in registers after LDS transposes.
//   argmax   over the lane's bins, then across the symbol's T lanes (lowest index
//            wins on ties, LoRaDetector.hpp:46-58), one uint16 store per symbol.
// Butterflies, twiddles and operation order are kissfft's (kissfft.hh:155-185), so
// every value is bit-identical to the reference; only the schedule differs.
#include "../../include/lora_mi355x.h"
#include "lora_internal.h"

#pragma clang fp contract(off)

namespace lora {
namespace {

template <int SF>
struct Geo {
  static constexpr int N = 1 << SF;
  static constexpr bool SMALL = SF <= 5;
  static constexpr int P = SMALL ? N : 16;                          // points per lane
  static constexpr int T = N / P;                                   // lanes per symbol
  static constexpr int R1 = SMALL ? N : ((SF & 1) ? 8 : 16);        // pass-1 span
  static constexpr int LOGR1 = SMALL ? SF : ((SF & 1) ? 3 : 4);
  static constexpr int G1 = P / R1;                                 // pass-1 groups/lane
  static constexpr bool R2FIRST = (SF & 1) != 0;                    // radix-2 innermost
  static constexpr int X = N / R1;                                  // span left after pass 1
  static constexpr int RA = X >= 16 ? 16 : X;                       // pass-A span
  static constexpr int RB = X > 16 ? X / 16 : 1;                    // pass-B span
  static constexpr int NPASS = 1 + (X > 1 ? 1 : 0) + (X > 16 ? 1 : 0);
  static constexpr int MA_A = R1;
  static constexpr int MA_B = R1 * RA;
  static constexpr int SPW = 256 / T;                               // symbols per workgroup
  static constexpr bool WAVE_LOCAL = T <= 64;
};

// kissfft leaf position of input v inside an R-point block (radices 4,..,4[,2]).
constexpr int leaf_pos(int R, int v) {
  int pos = 0, rem = R;
  while (rem > 1) {
    const int r = (rem % 4 == 0) ? 4 : 2;
    rem /= r;
    pos += (v % r) * rem;
    v /= r;
  }
  return pos;
}

// Padded LDS address of DIT position p: one spare complex per R1 block breaks the
// power-of-two stride of the pass-1 write-back (conflict-free ds_write_b64).
template <int LOGR1>
__device__ __forceinline__ int paddr(int p) {
  return p + (p >> LOGR1);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool WAVE_LOCAL>
__device__ __forceinline__ void block_sync() {
  if constexpr (WAVE_LOCAL)
    wave_sync();
  else
    __syncthreads();
}

// In-register DIT stages over x[0..R): positions base + MA*u, group offset k < MA.
// Radix-2 (optional, only with MA == 1) then radix-4 stages, as kf_work unwinds.
template <int R, bool R2, int N, int MA>
__device__ __forceinline__ void pass_regs(cf* x, int k, const cf* __restrict__ tw) {
  int S = 1;
  if constexpr (R2) {
    constexpr int fs = N / (2 * MA);
#pragma unroll
    for (int b = 0; b < R; b += 2) bfly2(x[b], x[b + 1], tw[k * fs]);
    S = 2;
  }
#pragma unroll
  for (; S < R; S *= 4) {
    const int fs = N / (4 * MA * S);
#pragma unroll
    for (int blk = 0; blk < R; blk += 4 * S) {
#pragma unroll
      for (int uu = 0; uu < S; ++uu) {
        const int kk = k + MA * uu;
        bfly4(x[blk + uu], x[blk + uu + S], x[blk + uu + 2 * S], x[blk + uu + 3 * S], tw[kk * fs],
              tw[2 * kk * fs], tw[3 * kk * fs]);
      }
    }
  }
}


// The other lanes' share of one pass: read R points from LDS, run the stages,
// either write them back or fold them into the argmax key.
template <int R, int N, int MA, int LOGR1, int T, int P, bool LAST>
__device__ __forceinline__ void pass_lds(cf* row, cf* x, int l, const cf* __restrict__ tw,
                                         uint64_t& key) {
  constexpr int NG = P / R;
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) {
    const int GI = l + T * gg;
    const int k = GI % MA, cc = GI / MA;
    cf* xs = x + gg * R;
#pragma unroll
    for (int u = 0; u < R; ++u) xs[u] = row[paddr<LOGR1>(cc * MA * R + k + MA * u)];
    pass_regs<R, false, N, MA>(xs, k, tw);
  }
  if constexpr (LAST) {
    // The last pass covers all N bins with cc == 0: bin = (l + T*gg) + MA*u.  Scanning
    // u-major / gg-minor visits the lane's bins in increasing order, so a strict '>'
    // keeps the lowest index among equal maxima (LoRaDetector.hpp:50-57).
    float best = 0.0f;
    uint32_t bi = (uint32_t)l;
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int gg = 0; gg < NG; ++gg) {
        const cf v = x[gg * R + u];
        const float m2 = v.re * v.re + v.im * v.im;
        const uint32_t bin = (uint32_t)(l + T * gg + MA * u);
        if (m2 > best) {
          best = m2;
          bi = bin;
        }
      }
    key = ((uint64_t)__float_as_uint(best) << 32) | (uint32_t)(~bi);
  }
}

template <int R, int MA, int LOGR1, int T, int P>
__device__ __forceinline__ void write_pass(cf* row, const cf* x, int l) {
  constexpr int NG = P / R;
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) {
    const int GI = l + T * gg;
    const int k = GI % MA, cc = GI / MA;
#pragma unroll
    for (int u = 0; u < R; ++u) row[paddr<LOGR1>(cc * MA * R + k + MA * u)] = x[gg * R + u];
  }
}

// MODE 0: LEGACY + fused dechirp, osr 1, no window (the benchmark configuration);
// MODE 1: LEGACY on already-dechirped input, osr 1, no window (lora_demodulate's own
//         contract); MODE 2: every other configuration, flags read at run time.
// ABL: profiling-only ablation mask (LORA_MI355X_ABLATE; results are NOT valid):
// 1 = identity rotation instead of sincosf, 2 = skip the pass-1 FFT stages, 4 = skip
// the HBM loads.
template <int SF, int MODE, int ABL = 0>
__global__ void __launch_bounds__(256) k_demod_fast(KArgs a, int s0, int64_t work, int rowc) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P, R1 = G::R1, SPW = G::SPW;
  constexpr bool WL = G::WAVE_LOCAL;
  constexpr bool DYN = MODE == 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cf* rows = reinterpret_cast<cf*>(smem);
  const int tid = threadIdx.x;
  const int per = a.total - s0;
  const int step = DYN ? a.step : N;
  const int osr = DYN ? a.osr : 1;
  const bool legacy = DYN ? a.mode != LORA_MODE_API : true;
  const bool dech = DYN ? (legacy && a.dechirp) : (MODE == 0);
  const bool hann = DYN ? (a.hann != 0) : false;

  // ---- symbol of this lane: window base with the t_off rule (LoRaDemod.cpp:142-149)
  // and rotation start phase (:151-152); every lane of the symbol computes it.
  const int g = tid / T;  // slot
  const int l = tid % T;  // lane within the symbol
  const int64_t w = (int64_t)blockIdx.x * SPW + g;
  const bool valid = w < work;
  const int64_t wc = valid ? w : work - 1;  // clamp: invalid lanes mirror a valid symbol
  const int64_t f = wc / per;
  const int s = s0 + (int)(wc - f * per);
  const FrameParams p = a.fp[f];
  int64_t base = (int64_t)s * step;
  int cg = 0;
  if (p.t_off > 0) {
    if (base + p.t_off + step <= a.frame_len) {
      base += p.t_off;
      cg = p.t_off;
    }
  } else if (p.t_off < 0) {
    const int64_t off = -(int64_t)p.t_off;
    if (off <= base) {
      base -= off;
      cg = step - (int)off;
    }
  }
  const cf* __restrict__ x = a.iq + f * a.frame_stride + base;
  const float start = p.rate * ((float)((uint32_t)s * (uint32_t)N) + (float)p.t_off / (float)osr);
  const float rate = p.rate;
  // LoRaDemod.cpp:68-77: scale is 1.0f when the frame is not rescaled (x*1.0f == x).
  const float scale = (legacy && p.scaled) ? p.scale : 1.0f;

  // ---- pass 1: gather 16 points (stride T), dechirp / scale / rotate / window ----
  cf in[P];
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const int i = l + T * q;
    if (ABL & 4)
      in[q] = cf{0.0f, 0.0f};
    else
      in[q] = x[(int64_t)i * osr];
  }
  if (!legacy) {
#pragma unroll
    for (int q = 0; q < P; ++q) in[q] = cmul(in[q], a.down1[l + T * q]);
  } else {
    if (dech) {
#pragma unroll
      for (int q = 0; q < P; ++q) {
        int d = cg + (l + T * q) * osr;
        if (d >= step) d -= step;
        in[q] = cmul(in[q], a.down[d]);
      }
    }
#pragma unroll
    for (int q = 0; q < P; ++q) in[q] = cscale(in[q], scale);
  }
  // The rotation phase is monotone in i, so the symbol's |ph| range is bounded by its
  // two end points; the branch-free sincosf covers |ph| < 120 (lora_libm.h).
  const bool sym_fast = lm_sincosf_fast_ok(start) && lm_sincosf_fast_ok(start + rate * (float)(N - 1));
  cf z[P];
  if (ABL & 1) {
#pragma unroll
    for (int q = 0; q < P; ++q) z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = in[q];
  } else if (__all(sym_fast)) {
    constexpr int K = 4;
#pragma unroll
    for (int q0 = 0; q0 < P; q0 += K) {
      float ph[K], sn[K], cs[K];
#pragma unroll
      for (int k = 0; k < K; ++k) ph[k] = start + rate * (float)(l + T * (q0 + k));
      lm_sincosf_fast_k<K>(ph, sn, cs);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int q = q0 + k;
        cf v = cmul(in[q], cf{cs[k], sn[k]});
        if (hann) v = cscale(v, a.win[l + T * q]);
        z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float ph = start + rate * (float)(l + T * q);
      float sn, cs;
      lm_sincosf(ph, &sn, &cs);
      cf v = cmul(in[q], cf{cs, sn});
      if (hann) v = cscale(v, a.win[l + T * q]);
      z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
    }
  }
  if (!(ABL & 2)) {
#pragma unroll
    for (int h = 0; h < G::G1; ++h) pass_regs<R1, G::R2FIRST, N, 1>(z + h * R1, 0, a.tw);
  }

  uint64_t key = 0;
  if constexpr (G::NPASS == 1) {
    float best = 0.0f;
    uint32_t bi = 0;
#pragma unroll
    for (int u = 0; u < R1; ++u) {
      const float m2 = z[u].re * z[u].re + z[u].im * z[u].im;
      if (m2 > best) {
        best = m2;
        bi = (uint32_t)u;
      }
    }
    key = ((uint64_t)__float_as_uint(best) << 32) | (uint32_t)(~bi);
  } else {
    cf* row = rows + (size_t)g * rowc;
    int c[G::G1];
#pragma unroll
    for (int h = 0; h < G::G1; ++h) c[h] = (int)(a.rev[l + T * h] >> G::LOGR1);
#pragma unroll
    for (int h = 0; h < G::G1; ++h)
#pragma unroll
      for (int u = 0; u < R1; ++u) row[paddr<G::LOGR1>(c[h] * R1 + u)] = z[h * R1 + u];
    block_sync<WL>();
    if constexpr (G::NPASS == 2) {
      pass_lds<G::RA, N, G::MA_A, G::LOGR1, T, P, true>(row, z, l, a.tw, key);
    } else {
      pass_lds<G::RA, N, G::MA_A, G::LOGR1, T, P, false>(row, z, l, a.tw, key);
      block_sync<WL>();
      write_pass<G::RA, G::MA_A, G::LOGR1, T, P>(row, z, l);
      block_sync<WL>();
      pass_lds<G::RB, N, G::MA_B, G::LOGR1, T, P, true>(row, z, l, a.tw, key);
    }
  }

  // ---- argmax across the T lanes of the symbol ----
  if constexpr (T <= 64) {
    key = group_max(key, T);
  } else {
    __shared__ uint64_t red[4];
    key = group_max(key, 64);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = key;
    __syncthreads();
    constexpr int WPS = T / 64;  // waves per symbol
    const int wb = ((tid >> 6) / WPS) * WPS;
    uint64_t r = red[wb];
#pragma unroll
    for (int q = 1; q < WPS; ++q) r = umax64(r, red[wb + q]);
    key = r;
  }
  if (l == 0 && valid && a.syms) a.syms[f * a.sym_stride + (s - s0)] = (uint16_t)key_index(key);
}

template <int SF, int MODE, int ABL = 0>
bool launch_mode(const KArgs& a, int s0, int64_t work, hipStream_t st) {
  using G = Geo<SF>;
  int rowc = G::N + (G::N >> G::LOGR1);                  // padded transpose image
  // rows 16-byte aligned and staggered by 16 banks (rowc = 8 mod 32 complex) so the
  // symbols of one wave hit different banks in the strided pass-1 gather
  while (rowc % 32 != 8) ++rowc;
  const size_t lds = G::NPASS == 1 ? 16 : sizeof(cf) * (size_t)G::SPW * rowc;
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_demod_fast<SF, MODE, ABL>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return false;
  const int64_t grid = (work + G::SPW - 1) / G::SPW;
  hipLaunchKernelGGL((k_demod_fast<SF, MODE, ABL>), dim3((unsigned)grid), dim3(256), lds, st, a, s0, work,
                     rowc);
  return true;
}

template <int SF>
bool launch_sf(const KArgs& a, int s0, int64_t work, hipStream_t st) {
  const bool simple = a.mode == LORA_MODE_LEGACY && a.osr == 1 && !a.hann;
  if constexpr (SF == 7 || SF == 12) {
    if (simple && a.dechirp && a.ablate) {
      switch (a.ablate) {
        case 1: return launch_mode<SF, 0, 1>(a, s0, work, st);
        case 2: return launch_mode<SF, 0, 2>(a, s0, work, st);
        case 3: return launch_mode<SF, 0, 3>(a, s0, work, st);
        case 4: return launch_mode<SF, 0, 4>(a, s0, work, st);
        case 7: return launch_mode<SF, 0, 7>(a, s0, work, st);
        default: break;
      }
    }
  }
  if (simple && a.dechirp) return launch_mode<SF, 0>(a, s0, work, st);
  if (simple) return launch_mode<SF, 1>(a, s0, work, st);
  return launch_mode<SF, 2>(a, s0, work, st);
}

}  // namespace

bool launch_demod_fast(const KArgs& a, int s0, int64_t work, hipStream_t st) {
  switch (a.sf) {
    case 2: return launch_sf<2>(a, s0, work, st);
    case 3: return launch_sf<3>(a, s0, work, st);
    case 4: return launch_sf<4>(a, s0, work, st);
    case 5: return launch_sf<5>(a, s0, work, st);
    case 6: return launch_sf<6>(a, s0, work, st);
    case 7: return launch_sf<7>(a, s0, work, st);
    case 8: return launch_sf<8>(a, s0, work, st);
    case 9: return launch_sf<9>(a, s0, work, st);
    case 10: return launch_sf<10>(a, s0, work, st);
    case 11: return launch_sf<11>(a, s0, work, st);
    case 12: return launch_sf<12>(a, s0, work, st);
    default: return false;
  }
}

}  // namespace lora
