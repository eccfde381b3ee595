// lora_demod_fast.hip — per-symbol demodulator with a register-blocked FFT (gfx950).
//
// Geometry: each symbol (N = 2^SF points) is handled by T = N/16 lanes holding 16
// points each (SF <= 5: one lane holds the whole symbol).  A 256-thread workgroup
// handles SPW = 256/T symbols.  When T <= 64 every symbol lives inside one wave and
// the wave works alone (wave-local LDS rows, no workgroup barrier).
//   gather   each lane loads its 16 points (stride T) straight from HBM (coalesced 8-B
//            lanes, compile-time offsets from one base pointer), applies the LEGACY
//            caller-side dechirp (e2e_chain_test.cpp:88-93, doubled table: no wrap) and
//            the normalisation (LoRaDemod.cpp:68-77), the window base following the
//            t_off rule (LoRaDemod.cpp:142-149).
//   pass 1   CFO rotation with glibc-faithful sincosf (LoRaDemod.cpp:151-157), window,
//            and the innermost FFT stages (radix-2 for odd SF, then radix-4) in
//            registers.
//   pass A/B the remaining radix-4 stages in registers after LDS transposes.
//   argmax   over the lane's bins, then across the symbol's T lanes (lowest index
//            wins on ties, LoRaDetector.hpp:46-58), one uint16 store per symbol.
// Butterflies, twiddles and operation order are kissfft's (kissfft.hh:155-185), so
// every value is bit-identical to the reference; only the schedule differs.
#include "../../include/lora_mi355x.h"
#include "lora_internal.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#pragma clang fp contract(off)

namespace lora {
namespace {

// Packed fp32 (v_pk_*_f32) only where it is written explicitly: the certified path's complex
// products and butterflies (lora_device.h).  The Makefile turns the compiler's own
// vectorisers off for this translation unit: its SLP-packed pairs cost operand-pairing moves
// (measured in round 1: SF7 demod -7 %, SF12 -13 % without them).  The same IEEE operations
// either way, so exact results are unchanged.

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

static_assert(pass_shape(7).RA == Geo<7>::RA && pass_shape(7).MA_A == Geo<7>::MA_A &&
                  pass_shape(12).RB == Geo<12>::RB && pass_shape(12).MA_B == Geo<12>::MA_B &&
                  pass_shape(9).RB == Geo<9>::RB && pass_shape(10).MA_B == Geo<10>::MA_B &&
                  pass_shape(6).RA == Geo<6>::RA && pass_shape(11).MA_B == Geo<11>::MA_B,
              "host pass_shape must match the kernels' Geo");

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

// LDS image of DIT position p: slot(p) = p + bit_3(p) * W3 + sum_{i>=0} bit_{4+i}(p) * W[i].
// The weights (and the row pad) were searched with tools/lds/lds_search_add.py against the
// MI355X banking rules (ds_read_b64: 2 x 32 lanes, 64 banks; ds_write_b64: 4 x 16
// lanes, 32 banks) over every access of the transform - pass-1 write-back, LDS-pass
// reads and write-backs, natural-order write: mean conflict degree 1.0-1.4 (the
// former p + p/R1 map reached 2-5.5, 16-way on the SF11/12 pass-1 write-back).  The
// search keeps every weight >= the sum of the lower ones (injective, asserted below).
// W3 (bit 3, default 0): SF7's pass-1 write-back puts a lane's two 8-position blocks
// (positions c 8 + u, c = rev[l] >> 3) 8 slots apart, which no map over bits >= 4 can
// separate from the neighbouring symbol's row (rowc = 8 mod 16, what the pass-A reads
// need): 2-way on every write (SQ_LDS_BANK_CONFLICT 1.9 per LDS instruction of the SF7
// symbol pass).  W3 = 1 with W = {1, 2, 4} (tools/lds/lds_search_bit3.py) is conflict-free
// on the write-back, the pass-A reads (ds_read_b64 and ds_read2_b64) and the
// natural-order write, at the same row length.
// Being linear in the bits of p, slot(base | off) = slot(base) + slot(off) when base and
// off use disjoint bits: every access splits into a per-lane part and a compile-time
// part that folds into the ds_* immediate offset.
template <int SF>
struct LdsMap;
template <> struct LdsMap<6> { static constexpr int W[2] = {1, 2}; static constexpr int PAD = 1; };
template <> struct LdsMap<7> {
  static constexpr int W3 = 1;
  static constexpr int W[3] = {1, 2, 4};
  static constexpr int PAD = 0;
};
template <> struct LdsMap<8> { static constexpr int W[4] = {1, 2, 4, 8}; static constexpr int PAD = 1; };
template <> struct LdsMap<9> { static constexpr int W[5] = {0, 1, 4, 8, 14}; static constexpr int PAD = 0; };
template <> struct LdsMap<10> { static constexpr int W[6] = {0, 0, 1, 2, 4, 8}; static constexpr int PAD = 0; };
template <> struct LdsMap<11> { static constexpr int W[7] = {0, 0, 2, 8, 10, 20, 43}; static constexpr int PAD = 0; };
template <> struct LdsMap<12> { static constexpr int W[8] = {0, 0, 0, 0, 1, 2, 4, 8}; static constexpr int PAD = 0; };

// bit 3's weight: LdsMap<SF>::W3 where declared, else 0
template <int SF, class = void>
struct LdsW3 {
  static constexpr int v = 0;
};
template <int SF>
struct LdsW3<SF, std::void_t<decltype(LdsMap<SF>::W3)>> {
  static constexpr int v = LdsMap<SF>::W3;
};

// Injectivity: each weight (W3 the lowest) is at least the sum of the lower ones, so
// slot(p) is strictly increasing in p and blocks never overlap.
template <int SF>
constexpr bool lds_map_injective() {
  int acc = LdsW3<SF>::v;
  for (int i = 0; i < SF - 4; ++i) {
    if (LdsMap<SF>::W[i] < acc) return false;
    acc += LdsMap<SF>::W[i];
  }
  return true;
}
static_assert(lds_map_injective<6>() && lds_map_injective<7>() && lds_map_injective<8>() &&
                  lds_map_injective<9>() && lds_map_injective<10>() && lds_map_injective<11>() &&
                  lds_map_injective<12>(),
              "LDS slot map must be injective");

template <int SF>
__host__ __device__ constexpr int lds_slot(int p) {
  if constexpr (SF <= 5) {
    return p;
  } else {
    int s = p + ((p >> 3) & 1) * LdsW3<SF>::v;
    for (int i = 0; i < SF - 4; ++i) s += ((p >> (4 + i)) & 1) * LdsMap<SF>::W[i];
    return s;
  }
}

template <int SF>
constexpr int lds_row() {  // complex elements per symbol row
  if constexpr (SF <= 5) {
    return 1 << SF;
  } else {
    int w = LdsW3<SF>::v;
    for (int i = 0; i < SF - 4; ++i) w += LdsMap<SF>::W[i];
    return (1 << SF) + w + LdsMap<SF>::PAD;
  }
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

// Speculative demod argmax keys: |X|^2's bits with the low 4 mantissa bits replaced by the
// bin's ordinal within the lane.  Non-negative floats order like their bits, so the key
// order is |X|^2's up to a truncation of < 16 ulp (relative 2^-19, carried by the
// certification bound); two bins within it are never certified (their keys' values tie).
__device__ __forceinline__ uint32_t spec_key(float m2, int ordinal) {
  return (__float_as_uint(m2) & 0xFFFFFFF0u) | (uint32_t)ordinal;
}
__device__ __forceinline__ float spec_key_value(uint32_t k) { return __uint_as_float(k & 0xFFFFFFF0u); }
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_max3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// In-register DIT stages over x[0..R): positions base + MA*u, group offset k < MA.
// Radix-2 (optional, only with MA == 1) then radix-4 stages, as kf_work unwinds.
// UNIT (argmax-only transforms with k == 0): the butterflies whose twiddles are all
// tw[0] = (1, 0) skip the multiplies.  x*(1,0) = (a*1 - b*0, a*0 + b*1) equals x except
// for the sign of a zero component, and a zero's sign never reaches a non-zero result
// or |X|^2, so every bin magnitude - hence the argmax - is bit-identical.  Transforms
// whose bin values are used (the estimate's phase) keep the multiplies.
// SKIP1: the first stage (the radix-2 one, or the first radix-4 one) was already done by the
// caller (the certified symbol pass folds its rotation factors into it, fft_key FOLD).
template <int R, bool R2, int N, int MA, bool UNIT = false, bool FMA = false, class TWP = const cf*,
          bool SKIP1 = false>
__device__ __forceinline__ void pass_regs(cf* x, int k, TWP tw) {
  int S = 1;
  if constexpr (SKIP1) {
    S = R2 ? 2 : 4;
  } else if constexpr (R2) {
    constexpr int fs = N / (2 * MA);
#pragma unroll
    for (int b = 0; b < R; b += 2) {
      if (UNIT)
        bfly2_unit<FMA>(x[b], x[b + 1]);
      else
        bfly2<FMA>(x[b], x[b + 1], tw[k * fs]);
    }
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
        if (UNIT && uu == 0)
          bfly4_unit<FMA>(x[blk], x[blk + S], x[blk + 2 * S], x[blk + 3 * S]);
        else
          bfly4<FMA>(x[blk + uu], x[blk + uu + S], x[blk + uu + 2 * S], x[blk + uu + 3 * S], tw[kk * fs],
                tw[2 * kk * fs], tw[3 * kk * fs]);
      }
    }
  }
}


// pass_regs<16, false, N, MA> with the twiddles read from the slot-major copy
// twT[j*MA + k] (lora::twT_index): the same butterflies, operands and order.
template <int R, int MA, bool FMA = false>
__device__ __forceinline__ void pass_regs_T(cf* x, int k, const cf* __restrict__ twT) {
  static_assert(R == 4 || R == 16, "radix-4 / radix-16 passes");
#pragma unroll
  for (int blk = 0; blk < R; blk += 4)
    bfly4<FMA>(x[blk], x[blk + 1], x[blk + 2], x[blk + 3], twT[0 * MA + k], twT[1 * MA + k], twT[2 * MA + k]);
  if constexpr (R == 16) {
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
      bfly4<FMA>(x[uu], x[uu + 4], x[uu + 8], x[uu + 12], twT[(3 + 3 * uu) * MA + k], twT[(4 + 3 * uu) * MA + k],
            twT[(5 + 3 * uu) * MA + k]);
  }
}

// pass_regs_T with the twiddles in slot pairs (KArgs::twTB2): one 16-byte load per two.
template <int R, int MA>
__device__ __forceinline__ void load_tw2(cf* w, int k, const cf* __restrict__ twT2) {
  static_assert(R == 4 || R == 16, "radix-4 / radix-16 passes");
  constexpr int NT = R == 16 ? 15 : 3;
  const float4* __restrict__ p4 = reinterpret_cast<const float4*>(twT2);
#pragma unroll
  for (int pp = 0; pp < NT / 2; ++pp) {
    const float4 v = p4[pp * MA + k];
    w[2 * pp] = cf{v.x, v.y};
    w[2 * pp + 1] = cf{v.z, v.w};
  }
  w[NT - 1] = twT2[(NT / 2) * MA * 2 + k];
}
template <int R, bool FMA>
__device__ __forceinline__ void pass_regs_w(cf* x, const cf* w) {
#pragma unroll
  for (int blk = 0; blk < R; blk += 4) bfly4<FMA>(x[blk], x[blk + 1], x[blk + 2], x[blk + 3], w[0], w[1], w[2]);
  if constexpr (R == 16) {
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
      bfly4<FMA>(x[uu], x[uu + 4], x[uu + 8], x[uu + 12], w[3 + 3 * uu], w[4 + 3 * uu], w[5 + 3 * uu]);
  }
}
template <int R, int MA, bool FMA = false>
__device__ __forceinline__ void pass_regs_T2(cf* x, int k, const cf* __restrict__ twT2) {
  cf w[R == 16 ? 15 : 3];
  load_tw2<R, MA>(w, k, twT2);
  pass_regs_w<R, FMA>(x, w);
}

// fft_key's hook between pass B's twiddle loads and its LDS reads (the prefetching symbol
// pass requests the next block's samples there: vmcnt retires in order, so the transform's
// own loads are all issued before them)
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// The other lanes' share of one pass: read R points from LDS, run the stages,
// either write them back or fold them into the argmax key.
// TSET: twT is known to be non-null (the speculative demod's plans always carry the
// slot-major copies), so no fallback path is compiled.
// PACK (speculative demod, LAST): instead of the 64-bit argmax key and a float runner-up,
// the lane's best and runner-up as 32-bit keys whose high 28 bits are those of |X|^2 and
// whose low 4 bits hold the bin's ordinal within the lane (spec_key); `key` returns
// best | (uint64_t)second << 32.
template <int R, int N, int MA, int SF, int T, int P, bool LAST, bool FMA = false, bool PAIR = false,
          bool TSET = false, bool PACK = false>
__device__ __forceinline__ void pass_lds(cf* row, cf* x, int l, const cf* __restrict__ tw,
                                         uint64_t& key, const cf* __restrict__ twT = nullptr,
                                         float* second = nullptr, const cf* wpre = nullptr) {
  constexpr int NG = P / R;
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) {
    const int GI = l + T * gg;
    const int k = GI % MA, cc = GI / MA;
    cf* xs = x + gg * R;
    const cf* rb = row + lds_slot<SF>(cc * MA * R + k);  // k < MA, MA*u: disjoint bits
#pragma unroll
    for (int u = 0; u < R; ++u) xs[u] = rb[lds_slot<SF>(MA * u)];
    if (wpre) {  // the group's twiddles, loaded by the caller (pass_regs_T2's values)
      if constexpr (R == 4 || R == 16) {
        pass_regs_w<R, FMA>(xs, wpre + gg * (R == 16 ? 15 : 3));
        continue;
      }
    }
    if constexpr (R == 4 || R == 16) {
      if (TSET || twT) {
        if constexpr (PAIR)
          pass_regs_T2<R, MA, FMA>(xs, k, twT);
        else
          pass_regs_T<R, MA, FMA>(xs, k, twT);
        continue;
      }
    }
    pass_regs<R, false, N, MA, false, FMA>(xs, k, tw);
  }
  if constexpr (LAST && PACK) {
    static_assert(NG * R == 16, "16 bins per lane: a 4-bit ordinal");
    // keys two at a time: with sec <= best, the runner-up of {best, sec, k1, k2} is
    // max(sec, med3(best, k1, k2)) and the best max3(best, k1, k2) - the same two keys as
    // one med3 + max per key (a lane's 16 keys are distinct: their ordinals differ)
    uint32_t best = 0, sec = 0;
    uint32_t kk[16];
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int gg = 0; gg < NG; ++gg) {
        const cf v = x[gg * R + u];
        const float m2 = __builtin_fmaf(v.re, v.re, v.im * v.im);
        kk[u * NG + gg] = spec_key(m2, u * NG + gg);
      }
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const uint32_t m = umed3(best, kk[i], kk[i + 1]);
      sec = sec > m ? sec : m;
      best = umax3(best, kk[i], kk[i + 1]);
    }
    key = (uint64_t)best | ((uint64_t)sec << 32);
  } else if constexpr (LAST) {
    // The last pass covers all N bins with cc == 0: bin = (l + T*gg) + MA*u.  Scanning
    // u-major / gg-minor visits the lane's bins in increasing order, so a strict '>'
    // keeps the lowest index among equal maxima (LoRaDetector.hpp:50-57).
    float best = 0.0f, sec = 0.0f;
    uint32_t bi = (uint32_t)l;
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int gg = 0; gg < NG; ++gg) {
        const cf v = x[gg * R + u];
        // FMA (certified demod): |X|^2 with one rounding fewer, inside the bound's E
        const float m2 = FMA ? __builtin_fmaf(v.re, v.re, v.im * v.im) : v.re * v.re + v.im * v.im;
        const uint32_t bin = (uint32_t)(l + T * gg + MA * u);
        // runner-up |X|^2 of the lane (an equal value counts: margin 0); sec <= best, so
        // the median of (sec, m2, best) is best if m2 > best, else max(sec, m2)
        if (second) sec = __builtin_amdgcn_fmed3f(sec, m2, best);
        if (m2 > best) {
          best = m2;
          bi = bin;
        }
      }
    key = ((uint64_t)__float_as_uint(best) << 32) | (uint32_t)(~bi);
    if (second) *second = sec;
  }
}

template <int R, int MA, int SF, int T, int P>
__device__ __forceinline__ void write_pass(cf* row, const cf* x, int l) {
  constexpr int NG = P / R;
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) {
    const int GI = l + T * gg;
    const int k = GI % MA, cc = GI / MA;
    cf* rb = row + lds_slot<SF>(cc * MA * R + k);
#pragma unroll
    for (int u = 0; u < R; ++u) rb[lds_slot<SF>(MA * u)] = x[gg * R + u];
  }
}

// ---- shared building blocks of the demod and estimate kernels --------------------

// Window base of symbol s with the t_off rule (LoRaDemod.cpp:142-149): `base` is the
// sample offset in the frame, `cg` the phase of the caller-side dechirp table there.
__device__ __forceinline__ void sym_base(int s, int step, int64_t frame_len, int t_off,
                                         int64_t& base, int& cg) {
  base = (int64_t)s * step;
  cg = 0;
  if (t_off > 0) {
    if (base + t_off + step <= frame_len) {
      base += t_off;
      cg = t_off;
    }
  } else if (t_off < 0) {
    const int64_t off = -(int64_t)t_off;
    if (off <= base) {
      base -= off;
      cg = step - (int)off;
    }
  }
}

// Gather the lane's P points x[(l + T*q)*osr] of one symbol window straight from HBM
// and apply what precedes the rotation: KIND 0 raw (API estimate, phy.cpp:91-99),
// KIND 1 LEGACY (caller dechirp, e2e_chain_test.cpp:88-93, then normalisation,
// LoRaDemod.cpp:68-77), KIND 2 API down-chirp (phy.cpp:216-225).
template <int SF, bool PAIRD = false>
__device__ __forceinline__ void gather_points(const KArgs& a, const cf* __restrict__ x, int l,
                                              int osr, int step, int cg, int kind, bool dech,
                                              float scale, cf* in) {
  using G = Geo<SF>;
  constexpr int T = G::T, P = G::P;
  if constexpr (PAIRD && P == 16) {
    // speculative demod, LEGACY osr 1 with the fused dechirp: the table values two per
    // 16-byte load from KArgs::downP (same values, same products)
    const cf* __restrict__ xl = x + l;
    // each sample is read once: nontemporal loads leave the caches to the tables
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f* __restrict__ xl2 = reinterpret_cast<const v2f*>(xl);
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const v2f v = __builtin_nontemporal_load(xl2 + T * q);
      in[q] = cf{v.x, v.y};
    }
    const float4* __restrict__ dp = reinterpret_cast<const float4*>(a.downP) + cg + l;
#pragma unroll
    for (int pp = 0; pp < P / 2; ++pp) {
      const float4 d = dp[pp * (G::N + T)];
      in[2 * pp] = cmul(in[2 * pp], cf{d.x, d.y});
      in[2 * pp + 1] = cmul(in[2 * pp + 1], cf{d.z, d.w});
    }
    return;
  }
  // One per-lane base pointer per stream; the points are then at compile-time offsets
  // T*q (times osr) from it, which fold into the loads' immediate offsets at osr 1.
  const cf* __restrict__ xl = x + (int64_t)l * osr;
#pragma unroll
  for (int q = 0; q < P; ++q) in[q] = xl[(int64_t)(T * q) * osr];
  if (kind == 2) {
    const cf* __restrict__ dl = a.down1 + l;
#pragma unroll
    for (int q = 0; q < P; ++q) in[q] = cmul(in[q], dl[T * q]);
  } else if (kind == 1) {
    if (dech) {
      // caller-side dechirp phase cg + i*osr < 2*step: the doubled table needs no wrap
      const cf* __restrict__ dl = a.down + cg + l * osr;
#pragma unroll
      for (int q = 0; q < P; ++q) in[q] = cmul(in[q], dl[(T * q) * osr]);
    }
#pragma unroll
    for (int q = 0; q < P; ++q) in[q] = cscale(in[q], scale);
  }
}

// CFO rotation (glibc-faithful sincosf, LoRaDemod.cpp:151-157) when ROT, window
// (:158-160), and placement in pass-1 leaf order.
// Speculative demod table access (A/B knobs): pass-A twiddles staged in LDS, pass-B
// twiddles in slot pairs (KArgs::twTB2).
template <int SF, bool ROT, bool FAST = false, bool FMA = false>
__device__ __forceinline__ void rotate_place(const cf* in, cf* z, float start, float rate,
                                             bool hann, const float* __restrict__ win, int l) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P, R1 = G::R1;
  if constexpr (FAST && ROT) {
    // LORA_PRECISION_FAST: the same fp32 phase (LoRaDemod.cpp:151-154), then the hardware
    // sine/cosine on its fractional revolution (v_fract, v_sin_f32, v_cos_f32) instead of
    // glibc's sincosf - not bit-exact (include/lora_mi355x.h states the tolerance).
    constexpr float INV_2PI = 0.159154943091895335768883763372514362f;
    static_assert(!FMA, "the certified demod rotates with spec_rotate_place");
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float ph = start + rate * (float)(l + T * q);
      const float rev = __builtin_amdgcn_fractf(ph * INV_2PI);
      cf v = cmul_t<FMA>(in[q], cf{__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)});
      if (hann) v = cscale(v, win[l + T * q]);
      z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
    }
    return;
  }
  if constexpr (!ROT) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      cf v = in[q];
      if (hann) v = cscale(v, win[l + T * q]);
      z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
    }
    return;
  }
  // The rotation phase is monotone in i, so the symbol's |ph| range is bounded by its
  // two end points; the branch-free sincosf covers |ph| < 120 (lora_libm.h).
  const bool sym_fast = lm_sincosf_fast_ok(start) && lm_sincosf_fast_ok(start + rate * (float)(N - 1));
  if (__all(sym_fast)) {
    constexpr int K = 4;
#pragma unroll
    for (int q0 = 0; q0 < P; q0 += K) {
      float ph[K], sn[K], cs[K];
#pragma unroll
      for (int k = 0; k < K; ++k) ph[k] = start + rate * (float)(l + T * (q0 + k));
      lm_sincosf_fast_k_nz<K>(ph, sn, cs);  // argmax-only: sign of a zero sine is immaterial
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int q = q0 + k;
        cf v = cmul(in[q], cf{cs[k], sn[k]});
        if (hann) v = cscale(v, win[l + T * q]);
        z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
      }
    }
  } else {  // some phase beyond the fast range: branch-free reduction select per point
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float ph = start + rate * (float)(l + T * q);
      float sn, cs;
      lm_sincosf_bf(ph, &sn, &cs);
      cf v = cmul(in[q], cf{cs, sn});
      if (hann) v = cscale(v, win[l + T * q]);
      z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = v;
    }
  }
}

// The certified speculative demod's rotation (LoRaDemod.cpp:151-157 up to one constant
// factor per symbol).  The reference rotates point i of symbol s by e^{i (c + rate i)} with
// c = rate (s N + t_off): the factor e^{i c} is common to the symbol's points, so it
// multiplies every bin by one unit-modulus number and changes no |X| - the speculative
// transform leaves it out and rotates by e^{i rate i} alone.  The lane's points i = l + T q
// are T apart: factor q is r0 wd^q with r0 = e^{i rate l} and wd = e^{i rate T} (rate T is
// exact: T is a power of two), each from one hardware sin/cos pair of its fractional
// revolution, then a packed complex-product recurrence.  certify_list bounds the factors'
// error (e_spec); the phases stay below rmax N, whatever the symbol's position in the frame.
template <int SF>
__device__ __forceinline__ void spec_factors(float rate, int l, v2f* F) {
  constexpr int T = Geo<SF>::T, P = Geo<SF>::P;
  constexpr float INV_2PI = 0.159154943091895335768883763372514362f;
  const float rev0 = __builtin_amdgcn_fractf((rate * (float)l) * INV_2PI);
  const float revd = __builtin_amdgcn_fractf((rate * (float)T) * INV_2PI);
  const float cd = __builtin_amdgcn_cosf(revd), sd = __builtin_amdgcn_sinf(revd);
  // Plain vector arithmetic (scalar fp32 in this TU), at least for the first step: the
  // hazard recognizer does not see an asm instruction read a transcendental's result (gfx950
  // needs a wait state there), and that step's own operations put the distance between the
  // sin/cos and any packed step after it.  SF 10-12 (16 factors per lane): the later steps
  // two per asm statement (pk_cmul_chain2, the same operations bit for bit; SF12 symbol pass
  // -0.3 %, SF7 +0.2 % - kept scalar there).
  const v2f wdr = {cd, cd}, wdi = {-sd, sd};
  F[0] = v2f{__builtin_amdgcn_cosf(rev0), __builtin_amdgcn_sinf(rev0)};
  constexpr int QS = SF >= 10 ? 2 : P;  // first packed step
#pragma unroll
  for (int q = 1; q < QS && q < P; ++q) F[q] = __builtin_elementwise_fma(F[q - 1].yx, wdi, F[q - 1] * wdr);
  const v2f wd = {cd, sd};
#pragma unroll
  for (int q = QS; q + 1 < P; q += 2) pk_cmul_chain2(F[q - 1], wd, F[q], F[q + 1]);
  if constexpr (QS < P && ((P - QS) % 2) == 1) F[P - 1] = pk_cmul(F[P - 2], wd);
}
// The SF7 pair-load symbol pass's factors (k_spec_demod PL): F[h + 2 m] = e^{i rate (r_h + 16 m)}
// for the lane's two residues r_h: e^{i rate r_h} and w = e^{i rate 16} from one hardware
// sin/cos pair each (rate 16 is exact), then 7 complex-product steps per residue (the form
// of spec_factors' steps).  Error per factor (certify_list's e_spec): the arguments fl(rate r_h)
// and their products by 1/2pi (3 u rmax 15), w's product (2 u rmax 16) times up to 7 steps -
// 33.6 u rmax T at T = 8, inside the bound's 36 u rmax T; up to 8 sin/cos and fract errors
// and 7 product roundings, inside its 16 and 15.
__device__ __forceinline__ void spec_factors_pl(float rate, const int* r, v2f* F) {
  constexpr float INV_2PI = 0.159154943091895335768883763372514362f;
  const float revw = __builtin_amdgcn_fractf((rate * 16.0f) * INV_2PI);
  const float cw = __builtin_amdgcn_cosf(revw), sw = __builtin_amdgcn_sinf(revw);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float rev0 = __builtin_amdgcn_fractf((rate * (float)r[h]) * INV_2PI);
    F[h] = v2f{__builtin_amdgcn_cosf(rev0), __builtin_amdgcn_sinf(rev0)};
  }
  const v2f wr = {cw, cw}, wi = {-sw, sw};
#pragma unroll
  for (int m = 1; m < 8; ++m)
#pragma unroll
    for (int h = 0; h < 2; ++h) F[h + 2 * m] = __builtin_elementwise_fma(F[h + 2 * m - 2].yx, wi, F[h + 2 * m - 2] * wr);
}

// the window's samples times the factors (and the Hann window, LoRaDemod.cpp:158-160), in
// pass-1 leaf order
// FOLD: only the leading input of each of pass 1's first-stage butterflies (position p with
// p % 4 == 0, or p % 2 == 0 for the odd-SF radix-2 stage) is multiplied here; the others keep
// their samples (times the window) and hand their factor to fft_key<..., FOLD> as the
// butterfly's twiddle (wz[p]).  The same rounding terms as the separate product (the bound's
// rotation product and butterfly levels), in a different order.
template <int SF, bool HANN, bool FOLD = false>
__device__ __forceinline__ void spec_rotate_place(const cf* in, cf* z, const v2f* F, const float* __restrict__ win,
                                                  int l, cf* wz = nullptr) {
  using G = Geo<SF>;
  constexpr int T = G::T, P = G::P, R1 = G::R1;
  constexpr int LEAD = G::R2FIRST ? 2 : 4;  // first-stage butterfly span
  if constexpr (SF >= 10 && !FOLD && !HANN && P % 2 == 0) {  // products two per asm statement
#pragma unroll
    for (int q = 0; q < P; q += 2) {
      v2f r0, r1;
      pk_cmul2(pk(in[q]), F[q], pk(in[q + 1]), F[q + 1], r0, r1);
      z[(q % G::G1) * R1 + leaf_pos(R1, q / G::G1)] = unpk(r0);
      z[((q + 1) % G::G1) * R1 + leaf_pos(R1, (q + 1) / G::G1)] = unpk(r1);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < P; ++q) {
    const int p = (q % G::G1) * R1 + leaf_pos(R1, q / G::G1);
    if (FOLD && (p % LEAD) != 0) {
      cf v = in[q];
      if constexpr (HANN) v = cscale(v, win[l + T * q]);
      z[p] = v;
      wz[p] = unpk(F[q]);
    } else {
      cf v = unpk(pk_cmul(pk(in[q]), F[q]));
      if constexpr (HANN) v = cscale(v, win[l + T * q]);
      z[p] = v;
    }
  }
}

// Pass 1's twiddles in the certified transforms: indices m N/16 (MA = 1; m <= 9), i.e.
// e^{-2 pi i m / 16}, as fp32 constants (correctly rounded: the table's values up to its own
// rounding, which the certification's E carries either way).  Loaded from the table every
// round they cost the prefetching symbol pass 5 % at SF7 (an L2 round trip per round).
__device__ __forceinline__ cf w16(int m) {
  constexpr float C1 = 0.923879532511286756f, S1 = 0.382683432365089772f, R2 = 0.707106781186547524f;
  switch (m) {
    case 0: return cf{1.0f, 0.0f};
    case 1: return cf{C1, -S1};
    case 2: return cf{R2, -R2};
    case 3: return cf{S1, -C1};
    case 4: return cf{0.0f, -1.0f};
    case 5: return cf{-S1, -C1};
    case 6: return cf{-R2, -R2};
    case 7: return cf{-C1, -S1};
    case 8: return cf{-1.0f, 0.0f};
    default: return cf{-C1, S1};
  }
}
template <int N>
struct ConstTw1 {
  __device__ __forceinline__ cf operator[](int i) const { return w16(i / (N / 16)); }
};

// FFT of the symbol held as pass-1 inputs in z (T lanes x P points) and the lane's
// argmax key.  KEEP: leave the spectrum in natural order in `row` (padded address
// paddr(bin)) for the estimate's neighbour bins; NPASS == 1 keeps it in z.
// CPRE: the pass-1 write-back positions c[h] (rev[l + T h] >> LOGR1) come from the caller
// instead of vector loads.  FMA (the certified transforms): pass 1's twiddles are constants
// (ConstTw1).
// FOLD (certified symbol pass, spec_rotate_place<..., true>): pass 1's first stage takes the
// rotation factors of its non-leading inputs as twiddles (wfold[p], position p in z) - their
// inputs arrive unrotated - instead of the unit butterflies after a separate product: a
// radix-4 stage 14 packed instructions per four points instead of 16, a radix-2 one 5 per
// two instead of 6.
template <int SF, bool KEEP, bool FMA = false, bool TWL = false, bool PACK = false, bool CPRE = false,
          class HOOK = NoHook, bool FOLD = false>
__device__ __forceinline__ uint64_t fft_key(cf* z, cf* row, int l, const KArgs& a, float* second = nullptr,
                                            const cf* twl = nullptr, const int* cpre = nullptr, HOOK hook = HOOK{},
                                            const cf* wbpre = nullptr, const cf* wfold = nullptr) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P, R1 = G::R1;
  constexpr bool WL = G::WAVE_LOCAL;
  static_assert(!FOLD || FMA, "the folded rotation is the certified path's");
#pragma unroll
  for (int h = 0; h < G::G1; ++h) {
    if constexpr (FOLD) {
      cf* x = z + h * R1;
      const cf* w = wfold + h * R1;
      if constexpr (G::R2FIRST) {
#pragma unroll
        for (int b = 0; b < R1; b += 2) bfly2<true>(x[b], x[b + 1], w[b + 1]);
      } else {
#pragma unroll
        for (int b = 0; b < R1; b += 4) bfly4<true>(x[b], x[b + 1], x[b + 2], x[b + 3], w[b + 1], w[b + 2], w[b + 3]);
      }
      pass_regs<R1, G::R2FIRST, N, 1, !KEEP, FMA, ConstTw1<N>, true>(x, 0, ConstTw1<N>{});
    } else if constexpr (FMA) {
      pass_regs<R1, G::R2FIRST, N, 1, !KEEP, FMA, ConstTw1<N>>(z + h * R1, 0, ConstTw1<N>{});
    } else {
      pass_regs<R1, G::R2FIRST, N, 1, !KEEP, FMA>(z + h * R1, 0, a.tw);
    }
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
    int c[G::G1];
#pragma unroll
    for (int h = 0; h < G::G1; ++h) c[h] = CPRE ? cpre[h] : (int)(a.rev[l + T * h] >> G::LOGR1);
#pragma unroll
    for (int h = 0; h < G::G1; ++h)
#pragma unroll
      for (int u = 0; u < R1; ++u)
        row[lds_slot<SF>(c[h] * R1) + u] = z[h * R1 + u];  // u < 16
    block_sync<WL>();
    constexpr int RL = G::NPASS == 2 ? G::RA : G::RB;   // last pass span
    constexpr int ML = G::NPASS == 2 ? G::MA_A : G::MA_B;
    // TWL: pass A's slot-major twiddles from the workgroup's LDS copy (k_demod_fast)
    const cf* twA = TWL ? twl : a.twTA;
    if constexpr (G::NPASS == 2) {
      pass_lds<G::RA, N, G::MA_A, SF, T, P, true, FMA, false, TWL, PACK>(row, z, l, a.tw, key, twA, second);
    } else {
      pass_lds<G::RA, N, G::MA_A, SF, T, P, false, FMA, false, TWL>(row, z, l, a.tw, key, twA);
      block_sync<WL>();
      write_pass<G::RA, G::MA_A, SF, T, P>(row, z, l);
      block_sync<WL>();
      // TWL (speculative demod): pass B's twiddles two per 16-byte load (KArgs::twTB2)
      if constexpr (!std::is_same_v<HOOK, NoHook>) {
        // every group's twiddles first, then the hook, then the pass
        // (the caller, which installs the hook, loaded them earlier in its round: wbpre)
        const cf* wb = wbpre;
        __builtin_amdgcn_sched_barrier(0);
        hook();
        __builtin_amdgcn_sched_barrier(0);
        pass_lds<G::RB, N, G::MA_B, SF, T, P, true, FMA, true, TWL, PACK>(row, z, l, a.tw, key, a.twTB2, second, wb);
      } else {
        pass_lds<G::RB, N, G::MA_B, SF, T, P, true, FMA, true, TWL, PACK>(row, z, l, a.tw, key, a.twTB2, second);
      }
    }
    if constexpr (KEEP) {
      // last-pass outputs: bin = (l + T*gg) + ML*u (cc == 0)
      block_sync<WL>();
#pragma unroll
      for (int gg = 0; gg < P / RL; ++gg)
#pragma unroll
        for (int u = 0; u < RL; ++u) row[lds_slot<SF>(l + T * gg) + lds_slot<SF>(ML * u)] = z[gg * RL + u];
      block_sync<WL>();
    }
  }
  return key;
}

// Two independent transforms of the same shape (the estimate's symbols 0 and 1) in
// lockstep, for the wave-local two-pass geometries: the same operations as two
// fft_key calls, interleaved so each transform's latency hides behind the other's.
template <int SF, bool KEEP>
__device__ __forceinline__ void fft_key2(cf* z0, cf* z1, cf* row0, cf* row1, int l, const KArgs& a,
                                         uint64_t& k0, uint64_t& k1) {
  using G = Geo<SF>;
  static_assert(G::NPASS == 2 && G::WAVE_LOCAL, "wave-local two-pass transforms only");
  constexpr int N = G::N, T = G::T, P = G::P, R1 = G::R1;
#pragma unroll
  for (int h = 0; h < G::G1; ++h) {
    pass_regs<R1, G::R2FIRST, N, 1, !KEEP>(z0 + h * R1, 0, a.tw);
    pass_regs<R1, G::R2FIRST, N, 1, !KEEP>(z1 + h * R1, 0, a.tw);
  }
  int c[G::G1];
#pragma unroll
  for (int h = 0; h < G::G1; ++h) c[h] = (int)(a.rev[l + T * h] >> G::LOGR1);
#pragma unroll
  for (int h = 0; h < G::G1; ++h)
#pragma unroll
    for (int u = 0; u < R1; ++u) {
      row0[lds_slot<SF>(c[h] * R1) + u] = z0[h * R1 + u];
      row1[lds_slot<SF>(c[h] * R1) + u] = z1[h * R1 + u];
    }
  wave_sync();
  pass_lds<G::RA, N, G::MA_A, SF, T, P, true>(row0, z0, l, a.tw, k0, a.twTA);
  pass_lds<G::RA, N, G::MA_A, SF, T, P, true>(row1, z1, l, a.tw, k1, a.twTA);
  if constexpr (KEEP) {
    wave_sync();
#pragma unroll
    for (int gg = 0; gg < P / G::RA; ++gg)
#pragma unroll
      for (int u = 0; u < G::RA; ++u) {
        row0[lds_slot<SF>(l + T * gg) + lds_slot<SF>(G::MA_A * u)] = z0[gg * G::RA + u];
        row1[lds_slot<SF>(l + T * gg) + lds_slot<SF>(G::MA_A * u)] = z1[gg * G::RA + u];
      }
    wave_sync();
  }
}

// Argmax key over the T lanes of a symbol; every lane of the symbol gets the result.
template <int SF>
__device__ __forceinline__ uint64_t symbol_key(uint64_t key, int tid, uint64_t* red) {
  constexpr int T = Geo<SF>::T;
  if constexpr (T <= 64) {
    return group_max(key, T);
  } else {
    key = group_max(key, 64);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = key;
    __syncthreads();
    constexpr int WPS = T / 64;  // waves per symbol
    const int wb = ((tid >> 6) / WPS) * WPS;
    uint64_t r = red[wb];
#pragma unroll
    for (int q = 1; q < WPS; ++q) r = umax64(r, red[wb + q]);
    return r;
  }
}

// max(m, |v.re|, |v.im|) in one instruction (fmaxf would canonicalize each operand).
// Callers pin the running maximum with an empty volatile asm next to the loads it
// consumes: left to itself the compiler sinks the chain to the maximum's use after the
// FFT and keeps every input live until then.
__device__ __forceinline__ float amax3(float m, cf v) {
  asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m) : "v"(v.re), "v"(v.im));
  return m;
}

// Speculative demod (SPEC): the maxima of `a` and `b` over the symbol's T lanes (every
// lane gets them).  Wave-local groups use shuffles; T > 64 adds one LDS round through
// `rf` (2 floats per wave), which must not alias live data.
template <int SF>
__device__ __forceinline__ void group_reduce2(float& a, float& b, int tid, float* rf) {
  constexpr int T = Geo<SF>::T;
  constexpr int W = T < 64 ? T : 64;
#pragma unroll
  for (int o = W >> 1; o > 0; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o, 64));
    b = fmaxf(b, __shfl_xor(b, o, 64));
  }
  if constexpr (T > 64) {
    const int w = tid >> 6;
    if ((tid & 63) == 0) {
      rf[2 * w] = a;
      rf[2 * w + 1] = b;
    }
    __syncthreads();
    constexpr int WPS = T / 64;
    const int wb = (w / WPS) * WPS;
    a = rf[2 * wb];
    b = rf[2 * wb + 1];
#pragma unroll
    for (int q = 1; q < WPS; ++q) {
      a = fmaxf(a, rf[2 * (wb + q)]);
      b = fmaxf(b, rf[2 * (wb + q) + 1]);
    }
  }
}

// (best, second) of the symbol's bins from every lane's (best, second) keys, and the max
// of pm, over the symbol's T lanes (every lane gets them): the second is the runner-up of
// the whole multiset of bins, so two lanes holding equal best keys give a zero margin.
// pm (a maximum of absolute values: never negative, never NaN) travels as its bits, which
// order like the values.  The merge of two (best, second, max) triples is symmetric, so an
// exchange may hand a lane its own values back in either slot: steps 1-8 are DPP movs the
// compiler folds into the unsigned max / min (aligned blocks hold one value per step, so a
// mirror inside the next block up is the xor exchange), 16 and 32 the row / half swaps
// (v_permlane16_swap_b32, v_permlane32_swap_b32: one lane ends with each of the two
// values of its pair in the two slots).
__device__ __forceinline__ void top2_merge(uint32_t& b, uint32_t& s, uint32_t& p, uint32_t b2, uint32_t s2,
                                           uint32_t p2) {
  const uint32_t lo = b < b2 ? b : b2;
  const uint32_t hs = s > s2 ? s : s2;
  s = hs > lo ? hs : lo;
  b = b > b2 ? b : b2;
  p = p > p2 ? p : p2;
}
template <int O>
__device__ __forceinline__ uint32_t dpp_xchg(uint32_t v) {
  constexpr int ctrl = O == 1 ? 0xB1 : O == 2 ? 0x4E : O == 4 ? 0x141 : 0x140;  // quad perms, half / row mirror
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, true);
}
template <int O, int W>
__device__ __forceinline__ void spec_reduce_step(uint32_t& best, uint32_t& sec, uint32_t& pm) {
  if constexpr (O < W) {
    if constexpr (O <= 8) {
      top2_merge(best, sec, pm, dpp_xchg<O>(best), dpp_xchg<O>(sec), dpp_xchg<O>(pm));
    } else if constexpr (O == 16) {
      const auto xb = __builtin_amdgcn_permlane16_swap(best, best, false, false);
      const auto xs = __builtin_amdgcn_permlane16_swap(sec, sec, false, false);
      const auto xp = __builtin_amdgcn_permlane16_swap(pm, pm, false, false);
      best = xb[0], sec = xs[0], pm = xp[0];
      top2_merge(best, sec, pm, xb[1], xs[1], xp[1]);
    } else {
      static_assert(O == 32, "wave64");
      const auto xb = __builtin_amdgcn_permlane32_swap(best, best, false, false);
      const auto xs = __builtin_amdgcn_permlane32_swap(sec, sec, false, false);
      const auto xp = __builtin_amdgcn_permlane32_swap(pm, pm, false, false);
      best = xb[0], sec = xs[0], pm = xp[0];
      top2_merge(best, sec, pm, xb[1], xs[1], xp[1]);
    }
    spec_reduce_step<2 * O, W>(best, sec, pm);
  }
}
template <int SF>
__device__ __forceinline__ void spec_reduce(uint32_t& best, uint32_t& sec, float& pmf, int tid, uint32_t* scratch) {
  constexpr int T = Geo<SF>::T;
  uint32_t pm = __float_as_uint(pmf);
  spec_reduce_step<1, (T < 64 ? T : 64)>(best, sec, pm);
  if constexpr (T > 64) {  // waves of one symbol: one LDS round (3 words per wave)
    const int w = tid >> 6;
    if ((tid & 63) == 0) {
      scratch[3 * w] = best;
      scratch[3 * w + 1] = sec;
      scratch[3 * w + 2] = pm;
    }
    __syncthreads();
    constexpr int WPS = T / 64;
    const int wb = (w / WPS) * WPS;
    best = scratch[3 * wb];
    sec = scratch[3 * wb + 1];
    pm = scratch[3 * wb + 2];
#pragma unroll
    for (int q = 1; q < WPS; ++q)
      top2_merge(best, sec, pm, scratch[3 * (wb + q)], scratch[3 * (wb + q) + 1], scratch[3 * (wb + q) + 2]);
  }
  pmf = __uint_as_float(pm);
}

// MODE 0: LEGACY + fused dechirp, osr 1, no window (the benchmark configuration);
// MODE 1: LEGACY on already-dechirped input, osr 1, no window (lora_demodulate's own
//         contract); MODE 2: every other LEGACY / API configuration, flags read at run
//         time; MODE 3: RAW (detector only: no normalisation, estimate or rotation).
// Register budget: 4 waves per SIMD (<= 128 VGPRs) for SF >= 6 - the LDS rows allow
// 4 workgroups per CU, so this is the occupancy ceiling.  With scalar fp32 the kernels
// need 115-128 VGPRs and fit without spilling; SF <= 5 keeps a whole symbol per lane
// (P = N complex values) and is left to the compiler.  (Under packed fp32 the SF7 cap
// alone was worth 4-5 %, tools/exp/variant_ab.sh.)
template <int SF>
constexpr int demod_waves_per_eu() {
  return SF >= 6 ? 4 : 1;
}

// Speculative demod: pass A's slot-major twiddles (15 or 3 per butterfly group, MA_A
// groups: 48-240 values) are staged once per workgroup in LDS after the symbol rows, so
// the pass reads them with ds_read instead of 15 vector loads per lane - the vector
// memory path (texture addresser) is the demod's busiest unit.  Same values, same
// arithmetic.  Returns the number of staged values (0: off).
template <int SF, bool SPEC>
constexpr int demod_twl_entries() {
  if constexpr (!SPEC || SF < 6) {
    return 0;
  } else {
    using G = Geo<SF>;
    return (G::RA == 16 ? 15 : 3) * G::MA_A;
  }
}


// k_spec_demod's LDS: the symbol rows, pass A's twiddles, then (prefetching geometries) the
// dechirp table's pairs at table phase 0, 16-byte aligned.
template <int SF>
constexpr size_t spec_dtl_offset() {
  return (((size_t)Geo<SF>::SPW * lds_row<SF>() + demod_twl_entries<SF, true>()) * sizeof(cf) + 15) & ~(size_t)15;
}
// SF 6-8: instead of the table-phase-0 slice, the whole doubled dechirp table (KArgs::down,
// 2N entries: 1-4 KB), so a window at any table phase - every frame with t_off != 0, i.e.
// every captured frame - reads its table values from LDS too (four workgroups per CU still
// fit); SF9 keeps the slice (its 8 KB table would cost the fourth workgroup).  Same-box A/B
// against the slice (tools/r05_ab.py, three interleaved runs): SF7 symbol pass 0.2187 ->
// 0.2146 ms noiseless, 0.2467 -> 0.2352 at 0 dB, 0.2523 -> 0.2390 at -10 dB.
template <int SF>
constexpr bool spec_dtab() {
  return Geo<SF>::WAVE_LOCAL && Geo<SF>::NPASS == 2 &&
         4 * (spec_dtl_offset<SF>() + 2 * sizeof(cf) * Geo<SF>::N) <= 160 * 1024;
}
template <int SF>
constexpr size_t spec_lds_bytes() {
  constexpr bool pf2 = Geo<SF>::WAVE_LOCAL && Geo<SF>::NPASS == 2;
  return pf2 ? spec_dtl_offset<SF>() + (spec_dtab<SF>() ? 2 * sizeof(cf) * Geo<SF>::N : 16 * 8 * Geo<SF>::T)
             : sizeof(cf) * ((size_t)Geo<SF>::SPW * lds_row<SF>() + demod_twl_entries<SF, true>());
}

// osr 4 in the symbol pass: whole-line loads with a lane move (1) or two half-line loads per
// point (0, rounds 4-5)
#ifndef LORA_OSR4_LINES
#define LORA_OSR4_LINES 1
#endif

// SPEC: the speculative single-read pipeline's symbol pass (lora_capi.hip): the pre-pass
// offsets (fp_spec) on unscaled samples, and per data symbol (spec_marg, one 8-byte
// store) the margin |X1| - |X2| between the top bin and the runner-up and the window's
// max(|I|,|Q|), which k_est_fast<SPEC = 2> uses to normalise, certify or recompute.
template <int SF, int MODE, bool FAST = false, bool SPEC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(demod_waves_per_eu<SF>())))
k_demod_fast(KArgs a, int s0, int64_t work, int rowc) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P, SPW = G::SPW;
  constexpr bool RAW = MODE == 3;
  constexpr bool DYN = MODE >= 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint64_t red[4];
  cf* rows = reinterpret_cast<cf*>(smem);
  const int tid = threadIdx.x;
  const int per = a.total - s0;
  const int step = DYN ? a.step : N;
  const int osr = DYN ? a.osr : 1;
  const bool legacy = RAW ? true : DYN ? a.mode != LORA_MODE_API : true;
  const bool dech = DYN ? (legacy && a.dechirp) : (MODE == 0);
  const bool hann = DYN ? (a.hann != 0) : false;

  const int g = tid / T;  // slot
  const int l = tid % T;  // lane within the symbol
  // work item w -> (frame f, symbol s): one 64-bit division per workgroup on the scalar
  // unit, then a small per-lane quotient (the SPW symbols of a workgroup span few frames)
  const int64_t w0 = (int64_t)blockIdx.x * SPW;
  const int64_t f0 = w0 / per;
  const int r0 = (int)(w0 - f0 * per);
  const int64_t w = w0 + g;
  const bool valid = w < work;
  const int loc = r0 + (int)((valid ? w : work - 1) - w0);  // clamp: invalid lanes mirror a valid symbol
  const int q = per >= SPW ? (loc >= per ? 1 : 0) : (int)((unsigned)loc / (unsigned)per);
  const int64_t f = f0 + q;
  const int s = s0 + (loc - q * per);
  const FrameParams p = RAW ? FrameParams{0.0f, 0.0f, 0.0f, 1.0f, 0, 0, 0, 0} : (SPEC ? a.fp_spec[f] : a.fp[f]);
  int64_t base;
  int cg;
  sym_base(s, step, a.frame_len, p.t_off, base, cg);
  const cf* __restrict__ x = a.iq + f * a.frame_stride + base;
  const float start = p.rate * ((float)((uint32_t)s * (uint32_t)N) + (float)p.t_off / (float)osr);
  // LoRaDemod.cpp:68-77: scale is 1.0f when the frame is not rescaled (x*1.0f == x).
  const float scale = (legacy && p.scaled) ? p.scale : 1.0f;

  // The speculative demod with the hardware rotation (certified for every frame) also
  // uses fused multiply-adds for the rotation and the FFT, and skips the unit scale.  The
  // dechirp product keeps the reference's arithmetic: the frame maximum (hence the scale,
  // cfo, time_offset and max_amp outputs) is taken over exactly these samples.
  constexpr bool FMA = SPEC && FAST;
  constexpr int NTW = demod_twl_entries<SF, SPEC>();
  static_assert(NTW <= 256, "one staged twiddle per thread");
  cf* twl = rows + (size_t)SPW * rowc;
  cf tv{0.0f, 0.0f};
  if constexpr (NTW > 0) {  // issued first: it returns ahead of the symbol's gathers
    if (tid < NTW) tv = a.twTA ? a.twTA[tid] : a.tw[twT_index(N, G::MA_A, tid / G::MA_A, tid % G::MA_A)];
  }
  cf in[P], z[P];
  if (SPEC && MODE == 0 && a.downP)  // the speculative demod's scale is 1
    gather_points<SF, true>(a, x, l, 1, N, cg, 1, true, 1.0f, in);
  else
    gather_points<SF>(a, x, l, osr, step, cg, legacy ? 1 : 2, dech, SPEC ? 1.0f : scale, in);
  if constexpr (NTW > 0) {
    if (tid < NTW) twl[tid] = tv;
    // wave-local kernels have no workgroup barrier before pass A; the others' first one
    // (after the pass-1 write-back in fft_key) orders these writes
    if constexpr (G::WAVE_LOCAL) __syncthreads();
  }
  float pm = 0.0f;
  if constexpr (SPEC) {  // the window's dechirped, unscaled samples (scale is 1 here)
#pragma unroll
    for (int q = 0; q < P; ++q) pm = amax3(pm, in[q]);
  }
  rotate_place<SF, !RAW, FAST, FMA>(in, z, start, p.rate, hann, a.win, l);
  if constexpr (SPEC) asm volatile("" : "+v"(pm));
  float sec = 0.0f;
  const uint64_t lkey =
      fft_key<SF, false, FMA, (NTW > 0)>(z, rows + (size_t)g * rowc, l, a, SPEC ? &sec : nullptr, twl);
  const uint64_t key = symbol_key<SF>(lkey, tid, red);
  if (l == 0 && valid && a.syms) a.syms[f * a.sym_stride + (s - s0)] = (uint16_t)key_index(key);
  if constexpr (SPEC) {
    // runner-up over the symbol: the top lane offers its own runner-up, the others their best
    float r2 = lkey == key ? sec : key_value(lkey);
    group_reduce2<SF>(r2, pm, tid, reinterpret_cast<float*>(smem + 64));
    if (l == 0 && valid) {
      const int64_t per = a.total - s0;
      reinterpret_cast<float2*>(a.spec_marg)[f * per + (s - s0)] = make_float2(sqrtf(key_value(key)) - sqrtf(r2), pm);
    }
  }
}


// ---- the speculative pipeline's symbol pass -----------------------------------------
// k_spec_demod: every symbol of LEGACY osr-1 unwindowed frames (MODE 0: fused caller
// dechirp from the paired table KArgs::downP; MODE 1: dechirped input) with the pre-pass
// offsets (fp_spec) on UNSCALED samples, the hardware rotation and fused multiply-adds:
// per data symbol its index, top-bin / runner-up margin and window max(|I|,|Q|), per sync
// symbol its margin and index (one 8-byte spec_marg entry each), all certified or
// recomputed exactly by k_est_fast<SPEC = 2> / k_spec_fix.  The arithmetic is
// k_demod_fast<SF, MODE, true, true>'s.
// The work is cut into blocks of SPB symbols (a wave's 64/T for T <= 64, the workgroup's
// SPW beyond): first every frame's data symbols, SPB consecutive ones of one frame per block
// (a frame's last block may be partial), so the frame, its offsets and every address but
// the lane's own are wave-uniform (scalar registers and loads); then the sync symbols, the
// two of SPB/2 consecutive frames per block.  Persistent: a workgroup takes groups of BPG
// blocks blockIdx.x, blockIdx.x + gstride, ... (gstride = the grid: a few workgroups per CU,
// launch_spec_demod) - short waves (about 4 us at SF7) left the CUs half occupied between
// one workgroup's end and the next one's start.
// OSRV != 1: oversampled frames (LEGACY osr 2-4): a symbol's points are every osr-th sample
// of its window (LoRaDemod.cpp:141-157 reads sym_samps[i * osr]), and the window's other
// samples are read with them for the frame maximum, which the reference takes over every
// sample (LoRaDemod.cpp:59-67) - the frame is still read once.  OSRV 2 / 4: osr known at
// compile time, a point's osr samples in one / two 16-byte loads; OSRV 0: a.osr at run time
// (osr 3, and the Hann window), one 8-byte load per sample.
// SPM (lora_capi.hip) 1 = API (LORA_MODE_API at osr 1): each window times the down-chirp
// from table phase 0 (phy.cpp:211-225 multiplies sym[i] by a fresh down-chirp's [i]) with the
// exact offsets, no sync blocks (the estimate kernel demodulated symbols 0/1 exactly); 2 =
// RAW (LORA_MODE_RAW at osr 1, the detector alone, LoRaDetector.hpp:39-58): every symbol of
// the frame an output at t_off 0 with no rotation (the factors of rate 0 are exactly 1).
// Both zero the reject list's counters here (no pre-pass runs).
template <int SF, int MODE, bool HANN = false, int OSRV = 1, int SPM = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(demod_waves_per_eu<SF>())))
k_spec_demod(KArgs a, int64_t frames, int rowc, int64_t gstride) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P, SPW = G::SPW;
  constexpr bool WL = G::WAVE_LOCAL;
  constexpr int SPB = WL ? 64 / T : SPW;  // symbols per block
  constexpr int BPG = WL ? 4 : 1;         // blocks per workgroup round
  constexpr int NTW = demod_twl_entries<SF, true>();
  constexpr bool OSRN = OSRV != 1;
  // the rotation folded into pass 1's first stage (fft_key FOLD): where the registers allow it
  // (SF 9-12 and the windowed SF 6-8 kernels spill with the factors held until the stage)
  constexpr bool FOLD = SF <= 8 && !HANN;
  static_assert(P == 16 && (MODE == 0 || MODE == 1), "SF >= 6, LEGACY (osr 1, or OSRN)");
  static_assert(OSRV == 0 || OSRV == 1 || OSRV == 2 || OSRV == 4, "osr 1, 2, 4 or run time");
  static_assert(NTW <= 256, "one staged twiddle per thread");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t red3[3 * 4];  // spec_reduce's cross-wave words (T > 64)
  cf* rows = reinterpret_cast<cf*>(smem);
  cf* twl = rows + (size_t)SPW * rowc;
  const int tot = a.total;
  constexpr bool API = SPM == 1, RAWM = SPM == 2;
  constexpr int S0 = RAWM ? 0 : 2;  // the frame's first output symbol
  const int per = tot - S0;
  // (PF geometries, MODE 0) the dechirp table's pairs at table phase 0 - what every window
  // of a t_off = 0 frame reads - staged after the twiddles: dtl[p T + c] = downP[p (N + T) + c]
  constexpr bool DTL = WL && G::NPASS == 2 && !OSRN && MODE == 0;
  // DTAB (SF 6-8): the whole doubled table instead, for every table phase
  constexpr bool DTAB = DTL && spec_dtab<SF>();
  float4* dtl = reinterpret_cast<float4*>(smem + spec_dtl_offset<SF>());
  cf* dtab = reinterpret_cast<cf*>(smem + spec_dtl_offset<SF>());
  if (SPM != 0 && blockIdx.x == 0 && threadIdx.x < kFixStripes) a.fix_count[16 * threadIdx.x] = 0;
  if constexpr (NTW > 0) {
    const int tid = threadIdx.x;
    if (tid < NTW) twl[tid] = a.twTA ? a.twTA[tid] : a.tw[twT_index(N, G::MA_A, tid / G::MA_A, tid % G::MA_A)];
    if constexpr (DTAB) {
      for (int i = tid; i < 2 * N; i += 256) dtab[i] = a.down[i];
    } else if constexpr (DTL) {
      static_assert(8 * T <= 256, "one staged pair per thread");
      if (tid < 8 * T) dtl[tid] = reinterpret_cast<const float4*>(a.downP)[(tid / T) * (N + T) + tid % T];
    }
    __syncthreads();
  }
  const int bpf = (per + SPB - 1) / SPB;  // data blocks per frame
  const int64_t dblocks = frames * bpf;
  const int64_t blocks = dblocks + (SPM != 0 ? 0 : (2 * frames + SPB - 1) / SPB);
  const int64_t groups = (blocks + BPG - 1) / BPG;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  typedef float v2f __attribute__((ext_vector_type(2)));

  // one block: SYNC = false a data block (frame-uniform), true a sync block
  // b: the block; data blocks come with b = fb bpf + rb (the loop keeps the quotient)
  auto run_block = [&](auto sync_c, int64_t b, int64_t fb, int rb) {
    constexpr bool SYNC = decltype(sync_c)::value;
    // the lane index, opaque per round: left visible, the compiler hoists every lane
    // address out of the loop and keeps them live across it (more VGPRs, spills at SF12)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int g = SPW == 1 ? 0 : tid / T;  // slot in the workgroup (its LDS row)
    const int l = tid % T;                 // lane within the symbol
    const int gi = WL ? (g % SPB) : g;     // symbol within the block
    int64_t f, fu;  // the lane's frame; the block's first (wave-uniform)
    int s;          // symbol within the frame
    bool valid;
    int rel = 0;    // byte offset of frame f from frame fu
    if constexpr (!SYNC) {
      f = fu = fb;
      const int jl = rb * SPB + gi;
      valid = jl < per;
      s = S0 + (valid ? jl : per - 1);  // a partial block's spare slots mirror a valid symbol
    } else {
      const int64_t k0 = (b - dblocks) * SPB;
      int64_t k = k0 + gi;
      valid = k < 2 * frames;
      if (!valid) k = 2 * frames - 1;
      f = k >> 1;
      s = (int)(k & 1);
      fu = k0 >> 1;
      rel = (int)((f - fu) * a.frame_stride * 8);  // < 2^31: lora_demod_batch checks the stride
    }
    const FrameParams fp = RAWM ? FrameParams{} : a.fp_spec[f];
    const float rate = RAWM ? 0.0f : fp.rate;
    const int toff = RAWM ? 0 : fp.t_off;
    const int step = OSRN ? a.step : N;
    int64_t base;
    int cg;
    sym_base(s, step, a.frame_len, toff, base, cg);
    if constexpr (API) cg = 0;
    cf in[P];
    float pm = 0.0f;
    int lr = l;
    if constexpr (OSRN) {
      // point q of lane l is sample base + (l + T q) osr; the osr samples from it on are
      // dechirped (MODE 0: table down[cg + j], no wrap) and enter the window's maximum
      const int osr = OSRV ? OSRV : a.osr;
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.iq + fu * a.frame_stride), (short)0, 0x7fffffff, 0x00020000);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)a.down, (short)0, 0x7fffffff, 0x00020000);
      const int vo = rel + (int)(base + (int64_t)l * osr) * 8;
      const int vt = (cg + l * osr) * 8;
      const int so = T * osr * 8;  // bytes between a lane's points
      if constexpr (OSRV == 4 && LORA_OSR4_LINES) {
        // osr 4, whole lines: load i (< 2P) covers 2T consecutive samples of the window, lane l
        // the pair base + 2T i + 2l, +1 (16 bytes; a wave instruction reads whole 128-byte
        // lines).  The points (every 4th sample) are the first of an even lane's pairs - those
        // of even i role l/2's points, those of odd i role T/2 + l/2's, which the odd lane
        // l + 1 takes by a row_shr:1 lane move: every byte read once, by one load, in whole
        // lines (the two half-line 16-byte loads per point fetched 1.24x the window's bytes).
        const bool odd = (l & 1) != 0;
        lr = odd ? T / 2 + (l >> 1) : (l >> 1);
        const int vo2 = rel + (int)base * 8 + 16 * l;
        const int vt2 = (cg + 2 * l) * 8;
#pragma unroll
        for (int q = 0; q < P; ++q) {
          cf e0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * q + h;
            const float4 y2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo2, i * 2 * T * 8, 2 /* nt */));
            cf y0 = cf{y2.x, y2.y}, y1 = cf{y2.z, y2.w};
            if constexpr (MODE == 0) {
              const float4 d2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, vt2, i * 2 * T * 8, 0));
              y0 = pk_cmul_ref(y0, cf{d2.x, d2.y});
              y1 = pk_cmul_ref(y1, cf{d2.z, d2.w});
            }
            if constexpr (!SYNC) pm = amax3(amax3(pm, y0), y1);
            if (h == 0) {
              e0 = y0;
            } else {
              // lane l - 1's pair (row_shr:1; even lanes' own values are replaced below)
              const cf m = cf{__int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y0.re), 0x111, 0xF, 0xF, false)),
                              __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y0.im), 0x111, 0xF, 0xF, false))};
              in[q] = odd ? m : e0;
            }
          }
        }
      } else if constexpr (OSRV == 2 || OSRV == 4) {
        // the point's osr consecutive samples (and table values) two per 16-byte load: every
        // byte of the window is fetched by exactly one load (8-byte loads of every osr-th
        // sample, osr of them over the same lines, cost 1.31x the window's bytes at osr 2
        // and 0.75 ms per 15,625-frame SF7 step against 0.41)
#pragma unroll
        for (int q = 0; q < P; ++q) {
#pragma unroll
          for (int h = 0; h < OSRV / 2; ++h) {
            const float4 y2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo + 16 * h, q * so, 2 /* nt */));
            cf y0 = cf{y2.x, y2.y}, y1 = cf{y2.z, y2.w};
            if constexpr (MODE == 0) {
              const float4 d2 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, vt + 16 * h, q * so, 0));
              y0 = pk_cmul_ref(y0, cf{d2.x, d2.y});
              y1 = pk_cmul_ref(y1, cf{d2.z, d2.w});
            }
            if constexpr (!SYNC) pm = amax3(amax3(pm, y0), y1);
            if (h == 0) in[q] = y0;
          }
        }
      } else {
#pragma unroll
      for (int q = 0; q < P; ++q) {
        for (int k = 0; k < osr; ++k) {
          cf y = __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(rx, vo + 8 * k, q * so, 2 /* nt */));
          if constexpr (MODE == 0)
            y = pk_cmul_ref(y, __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(rd, vt + 8 * k, q * so, 0)));
          if constexpr (!SYNC) pm = amax3(pm, y);
          if (k == 0) in[q] = y;
        }
      }
      }
    } else {
    // The window's samples (read once: nontemporal) through a buffer resource on the
    // wave-uniform frame base: the point offsets T q (up to 30 KB at SF12) go in the scalar
    // offset or the immediate, not in 64-bit vector adds.  Byte offsets fit 31 bits: the
    // pipeline's frames hold < 2^26 samples.
    // Alignment: a load instruction fetches T consecutive samples
    // per symbol; a window at base = A + d (A a multiple of D = min(T, 8) samples, so the
    // chunks never straddle a 128-byte line: one straddling in two cost the SF7 demod 19 %)
    // is read from A instead, and lane l plays the role lr = (l - d) mod T of the FFT: its
    // points lr + T q are the samples A + l + T q (l >= d) or A + l + T (q + 1) (l < d), so
    // the lane takes 17 loads and selects.  The roles permute the lanes of each symbol, so
    // the LDS accesses (and their banks) of every instruction are the same set.
    constexpr int D = T < 8 ? T : 8;
    constexpr bool AL = true;
    const int d = AL ? (int)(base & (D - 1)) : 0;
    lr = AL ? ((l - d) & (T - 1)) : l;
    v2f ld[P + 1];
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.iq + fu * a.frame_stride), (short)0, 0x7fffffff, 0x00020000);
    const int vo = rel + (int)(base - d + l) * 8;
    // with the caller-side dechirp's table pairs (two values per 16-byte load), issued in
    // the order the products consume them (vmcnt retires in order: a table load issued
    // after every sample would hold the first product until the last sample arrives -
    // 7 % of the SF7 demod)
    float4 dt[MODE == 0 ? P / 2 : 1];
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)a.downP, (short)0, 0x7fffffff, 0x00020000);
    const int vt = (cg + lr) * 16;
    // data windows are read once (nontemporal); the sync symbols, the grid's last blocks, with
    // the default policy: stage 2 re-reads symbols 0/1 right after this pass
    constexpr int AUX = SYNC ? 0 : 2;
#pragma unroll
    for (int pp = 0; pp < P / 2; ++pp) {
      if constexpr (MODE == 0)
        dt[pp] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, vt, pp * (N + T) * 16, 0));
#pragma unroll
      for (int q = 2 * pp; q < 2 * pp + 2; ++q)
        ld[q] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo, q * T * 8, AUX));
    }
    // (only waves holding a lane l < d: for T > 64 the symbol's first wave)
    if (AL && __builtin_amdgcn_readfirstlane(__ballot(l < d) != 0)) {
      // the 17th load: lanes l < d take window points; the others (whose load would fall up
      // to T samples past the window, possibly past the batch) re-read load 15's sample
      const bool late = l < d;
      ld[P] = __builtin_bit_cast(
          v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, late ? vo : vo - T * 8, P * T * 8, AUX));
#pragma unroll
      for (int q = 0; q < P; ++q) ld[q] = late ? ld[q + 1] : ld[q];  // ascending: ld[q + 1] not yet moved
    }
#pragma unroll
    for (int q = 0; q < P; ++q) in[q] = cf{ld[q].x, ld[q].y};
    // caller-side dechirp (e2e_chain_test.cpp:88-93) with the reference's products, the
    // window's max(|I|,|Q|) of exactly these samples (data symbols: the pre-pass covered
    // the sync windows), then the rotation
    if constexpr (MODE == 0) {
#pragma unroll
      for (int pp = 0; pp < P / 2; ++pp) {
        in[2 * pp] = pk_cmul_ref(in[2 * pp], cf{dt[pp].x, dt[pp].y});
        in[2 * pp + 1] = pk_cmul_ref(in[2 * pp + 1], cf{dt[pp].z, dt[pp].w});
      }
    }
    if constexpr (!SYNC) {
#pragma unroll
      for (int q = 0; q < P; ++q) pm = amax3(pm, in[q]);
    }
    }  // osr 1
    cf z[P], wz[P];
    {
      v2f F[P];
      spec_factors<SF>(rate, lr, F);
      spec_rotate_place<SF, HANN, FOLD>(in, z, F, a.win, lr, wz);
    }
    asm volatile("" : "+v"(pm));
    const uint64_t lk = fft_key<SF, false, true, (NTW > 0), true, false, NoHook, FOLD>(
        z, rows + (size_t)g * rowc, lr, a, nullptr, twl, nullptr, NoHook{}, nullptr, wz);
    // the symbol's best and runner-up keys over its lanes; the lane holding the best key
    // has the index (equal best keys in two lanes: a zero margin, so the symbol is
    // recomputed and overwritten)
    const uint32_t lbest = (uint32_t)lk;
    uint32_t best = lbest, sec = (uint32_t)(lk >> 32);
    spec_reduce<SF>(best, sec, pm, tid, red3);
    if (valid) {
      constexpr int NG = (G::NPASS == 2 ? P / G::RA : P / G::RB);
      constexpr int ML = G::NPASS == 2 ? G::MA_A : G::MA_B;
      const int o = (int)(best & 15u);  // ordinal u * NG + gg: bin = l + T gg + ML u
      const uint32_t idx = (uint32_t)(lr + T * (o % NG) + ML * (o / NG));
      // v_sqrt_f32: within 1 ulp, a denormal argument may give 0 (an absolute error below
      // 2^-63); the certification's E and absolute term carry it
      const float margin = __builtin_amdgcn_sqrtf(spec_key_value(best)) - __builtin_amdgcn_sqrtf(spec_key_value(sec));
      uint2* mg = reinterpret_cast<uint2*>(a.spec_marg) + f * tot + s;
      if constexpr (!SYNC) {
        if (lbest == best && a.syms) a.syms[f * a.sym_stride + (s - S0)] = (uint16_t)idx;
        if (l == 0) *mg = make_uint2(__float_as_uint(margin), __float_as_uint(pm));
      } else {
        if (lbest == best) *mg = make_uint2(__float_as_uint(margin), idx);
      }
    }
    block_sync<WL>();  // the rows (and red3) are rewritten by the next round
  };
  int64_t grp0 = blockIdx.x;
  // PF (two-pass wave-local geometries, SF 6-9): the data blocks with the next block's
  // samples requested during this one.  Nothing in the transform is a vector load - the
  // pass-1 positions come from a loop-invariant copy by lane permute, pass 1's twiddles are
  // loaded with the table pairs ahead of the prefetch, pass A's are in LDS - so no wait on
  // the current block's operands also waits for the next block's samples (vmcnt retires in
  // order).
  // PL (SF7 unwindowed, round 6): the PF loop with 16-byte sample loads.  A load instruction
  // reads one whole 128-byte line per symbol (lane l: samples A + 2 l + 16 j and the next,
  // j < 8) instead of half a line per 8-byte load (lane l: A + l + 8 q, q < 16): half the load
  // instructions and whole-line requests (an ablation with these loads and unchanged
  // arithmetic ran the pass 15 % faster).  The transform is the same radix-8 x radix-16 DIT;
  // only which residues (point index mod 16) a lane holds changes: the two residues r_h =
  // (2 l + h - d) mod 16 of its elements h (d = the window's offset in its line), instead of
  // role lr's lr and lr + 8.  Its pass-1 groups are those residues' 8-point transforms, written
  // back to their positions (rev[r] >> 3 = 4 (r & 3) + (r >> 2) at N = 128); pass A reads by
  // the lane's own index.  A late element (2 l + h < d) is point m of its residue from load
  // m + 1 (the 9th: the next window's first line, from the next lane group when contiguous).
  // Rotation factors e^{i rate (r_h + 16 m)} (spec_factors_pl); the certification's bound
  // covers them (certify_list: 36 u rmax T).
#ifndef LORA_SPEC_PAIRLD
#define LORA_SPEC_PAIRLD 1
#endif
#ifndef LORA_PL_CPOL
#define LORA_PL_CPOL 2  // nt
#endif
#ifndef LORA_SPEC_EARLY
#define LORA_SPEC_EARLY 1
#endif
  constexpr bool PL = LORA_SPEC_PAIRLD && SF == 7 && !HANN && WL && G::NPASS == 2 && !OSRN;
  if constexpr (PL) {
    static_assert(T == 8 && P == 16 && G::G1 == 2 && G::R1 == 8 && G::LOGR1 == 3 && FOLD, "SF7 geometry");
    constexpr int DL = 16;  // samples per 128-byte line
    const int tid0 = threadIdx.x;
    const int g = tid0 / T;
    const int l = tid0 % T;
    const int gi = g % SPB;
    const __attribute__((address_space(4))) FrameParams* fps =
        (const __attribute__((address_space(4))) FrameParams*)a.fp_spec;
    struct Blk {
      int64_t f;
      int s, d, cg;
      bool valid, mis, nbr;
      float rate;
      int toff;
    };
    float4 nx[P / 2 + 1];  // loads j < 8, and the 9th (late elements)
    // a block's frame bb / bpf by a reciprocal (exact while dblocks * bpf < 2^32: the
    // round-up multiplier's error stays below 1 / bpf) instead of a 64-bit division on the
    // scalar unit per block
    const bool fdiv = (uint64_t)dblocks * (uint64_t)bpf < (1ull << 32);
    const uint64_t mq = ((1ull << 32) + (uint64_t)bpf - 1) / (uint64_t)bpf;
    auto issue = [&](int64_t bb, Blk& B) {
      B.f = fdiv ? (bpf == 1 ? bb : (int64_t)(((uint64_t)(uint32_t)bb * mq) >> 32)) : bb / bpf;
      const int jl = (int)(bb - B.f * bpf) * SPB + gi;
      B.valid = jl < per;
      B.s = S0 + (B.valid ? jl : per - 1);
      B.rate = RAWM ? 0.0f : fps[B.f].rate;  // scalar loads (constant address space, uniform frame)
      B.toff = RAWM ? 0 : fps[B.f].t_off;
      int64_t base;
      sym_base(B.s, N, a.frame_len, B.toff, base, B.cg);
      if constexpr (API) B.cg = 0;
      B.d = (int)(base & (DL - 1));
      B.mis = __builtin_amdgcn_readfirstlane(__ballot(B.d != 0) != 0);
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.iq + B.f * a.frame_stride), (short)0, 0x7fffffff, 0x00020000);
      const int vo = (int)(base - B.d) * 8 + 16 * l;
#pragma unroll
      for (int j = 0; j < P / 2; ++j)
        nx[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, j * DL * 8, LORA_PL_CPOL));
      B.nbr = false;
      if (B.mis) {
        // the late elements' 9th line is the next window's first: when that window is the next
        // group's (the frame's next symbol, contiguous), taken from it by a lane permute where
        // the block is consumed; else each late element's own 8-byte load (the line's other
        // half may lie past the window, past the batch)
        int64_t bnext;
        int cgn;
        sym_base(B.s + 1, N, a.frame_len, B.toff, bnext, cgn);
        B.nbr = gi < SPB - 1 && jl + 1 < per && bnext == base + N;
        if (!B.nbr) {
          if (2 * l < B.d) {
            const v2f e0 = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo, (P / 2) * DL * 8, 2));
            nx[P / 2].x = e0.x;
            nx[P / 2].y = e0.y;
          }
          if (2 * l + 1 < B.d) {
            const v2f e1 = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo + 8, (P / 2) * DL * 8, 2));
            nx[P / 2].z = e1.x;
            nx[P / 2].w = e1.y;
          }
        }
      }
    };
    int64_t b = grp0 * BPG + wave;
    Blk nb{};
    if (b < dblocks) issue(b, nb);
    for (; b < dblocks; b += gstride * BPG, grp0 += gstride) {
      const Blk B = nb;
      float4(&ld)[P / 2 + 1] = nx;  // this block's samples, consumed in place
      const int d = B.d;
      // the residues of the lane's two elements
      int r[2];
      bool late[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int x = 2 * l + h - d;
        late[h] = x < 0;
        r[h] = x & (DL - 1);
      }
      // the table values of point (h, m) = window point r_h + 16 m (the staged doubled table,
      // any table phase)
      cf dv[MODE == 0 ? P : 1];
      if constexpr (MODE == 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const cf* dq = dtab + B.cg + r[h];
#pragma unroll
          for (int m = 0; m < P / 2; ++m) dv[h + 2 * m] = dq[DL * m];
        }
      }
      cf in[P];
      if (B.mis) {
        // the next group's first line (lane + T), before any lane moves its elements
        const int src = ((int)__lane_id() + T) & 63;
        const float4 n0 = {__shfl(ld[0].x, src, 64), __shfl(ld[0].y, src, 64), __shfl(ld[0].z, src, 64),
                           __shfl(ld[0].w, src, 64)};
        if (B.nbr) ld[P / 2] = n0;
#pragma unroll
        for (int m = 0; m < P / 2; ++m) {
          in[2 * m] = late[0] ? cf{ld[m + 1].x, ld[m + 1].y} : cf{ld[m].x, ld[m].y};
          in[2 * m + 1] = late[1] ? cf{ld[m + 1].z, ld[m + 1].w} : cf{ld[m].z, ld[m].w};
        }
      } else {
#pragma unroll
        for (int m = 0; m < P / 2; ++m) {
          in[2 * m] = cf{ld[m].x, ld[m].y};
          in[2 * m + 1] = cf{ld[m].z, ld[m].w};
        }
      }
      // the next block's samples, requested once this block's are in registers of their own:
      // before the table products with the fused dechirp (MODE 0: SF7 pass -0.8 %), after
      // the rotation otherwise (the RAW pass gained nothing there: +0.6 %)
      constexpr bool EARLY = LORA_SPEC_EARLY && MODE == 0;
      if constexpr (EARLY) {
        __builtin_amdgcn_sched_barrier(0);
        if (b + gstride * BPG < dblocks) issue(b + gstride * BPG, nb);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (MODE == 0) {
#pragma unroll
        for (int q = 0; q < P; ++q) in[q] = pk_cmul_ref(in[q], dv[q]);
      }
      float pm = 0.0f;
#pragma unroll
      for (int q = 0; q < P; ++q) pm = amax3(pm, in[q]);
      asm volatile("" : "+v"(pm));
      cf z[P], wz[P];
      {
        v2f F[P];
        spec_factors_pl(B.rate, r, F);
        spec_rotate_place<SF, false, FOLD>(in, z, F, a.win, l, wz);
      }
      asm volatile("" : "+v"(pm));
      if constexpr (!EARLY) {
        __builtin_amdgcn_sched_barrier(0);
        if (b + gstride * BPG < dblocks) issue(b + gstride * BPG, nb);
        __builtin_amdgcn_sched_barrier(0);
      }
      // the residues' pass-1 positions: rev[r] >> 3 at N = 128 (kissfft radices 4, 4, 4, 2:
      // tests/test_capi.py::test_sf7_pair_load_positions checks the identity)
      int cpre[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) cpre[h] = ((r[h] & 3) << 2) | (r[h] >> 2);
      const uint64_t lk = fft_key<SF, false, true, (NTW > 0), true, true, NoHook, FOLD>(
          z, rows + (size_t)g * rowc, l, a, nullptr, twl, cpre, NoHook{}, nullptr, wz);
      const uint32_t lbest = (uint32_t)lk;
      uint32_t best = lbest, sec = (uint32_t)(lk >> 32);
      spec_reduce<SF>(best, sec, pm, tid0, red3);
      if (B.valid) {
        constexpr int NG = P / G::RA;
        constexpr int ML = G::MA_A;
        const int o = (int)(best & 15u);
        const uint32_t idx = (uint32_t)(l + T * (o % NG) + ML * (o / NG));
        const float margin = __builtin_amdgcn_sqrtf(spec_key_value(best)) - __builtin_amdgcn_sqrtf(spec_key_value(sec));
        if (lbest == best && a.syms) a.syms[B.f * a.sym_stride + (B.s - S0)] = (uint16_t)idx;
        if (l == 0)
          reinterpret_cast<uint2*>(a.spec_marg)[B.f * tot + B.s] = make_uint2(__float_as_uint(margin), __float_as_uint(pm));
      }
      wave_sync();  // the rows are rewritten by the next round
    }
  }
  constexpr bool PF = WL && G::NPASS == 2 && !OSRN && !PL;
  if constexpr (PF) {
    constexpr int D = T < 8 ? T : 8;
    const int tid0 = threadIdx.x;
    const int g = SPW == 1 ? 0 : tid0 / T;
    const int l = tid0 % T;
    const int gi = g % SPB;
    const int lane0 = (int)(__lane_id()) - l;  // the symbol's first lane in the wave
    int cown[G::G1];  // pass-1 positions of role l
#pragma unroll
    for (int h = 0; h < G::G1; ++h) cown[h] = (int)(a.rev[l + T * h] >> G::LOGR1);
    const __attribute__((address_space(4))) FrameParams* fps =
        (const __attribute__((address_space(4))) FrameParams*)a.fp_spec;
    // the prefetched block: frame (uniform), symbol, window, alignment, samples
    struct Blk {
      int64_t f;
      int s, d, cg;
      bool valid, mis, nbr;
      float rate;
      int toff;
    };
    v2f nx[P + 1];
    auto issue = [&](int64_t bb, Blk& B) {
      B.f = bb / bpf;
      const int jl = (int)(bb - B.f * bpf) * SPB + gi;
      B.valid = jl < per;
      B.s = S0 + (B.valid ? jl : per - 1);
      B.rate = RAWM ? 0.0f : fps[B.f].rate;  // scalar loads (constant address space, uniform frame)
      B.toff = RAWM ? 0 : fps[B.f].t_off;
      int64_t base;
      sym_base(B.s, N, a.frame_len, B.toff, base, B.cg);
      if constexpr (API) B.cg = 0;
      B.d = (int)(base & (D - 1));
      B.mis = __builtin_amdgcn_readfirstlane(__ballot(B.d != 0) != 0);
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.iq + B.f * a.frame_stride), (short)0, 0x7fffffff, 0x00020000);
      const int vo = (int)(base - B.d + l) * 8;
#ifdef LORA_ABL_LD16
      // ablation (results invalid): the window's bytes in 16-byte loads, whole lines per symbol
      {
        const int vo2 = (int)(base - B.d) * 8 + 16 * l;
#pragma unroll
        for (int pp = 0; pp < P / 2; ++pp) {
          const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo2, pp * 2 * T * 8, 2));
          nx[2 * pp] = v2f{v.x, v.y};
          nx[2 * pp + 1] = v2f{v.z, v.w};
        }
      }
#else
#pragma unroll
      for (int q = 0; q < P; ++q)
        nx[q] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo, q * T * 8, 2 /* nt */));
#endif
      B.nbr = false;
      if (B.mis) {
        // a late lane's 17th point is the next window's first: when that window is the next
        // group's (the frame's next symbol, contiguous), taken from it by a lane permute
        // where the block is consumed, so the line the two windows share is fetched once
        int64_t bnext;
        int cgn;
        sym_base(B.s + 1, N, a.frame_len, B.toff, bnext, cgn);
        B.nbr = gi < SPB - 1 && jl + 1 < per && bnext == base + N;
        if (l < B.d && !B.nbr)
          nx[P] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo, P * T * 8, 2 /* nt */));
      }
    };
    int64_t b = grp0 * BPG + wave;
    Blk nb{};
    if (b < dblocks) issue(b, nb);
    for (; b < dblocks; b += gstride * BPG, grp0 += gstride) {
      const Blk B = nb;
      v2f(&ld)[P + 1] = nx;  // this block's samples, consumed in place (no copy per round)
      const int d = B.d;
      const int lr = (l - d) & (T - 1);
      // this block's table pairs and pass 1's twiddles, then the next block's samples
      float4 dt[MODE == 0 ? P / 2 : 1];
      if constexpr (MODE == 0) {
        const __amdgpu_buffer_rsrc_t rd =
            __builtin_amdgcn_make_buffer_rsrc((void*)a.downP, (short)0, 0x7fffffff, 0x00020000);
        const int vt = (B.cg + lr) * 16;
        if constexpr (DTAB) {
          // any table phase from the staged table: down[cg + lr + T q], two per ds_read2_b64
          const cf* dq = dtab + B.cg + lr;
#pragma unroll
          for (int pp = 0; pp < P / 2; ++pp) {
            const cf d0 = dq[2 * pp * T], d1 = dq[(2 * pp + 1) * T];
            dt[pp] = float4{d0.re, d0.im, d1.re, d1.im};
          }
        } else {
        // every window of the wave at table phase 0 (t_off = 0 frames): the LDS slice
        const bool cg0 = __builtin_amdgcn_readfirstlane(__ballot(B.cg != 0) == 0);
#pragma unroll
        for (int pp = 0; pp < P / 2; ++pp)
          dt[pp] = cg0 ? dtl[pp * T + lr]
                       : __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, vt, pp * (N + T) * 16, 0));
        }
      }

      // select (a misaligned window), dechirp, window max
      if (B.mis) {
        const bool late = l < d;
        // the next group's first point (lane + T), before any lane shifts its points
        const int src = ((int)__lane_id() + T) & 63;
        const v2f n0 = {__shfl(ld[0].x, src, 64), __shfl(ld[0].y, src, 64)};
        if (late && B.nbr) ld[P] = n0;
#pragma unroll
        for (int q = 0; q < P; ++q) ld[q] = late ? ld[q + 1] : ld[q];
      }
      cf in[P];
#pragma unroll
      for (int q = 0; q < P; ++q) in[q] = cf{ld[q].x, ld[q].y};
      if constexpr (MODE == 0) {
#pragma unroll
        for (int pp = 0; pp < P / 2; ++pp) {
          in[2 * pp] = pk_cmul_ref(in[2 * pp], cf{dt[pp].x, dt[pp].y});
          in[2 * pp + 1] = pk_cmul_ref(in[2 * pp + 1], cf{dt[pp].z, dt[pp].w});
        }
      }
      float pm = 0.0f;
#pragma unroll
      for (int q = 0; q < P; ++q) pm = amax3(pm, in[q]);
      asm volatile("" : "+v"(pm));
      cf z[P], wz[P];
      {
        v2f F[P];
        spec_factors<SF>(B.rate, lr, F);
        spec_rotate_place<SF, HANN, FOLD>(in, z, F, a.win, lr, wz);
      }
      asm volatile("" : "+v"(pm));
      // the next block's samples, requested once this block's are consumed (their registers
      // are free again)
      __builtin_amdgcn_sched_barrier(0);
      if (b + gstride * BPG < dblocks) issue(b + gstride * BPG, nb);
      __builtin_amdgcn_sched_barrier(0);
      // role lr's pass-1 positions from the lane that holds them (lane permute, no memory)
      int cpre[G::G1];
#pragma unroll
      for (int h = 0; h < G::G1; ++h) cpre[h] = __shfl(cown[h], lane0 + lr, 64);
      const uint64_t lk = fft_key<SF, false, true, (NTW > 0), true, true, NoHook, FOLD>(
          z, rows + (size_t)g * rowc, lr, a, nullptr, twl, cpre, NoHook{}, nullptr, wz);
      const uint32_t lbest = (uint32_t)lk;
      uint32_t best = lbest, sec = (uint32_t)(lk >> 32);
      spec_reduce<SF>(best, sec, pm, tid0, red3);
      if (B.valid) {
        constexpr int NG = P / G::RA;
        constexpr int ML = G::MA_A;
        const int o = (int)(best & 15u);
        const uint32_t idx = (uint32_t)(lr + T * (o % NG) + ML * (o / NG));
        const float margin = __builtin_amdgcn_sqrtf(spec_key_value(best)) - __builtin_amdgcn_sqrtf(spec_key_value(sec));
        if (lbest == best && a.syms) a.syms[B.f * a.sym_stride + (B.s - S0)] = (uint16_t)idx;
        if (l == 0)
          reinterpret_cast<uint2*>(a.spec_marg)[B.f * tot + B.s] = make_uint2(__float_as_uint(margin), __float_as_uint(pm));
      }
      wave_sync();  // the rows are rewritten by the next round
    }
  }
  // PF3 (three-pass geometries, SF 10-12): the same prefetching loop; the next block's
  // samples are requested at pass B, after every vector load of the transform (the pass-1
  // positions and twiddles, pass B's twiddle pairs - all older, so waiting for them never
  // waits for the prefetch).  SF 11-12: a block is the workgroup's symbol.
  constexpr bool PF3 = G::NPASS == 3 && !OSRN;
  if constexpr (PF3) {
    constexpr int D = T < 8 ? T : 8;
    const int tid0 = threadIdx.x;
    const int g = SPW == 1 ? 0 : tid0 / T;
    const int l = tid0 % T;
    const int gi = WL ? g % SPB : g;
    const __attribute__((address_space(4))) FrameParams* fps =
        (const __attribute__((address_space(4))) FrameParams*)a.fp_spec;
    struct Blk {
      int64_t f;
      int s, d, cg;
      bool valid, mis;
      float rate;
      int toff;
    };
    // pass-1 positions of role l (an aligned window's roles are the lanes themselves)
    int cown[G::G1];
#pragma unroll
    for (int h = 0; h < G::G1; ++h) cown[h] = (int)(a.rev[l + T * h] >> G::LOGR1);
    v2f nx[P + 1];
    auto issue = [&](int64_t bb, Blk& B) {
      B.f = bb / bpf;
      const int jl = (int)(bb - B.f * bpf) * SPB + gi;
      B.valid = jl < per;
      B.s = S0 + (B.valid ? jl : per - 1);
      B.rate = RAWM ? 0.0f : fps[B.f].rate;
      B.toff = RAWM ? 0 : fps[B.f].t_off;
      int64_t base;
      sym_base(B.s, N, a.frame_len, B.toff, base, B.cg);
      if constexpr (API) B.cg = 0;
      B.d = (int)(base & (D - 1));
      B.mis = __builtin_amdgcn_readfirstlane(__ballot(l < B.d) != 0);  // waves holding late lanes
      const __amdgpu_buffer_rsrc_t rx =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.iq + B.f * a.frame_stride), (short)0, 0x7fffffff, 0x00020000);
      const int vo = (int)(base - B.d + l) * 8;
#pragma unroll
      for (int q = 0; q < P; ++q)
        nx[q] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, vo, q * T * 8, 2 /* nt */));
      if (B.mis)
        nx[P] = __builtin_bit_cast(
            v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, l < B.d ? vo : vo - T * 8, P * T * 8, 2 /* nt */));
    };
    int64_t b = grp0 * BPG + (WL ? wave : 0);
    Blk nb{};
    if (b < dblocks) issue(b, nb);
    for (; b < dblocks; b += gstride * BPG, grp0 += gstride) {
      const Blk B = nb;
      v2f(&ld)[P + 1] = nx;
      const int d = B.d;
      const int lr = (l - d) & (T - 1);
      float4 dt[MODE == 0 ? P / 2 : 1];
      if constexpr (MODE == 0) {
        const __amdgpu_buffer_rsrc_t rd =
            __builtin_amdgcn_make_buffer_rsrc((void*)a.downP, (short)0, 0x7fffffff, 0x00020000);
        const int vt = (B.cg + lr) * 16;
#pragma unroll
        for (int pp = 0; pp < P / 2; ++pp)
          dt[pp] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, vt, pp * (N + T) * 16, 0));
      }
      if (B.mis) {
        const bool late = l < d;
#pragma unroll
        for (int q = 0; q < P; ++q) ld[q] = late ? ld[q + 1] : ld[q];
      }
      cf in[P];
#pragma unroll
      for (int q = 0; q < P; ++q) in[q] = cf{ld[q].x, ld[q].y};
      if constexpr (MODE == 0) {
#pragma unroll
        for (int pp = 0; pp < P / 2; ++pp) {
          in[2 * pp] = pk_cmul_ref(in[2 * pp], cf{dt[pp].x, dt[pp].y});
          in[2 * pp + 1] = pk_cmul_ref(in[2 * pp + 1], cf{dt[pp].z, dt[pp].w});
        }
      }
      float pm = 0.0f;
#pragma unroll
      for (int q = 0; q < P; ++q) pm = amax3(pm, in[q]);
      // pass B's twiddle pairs, requested once the table pairs are consumed: they have the
      // rotation and passes 1 and A to arrive
      constexpr int NTB = G::RB == 16 ? 15 : 3;
      cf wb[(P / G::RB) * NTB];
#pragma unroll
      for (int gg = 0; gg < P / G::RB; ++gg) load_tw2<G::RB, G::MA_B>(wb + gg * NTB, (lr + T * gg) % G::MA_B, a.twTB2);
      asm volatile("" : "+v"(pm));
      cf z[P], wz[P];
      {
        v2f F[P];
        spec_factors<SF>(B.rate, lr, F);
        spec_rotate_place<SF, HANN, FOLD>(in, z, F, a.win, lr, wz);
      }
      asm volatile("" : "+v"(pm));
      const int64_t bn = b + gstride * BPG;
      auto hook = [&]() {
        if (bn < dblocks) issue(bn, nb);
      };
      // role lr's pass-1 positions: the lane's own for an aligned window, else a table load
      // (issued before the prefetch, so waiting for it never waits for the next samples)
      int cpre[G::G1];
#pragma unroll
      for (int h = 0; h < G::G1; ++h) cpre[h] = d == 0 ? cown[h] : (int)(a.rev[lr + T * h] >> G::LOGR1);
      const uint64_t lk = fft_key<SF, false, true, (NTW > 0), true, true, decltype(hook), FOLD>(
          z, rows + (size_t)g * rowc, lr, a, nullptr, twl, cpre, hook, wb, wz);
      const uint32_t lbest = (uint32_t)lk;
      uint32_t best = lbest, sec = (uint32_t)(lk >> 32);
      spec_reduce<SF>(best, sec, pm, tid0, red3);
      if (B.valid) {
        constexpr int NG = P / G::RB;
        constexpr int ML = G::MA_B;
        const int o = (int)(best & 15u);
        const uint32_t idx = (uint32_t)(lr + T * (o % NG) + ML * (o / NG));
        const float margin =
            __builtin_amdgcn_sqrtf(spec_key_value(best)) - __builtin_amdgcn_sqrtf(spec_key_value(sec));
        if (lbest == best && a.syms) a.syms[B.f * a.sym_stride + (B.s - S0)] = (uint16_t)idx;
        if (l == 0)
          reinterpret_cast<uint2*>(a.spec_marg)[B.f * tot + B.s] = make_uint2(__float_as_uint(margin), __float_as_uint(pm));
      }
      block_sync<WL>();  // the rows (and red3) are rewritten by the next round
    }
  }
  // (an incremental quotient / remainder instead of the 64-bit division per round measured
  // 1 % slower: SF7 demod 0.251 vs 0.249 ms, SF12 10.03 vs 9.94 ms, four runs each)
  for (int64_t grp = grp0; grp < groups; grp += gstride) {
    const int64_t b = grp * BPG + (WL ? wave : 0);  // wave-uniform (workgroup-uniform beyond)
    if (WL && b >= blocks) break;
    if (b < dblocks) {
      const int64_t fb = b / bpf;
      run_block(std::false_type{}, b, fb, (int)(b - fb * bpf));
    } else {
      run_block(std::true_type{}, b, 0, 0);
    }
  }
}

// Offset estimate + sync symbols, one T-lane group per frame (LoRaDemod.cpp:79-135,
// 165-168, 177-192; phy.cpp:78-145, 228-237), for frames with >= 2 whole symbols.
// Per frame: for each of symbols 0,1 and osr phase t, the FFT of the (dechirped,
// normalised | raw) windowed samples, the detector tail on the winning bin (power,
// fractional index, LoRaDetector.hpp:60-71) and the phase of that bin; lane 0 keeps
// the estimator state.  Then symbols 0/1 are demodulated with the estimated offsets
// exactly as k_demod_fast does for the data symbols, giving the sync word.
// Latency-bound (a few sequential transforms per frame): occupancy matters more than
// ILP, so the register budget is capped at two waves per SIMD.
template <int SF>
struct EstGeo {
  static constexpr int T = Geo<SF>::T;
  static constexpr int BLOCK = T >= 64 ? 256 : 64;  // threads per block
  static constexpr int SPB = BLOCK / T;             // frames per block
  // symbols 0 and 1 transformed in lockstep (two LDS rows per frame)
  // (SF 7-8; SF 6 would spill)
  static constexpr bool PAIR = SF >= 7 && Geo<SF>::WAVE_LOCAL && Geo<SF>::NPASS == 2;
};

// SPEC (the speculative single-read pipeline, LEGACY osr-1 unwindowed frames, see
// lora_capi.hip): 0 = the estimate as above; 1 = pre-pass: the estimate on UNSCALED
// samples into fp_spec plus the maximum of the samples no data-symbol window covers
// (symbols 0/1 and the frame tail, one partial slot), and unless that maximum already
// exceeds 1, the sync word (fp_spec pad0; no outputs); 2 = with the maximum assembled from the demod's window partials: a frame
// that is not rescaled takes the pre-pass results as they are; any other gets the exact
// estimate, its outputs and sync word, then the certification of every data symbol the
// demod computed from unscaled samples with the pre-pass offsets: a symbol whose argmax
// margin exceeds the rounding bound keeps its index, any other is recomputed exactly here.
// One symbol s of the frame at x exactly as the reference computes it with the offsets q
// (scaled samples, glibc-faithful rotation, kissfft order; LoRaDemod.cpp:137-175,
// phy.cpp:209-237): its argmax index, on every lane of the group - the estimate kernels'
// sync symbols and the data symbols the speculative demod could not certify.  (Out of
// line it cut the SF12 pre-pass from 248 to 180 VGPRs but the calls' register saves made
// the SF12 step 0.8-1.2 ms slower at 2-4 waves per SIMD; inlined.)
template <int SF, int MODE>
__device__ __forceinline__ uint32_t exact_symbol(const KArgs& a, const cf* __restrict__ x,
                                                           const FrameParams& q, int s, cf* row, int l, int tid,
                                                           uint64_t* red) {
  using G = Geo<SF>;
  constexpr int N = G::N, P = G::P;
  constexpr bool DYN = MODE == 2;
  const int step = DYN ? a.step : N;
  const int osr = DYN ? a.osr : 1;
  const bool legacy = DYN ? a.mode != LORA_MODE_API : true;
  const bool dech = DYN ? (legacy && a.dechirp) : (MODE == 0);
  const bool hann = a.hann != 0;  // MODE 0/1: only the pipeline's frames may be windowed
  int64_t base;
  int cg;
  sym_base(s, step, a.frame_len, q.t_off, base, cg);
  const float start = q.rate * ((float)((uint32_t)s * (uint32_t)N) + (float)q.t_off / (float)osr);
  cf in[P], z[P];
  gather_points<SF>(a, x + base, l, osr, step, cg, legacy ? 1 : 2, dech, (legacy && q.scaled) ? q.scale : 1.0f, in);
  rotate_place<SF, true>(in, z, start, q.rate, hann, a.win, l);
  uint64_t key = fft_key<SF, false>(z, row, l, a);
  key = symbol_key<SF>(key, tid, red);
  block_sync<G::WAVE_LOCAL>();  // the row (and red) are rewritten by the next transform
  return key_index(key);
}

// Largest error of the hardware sine / cosine the speculative rotation uses: v_sin_f32 /
// v_cos_f32 of every fp32 x in [0, 1) lie within 1.2541e-7 of sin / cos(2 pi x) (measured
// exhaustively by tools/micro/hw_sincos_err.hip, re-checked on every GPU test run by
// test_gpu_dropin); the bound carries 2e-7 (60 % headroom).
constexpr double kHwSinCosErr = 2.0e-7;

// The certification of a frame's speculative symbols (k_est_fast<SPEC = 2>, k_cert_split):
// q the frame's exact offsets, LANES lanes per frame (li < LANES this lane's index), the
// certified sync word written, the rejected symbols listed for k_spec_fix.  Derivation of
// the bound at k_est_fast<SPEC = 2>.
template <int SF, int LANES>
__device__ __forceinline__ void certify_list(const KArgs& a, int64_t f, const FrameParams& q, bool valid, int li) {
  constexpr int N = 1 << SF;
  const FrameParams qs = a.fp_spec[f];
  const int per = a.total - 2;
  const bool same_t = qs.t_off == q.t_off;
  constexpr int T = N >= 16 ? N / 16 : 1;
  const double u = 1.0 / 16777216.0;
  const double E = (8.0 * SF + 42.0) * u;
  const double drate = fabs((double)q.rate - (double)qs.rate);
  const double rmax = fmax(fabs((double)q.rate), fabs((double)qs.rate));
  const double tabs = (double)abs(q.t_off);
  // the speculative rotation factors' error (spec_factors, spec_factors_pl): 36 u rmax T + 16 (fract's
  // rounding 2 pi 2^-25 + sqrt2 kHwSinCosErr) + 15 (2 sqrt2 u) + the keys' truncation 2^-20
  const double e_spec = 36.0 * u * rmax * T + 16.0 * (1.87e-7 + 1.4143 * kHwSinCosErr) + 2.6e-6 + 9.6e-7;
  // symbol s certified: its margin d exceeds 4 B (n1 = 2 N x the window's max(|I|,|Q|))
  auto certified = [&](double d, double wmax, int s) {
    const double n1 = 2.0 * N * wmax;
    const double L = (double)(s + 1) * N + tabs;
    const double e_ref = u * rmax * (L + 2.0 * N);
    const double B = n1 * (drate * N + e_ref + e_spec + 2.0 * E);
    return same_t && d > 4.0 * B + 0x1p-60;
  };
  const uint2* __restrict__ mg = reinterpret_cast<const uint2*>(a.spec_marg) + f * a.total;
  // the sync symbols (entries 0, 1: margin, index) on lanes 0 and 1: their windows lie in
  // [0, 2N + t_off), whose maximum the pre-pass took (a.maxbits[f] <= maxv)
  bool sync_rej = false;
  if (a.mode != LORA_MODE_API) {  // (API: the estimate kernel demodulated symbols 0/1 exactly)
    const uint2 e = mg[li < 2 ? li : 0];
    const bool ok = certified((double)__uint_as_float(e.x), (double)__uint_as_float(a.maxbits[f]), li & 1);
    const uint32_t ok1 = (uint32_t)__shfl_down((int)ok, 1, 64), i1 = (uint32_t)__shfl_down((int)e.y, 1, 64);
    if (li == 0 && valid) {
      if (ok && ok1) {
        if (a.sync) {
          const unsigned shift = a.sf > 4 ? a.sf - 4 : 0;
          a.sync[f] = (uint8_t)((((e.y >> shift) & 0x0f) << 4) | ((i1 >> shift) & 0x0f));
        }
      } else {
        sync_rej = true;
      }
    }
  }
  if (valid) {
    // the data symbols' certification tests (eight margin loads in flight per lane), then
    // the rejected symbols listed for k_spec_fix: the rounds' ballots first, one list
    // reservation per wave in the workgroup's stripe (a -10 dB batch rejects thousands of
    // symbols: per-round or per-lane atomics on one counter serialise); the last round
    // carries the sync word's entry (data symbol 0xFFFFFFFF)
    uint64_t rejbits = 0;  // bit k: symbol li + LANES k (per <= kSpecChunks T)
#pragma unroll 8
    for (int j = li, k = 0; j < per; j += LANES, ++k) {
      const uint2 v = mg[2 + j];
      if (!certified((double)__uint_as_float(v.x), (double)__uint_as_float(v.y), 2 + j)) rejbits |= 1ull << k;
    }
    const int rounds = (per + LANES - 1) / LANES;  // uniform
    unsigned total = 0;
    for (int k = 0; k <= rounds; ++k)
      total += (unsigned)__popcll(__ballot(k < rounds ? ((rejbits >> k) & 1) != 0 : sync_rej));
    if (total) {  // wave-uniform
      const int lane = (int)__lane_id();
      const int first = __builtin_ctzll(__ballot(1));
      const int stripe = (int)(blockIdx.x % kFixStripes);
      unsigned base = 0;
      if (lane == first) base = atomicAdd(a.fix_count + 16 * stripe, total);
      base = (unsigned)__shfl((int)base, first, 64);
      uint32_t* list = a.fix_list + 2 * (size_t)stripe * (size_t)a.fix_cap;
      for (int k = 0; k <= rounds; ++k) {
        const bool rej = k < rounds ? ((rejbits >> k) & 1) != 0 : sync_rej;
        const uint64_t m = __ballot(rej);
        if (rej) {
          const size_t slot = base + (unsigned)__popcll(m & ((1ull << lane) - 1));
          list[2 * slot] = (uint32_t)f;
          list[2 * slot + 1] = k < rounds ? (uint32_t)(li + LANES * k) : 0xFFFFFFFFu;
        }
        base += (unsigned)__popcll(m);
      }
    }
  }
}

// Waves per SIMD the estimate kernels' registers are budgeted for.  SF 10-12 (T >= 64 lanes
// per frame): the pipeline's pre-pass and stage 2 at 4 (osr > 1 pre-pass and SF11 stage 2
// at 3, where 4 spilled) - with the lane index opaque per transform they fit; before, the
// hoisted lane addresses took 256 VGPRs and held them at 2.  Tried and not kept: the
// pre-pass with the certified (FMA) transforms, its estimate only steering the symbol pass
// and stage 2 estimating every frame exactly - even for rescaled frames, and 0.34 ms slower
// per SF12 step for unscaled ones, whose exact pre-pass estimate stage 2 takes as it is.
constexpr int est_waves_per_eu(int SF, int MODE, int SPEC) {
  if (SF < 10) return 2;
  if (SPEC == 1) return MODE == 2 ? 3 : 4;
  if (SPEC == 2) return SF == 11 ? 3 : 4;
  return 2;
}

template <int SF, int MODE, int SPEC = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(est_waves_per_eu(SF, MODE, SPEC))))
k_est_fast(KArgs a, int64_t frames, int rowc) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P;
  constexpr int SPB = (T >= 64 ? 256 : 64) / T;  // frames per block (block = max(T, 64))
  constexpr bool DYN = MODE == 2;
  // (the speculative pipeline's stages run MODE 0/1 at osr 1 and MODE 2 for oversampled
  // LEGACY frames)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint64_t red[4];
  __shared__ FrameParams sp[SPB];
  const int tid = threadIdx.x;
  if (SPEC == 1 && blockIdx.x == 0 && tid < kFixStripes) a.fix_count[16 * tid] = 0;  // the reject list
  const int step = DYN ? a.step : N;
  const int osr = DYN ? a.osr : 1;
  const bool legacy = DYN ? a.mode != LORA_MODE_API : true;
  const bool dech = DYN ? (legacy && a.dechirp) : (MODE == 0);
  const bool hann = (DYN || SPEC != 0) ? (a.hann != 0) : false;  // the pipeline's frames may be windowed
  const int g = tid / T;
  const int l = tid % T;
  const int64_t f0 = (int64_t)blockIdx.x * SPB + g;
  const bool valid = f0 < frames;
  const int64_t f = valid ? f0 : frames - 1;
  const cf* __restrict__ x = a.iq + f * a.frame_stride;
  cf* row = reinterpret_cast<cf*>(smem) + (size_t)g * rowc;
  // LoRaDemod.cpp:59-67 max_amp from the frame's partials: the group's lanes load them
  // in parallel (one dependent load chain per lane is latency-bound)
  float maxv = 0.0f;
  if (legacy && SPEC != 1) {
    if constexpr (SPEC == 2) {
      // the pre-pass's slot (samples outside the data windows) and every data window's
      // maximum from the demod's (margin, max) pairs, eight loads in flight per lane
      maxv = __uint_as_float(a.maxbits[f]);
      const int per = a.total - 2;
      const float2* __restrict__ mg = reinterpret_cast<const float2*>(a.spec_marg) + f * a.total + 2;
#pragma unroll 8
      for (int j = l; j < per; j += T) maxv = fmaxf(maxv, mg[j].y);
    } else {
      for (int c = l; c < a.mx_bpf; c += T) maxv = fmaxf(maxv, __uint_as_float(a.maxbits[f * a.mx_bpf + c]));
    }
    maxv = __uint_as_float((uint32_t)(symbol_key<SF>((uint64_t)__float_as_uint(maxv) << 32, tid, red) >> 32));
  }
  const int scaled = maxv > 1.0f;
  const float scale = scaled ? 1.0f / maxv : 1.0f;
  if constexpr (SPEC == 2) {
    // max <= 1: no rescaling, so the pre-pass estimate and its sync word are already the
    // reference's (identical inputs and arithmetic); the symbols, rotated with the
    // hardware sine/cosine, go through the certification below like a rescaled frame's.
    if (!scaled) {
      if (l == 0 && valid) {
        const FrameParams qs = load_fp(a.fp_spec + f);
        store_fp(a.fp + f, qs);
        if (a.cfo) a.cfo[f] = qs.cfo;
        if (a.toff) a.toff[f] = qs.toff;
        if (a.max_amp) a.max_amp[f] = maxv;
      }
    }
  }
  // The frame's exact offsets: estimated below, or for an unscaled frame of the
  // speculative pipeline the pre-pass's (identical), whose symbols are then certified.
  FrameParams q;
  if (SPEC == 2 && !scaled) {
    q = a.fp_spec[f];
  } else {

    float sum_index = 0.0f, phase_diff = 0.0f, prev_phase = 0.0f;
    bool have_prev = false;
    unsigned sum_t = 0;
    cf in[P], z[P];
    float mo = 0.0f;  // SPEC == 1: max(|I|,|Q|) over symbols 0/1 (the estimate's gathers)
    constexpr bool PAIR = EstGeo<SF>::PAIR && MODE <= 1;  // MODE 2 (osr / window) would spill
    if constexpr (PAIR) {
      // symbols 0 and 1 in lockstep (fft_key2); the per-symbol bookkeeping below is the
      // same, applied in the same order (symbol 0 first)
      cf* row1 = row + (size_t)EstGeo<SF>::SPB * rowc;
      cf in1[P], z1[P];
      float bp[2] = {-1e30f, -1e30f}, bfi[2] = {0.0f, 0.0f};
      uint32_t bidx[2] = {0, 0};
      unsigned bt[2] = {0, 0};
      cf bbin[2] = {cf{0.0f, 0.0f}, cf{0.0f, 0.0f}};
      for (int t = 0; t < osr; ++t) {
        gather_points<SF>(a, x + t, l, osr, step, t, legacy ? 1 : 0, dech, scale, in);
        gather_points<SF>(a, x + (int64_t)step + t, l, osr, step, t, legacy ? 1 : 0, dech, scale, in1);
        if constexpr (SPEC == 1) {
#pragma unroll
          for (int q = 0; q < P; ++q) mo = amax3(amax3(mo, in[q]), in1[q]);
          asm volatile("" : "+v"(mo));
        }
        rotate_place<SF, false>(in, z, 0.0f, 0.0f, hann, a.win, l);
        rotate_place<SF, false>(in1, z1, 0.0f, 0.0f, hann, a.win, l);
        uint64_t key[2];
        fft_key2<SF, true>(z, z1, row, row1, l, a, key[0], key[1]);
        key[0] = group_max(key[0], T);
        key[1] = group_max(key[1], T);
        if (l == 0) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const cf* rw = s ? row1 : row;
            const uint32_t idx = key_index(key[s]);
            const uint32_t im1 = idx > 0 ? idx - 1 : N - 1, ip1 = idx < (uint32_t)N - 1 ? idx + 1 : 0;
            const cf L = rw[lds_slot<SF>((int)im1)], R = rw[lds_slot<SF>((int)ip1)],
                     B = rw[lds_slot<SF>((int)idx)];
            float pw, fi;
            detect_tail(key_value(key[s]), L, R, a.power_scale, &pw, &fi);
            if (pw > bp[s] || (legacy && pw == bp[s] && idx < bidx[s])) {
              bp[s] = pw;
              bidx[s] = idx;
              bfi[s] = fi;
              bt[s] = (unsigned)t;
              bbin[s] = B;
            }
          }
        }
        wave_sync();  // the rows are rewritten by the next phase
      }
      if (l == 0) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          sum_t += bt[s];
          sum_index += (float)bidx[s] + bfi[s];
          const float phase = lm_atan2f(bbin[s].im, bbin[s].re);
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
    }
    for (int s = 0; s < (PAIR ? 0 : 2); ++s) {
      float best_p = -1e30f, best_fi = 0.0f;
      uint32_t best_idx = 0;
      unsigned best_t = 0;
      cf best_bin = {0.0f, 0.0f};
      for (int t = 0; t < osr; ++t) {
        // the lane index opaque per transform: left visible, the compiler hoists the lane's
        // 64-bit sample, table and twiddle addresses of both symbols out of the loops and
        // keeps them live across the transforms (SF12: 256 VGPRs with spills at a 2-wave
        // budget, 147 VGPRs of spills at 4)
        int lo = l;
        asm volatile("" : "+v"(lo));
        gather_points<SF>(a, x + (int64_t)s * step + t, lo, osr, step, t, legacy ? 1 : 0, dech,
                             scale, in);
        if constexpr (SPEC == 1) {
#pragma unroll
          for (int q = 0; q < P; ++q) mo = amax3(mo, in[q]);
          asm volatile("" : "+v"(mo));
        }
        rotate_place<SF, false>(in, z, 0.0f, 0.0f, hann, a.win, lo);
        uint64_t key = fft_key<SF, true>(z, row, lo, a);
        key = symbol_key<SF>(key, tid, red);
        if (l == 0) {
          const uint32_t idx = key_index(key);
          const uint32_t im1 = idx > 0 ? idx - 1 : N - 1, ip1 = idx < (uint32_t)N - 1 ? idx + 1 : 0;
          cf L, R, B;
          if constexpr (G::NPASS == 1) {
            L = R = B = cf{0.0f, 0.0f};
#pragma unroll
            for (int u = 0; u < N; ++u) {
              if ((uint32_t)u == im1) L = z[u];
              if ((uint32_t)u == ip1) R = z[u];
              if ((uint32_t)u == idx) B = z[u];
            }
          } else {
            L = row[lds_slot<SF>((int)im1)];
            R = row[lds_slot<SF>((int)ip1)];
            B = row[lds_slot<SF>((int)idx)];
          }
          float pw, fi;
          detect_tail(key_value(key), L, R, a.power_scale, &pw, &fi);
          if (pw > best_p || (legacy && pw == best_p && idx < best_idx)) {
            best_p = pw;
            best_idx = idx;
            best_fi = fi;
            best_t = (unsigned)t;
            best_bin = B;
          }
        }
        block_sync<G::WAVE_LOCAL>();  // row is rewritten by the next transform
      }
      if (l == 0) {
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
    if (l == 0) {
      const float avg_index = sum_index / 2.0f;
      const float cfo_coarse = avg_index / (float)N;
      const float cfo_fine = (phase_diff / 1.0f) / (2.0f * PI_F * (float)N);
      const float cfo = cfo_coarse + cfo_fine;
      const float frac = avg_index - floorf(avg_index + 0.5f);
      const float avg_t = (float)sum_t / 2.0f;
      const float toff = avg_t - frac * (float)N * (float)osr;
      FrameParams qe;
      qe.cfo = cfo;
      qe.toff = toff;
      qe.t_off = (int)roundf(toff);
      qe.rate = -2.0f * PI_F * cfo / (float)N;
      qe.scale = scale;
      qe.scaled = scaled;
      qe.pad0 = qe.pad1 = 0;
      sp[g] = qe;
      if (valid) {
        if constexpr (SPEC == 1) {
          a.fp_spec[f] = qe;
        } else {
          a.fp[f] = qe;
          if (a.cfo) a.cfo[f] = cfo;
          if (a.toff) a.toff[f] = toff;
          if (a.max_amp) a.max_amp[f] = maxv;
        }
      }
    }
    block_sync<G::WAVE_LOCAL>();
    q = sp[g];
    if constexpr (SPEC == 1) {
      // The samples outside every data-symbol window of the pre-pass offsets: [0, start of
      // symbol 2's window) and [end of the last window, frame_len).  With the windows'
      // maxima (k_demod_fast<SPEC>) they make up the whole frame's maximum; a sample counted
      // twice changes nothing, so [0, 2N) comes from the estimate's own gathers (osr 1) and
      // only a positive t_off's [2N, 2N + t_off) and a tail are read here.
      const int per = a.total - 2;
      int64_t b2, bl;
      int cg;
      sym_base(2, step, a.frame_len, q.t_off, b2, cg);
      sym_base(a.total - 1, step, a.frame_len, q.t_off, bl, cg);
      const int64_t xend = bl + step;
      float m = mo;
      for (int64_t j = 2 * (int64_t)step + l; j < b2; j += T) {
        cf v = x[j];
        if (dech) v = cmul(v, a.down[j % step]);
        m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
      }
      for (int64_t j = xend + l; j < a.frame_len; j += T) {
        cf v = x[j];
        if (dech) v = cmul(v, a.down[j % step]);
        m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
      }
      const uint64_t mk = symbol_key<SF>((uint64_t)__float_as_uint(m) << 32, tid, red);
      (void)per;
      if (l == 0 && valid) a.spec_max[f] = (uint32_t)(mk >> 32);
      // The sync word waits for the exact offsets: k_est_fast<SPEC = 2> computes it.
      return;
    }
  }  // exact estimate
  // The sync symbols with the frame's offsets (LoRaDemod.cpp:137-168, 177-192; phy.cpp:
  // 228-237); the speculative pipeline certifies k_spec_demod's instead (below).
  if constexpr (SPEC == 0) {
    constexpr bool PAIR = EstGeo<SF>::PAIR && MODE <= 1;
    cf in[P], z[P];
    uint32_t sw[2];
    if constexpr (PAIR) {
      cf* row1 = row + (size_t)EstGeo<SF>::SPB * rowc;
      cf in1[P], z1[P];
      int64_t base0, base1;
      int cg0, cg1;
      sym_base(0, step, a.frame_len, q.t_off, base0, cg0);
      sym_base(1, step, a.frame_len, q.t_off, base1, cg1);
      const float st0 = q.rate * ((float)((uint32_t)0 * (uint32_t)N) + (float)q.t_off / (float)osr);
      const float st1 = q.rate * ((float)((uint32_t)1 * (uint32_t)N) + (float)q.t_off / (float)osr);
      const float sc = (legacy && q.scaled) ? q.scale : 1.0f;
      gather_points<SF>(a, x + base0, l, osr, step, cg0, legacy ? 1 : 2, dech, sc, in);
      gather_points<SF>(a, x + base1, l, osr, step, cg1, legacy ? 1 : 2, dech, sc, in1);
      rotate_place<SF, true>(in, z, st0, q.rate, hann, a.win, l);
      rotate_place<SF, true>(in1, z1, st1, q.rate, hann, a.win, l);
      uint64_t k0, k1;
      fft_key2<SF, false>(z, z1, row, row1, l, a, k0, k1);
      sw[0] = key_index(group_max(k0, T));
      sw[1] = key_index(group_max(k1, T));
    }
    if constexpr (!PAIR) {  // two straight-line calls: sw[] stays in registers
      sw[0] = exact_symbol<SF, MODE>(a, x, q, 0, row, l, tid, red);
      sw[1] = exact_symbol<SF, MODE>(a, x, q, 1, row, l, tid, red);
    }
    if (l == 0 && valid && a.sync) {
      const unsigned shift = a.sf > 4 ? a.sf - 4 : 0;
      a.sync[f] = (uint8_t)((((sw[0] >> shift) & 0x0f) << 4) | ((sw[1] >> shift) & 0x0f));
    }
  }
  if constexpr (SPEC == 2) {
    // ---- certification of the data symbols the demod computed speculatively ----
    // The demod used the pre-pass offsets qs (rate r', t_off) on the unscaled samples y;
    // the reference uses q (rate r, the same t_off, else the symbol is recomputed) on
    // fl(y * scale).  Argmax ignores the positive factor `scale` and any unit-modulus
    // factor common to the symbol's points, so compare, bin by bin, the reference's
    // spectrum with scale x the demod's for symbol s (window of N points i; A = s N + t_off,
    // L = (s + 1) N + |t_off| >= |A + i|):
    //  * the reference's phase is fl(c + fl(r i)) with c = fl(r fl(A)) the same for every
    //    point of the symbol: e^{i c} is a common factor, and what varies with i is r i up
    //    to the rounding of fl(r i) (u rmax N) and of the sum (u (|c| + rmax N) <= u rmax
    //    (L + N)): e_ref = u rmax (L + 2 N);
    //  * the demod rotates by e^{i r' i} alone (spec_factors): r0 = e^{i r' l} from
    //    fl(r' l) (u rmax T), its product by fl(1/2pi) (2 u rmax T), v_fract_f32's rounding
    //    of a negative argument (2^-25 revolutions = 1.87e-7) and v_sin/v_cos_f32
    //    (kHwSinCosErr per component); wd = e^{i r' T} the same without the first term; then
    //    15 packed products by wd, each rounding by <= 2 sqrt2 u: every factor lies within
    //    33 u rmax T + 16 (1.87e-7 + sqrt2 kHwSinCosErr) + 15 (2 sqrt2 u) of e^{i r' i} (the
    //    SF7 pair-load pass's two chains of 8, spec_factors_pl: 33.6 u rmax T, 8 and 7 terms),
    //    so e_spec = 36 u rmax T + 16 (...) + 15 (...) holds for both; the demod ranks bins by
    //    keys that truncate |X|^2 by < 16 ulp (spec_key),
    //    moving |X| by < 2^-20 |X|, which e_spec adds;
    //  * the two exact phases r i and r' i differ by at most |r - r'| N;
    //  * every other rounding (the product y * scale, the rotation product, log2 N
    //    butterfly levels with table twiddles - the packed butterflies of the certified path
    //    round each output component by <= 6 u (|f0| + .. + |f3|) per radix-4 stage, within
    //    8 u per level (bfly4) - a Hann window's product (|w| <= 1), |X|^2, the demod's
    //    v_sqrt_f32 of it - within 1 ulp - and the margin's subtraction) moves a bin by at most
    //    E sum_i |y_i| per path, E = (8 log2 N + 42) u (a stage's rounding is bounded by its
    //    partial sums <= sum_i |y_i|); v_sqrt_f32 may flush a denormal argument to 0, an
    //    absolute error below 2^-63 that the absolute term 2^-60 of the test covers.
    // With n1 = 2 N max(|re|, |im|) over the window >= sum_i |y_i|, each bin moves by less
    // than B = n1 (|r - r'| N + e_ref + e_spec + 2 E) between the paths, so a speculative
    // top bin ahead of the runner-up by d > 2 B is the reference's argmax, strictly (no
    // tie to break).  The kernel requires d > 4 B + 2^-60; a symbol that fails is listed and
    // recomputed exactly with the reference's arithmetic by k_spec_fix, the pipeline's
    // fourth launch, across the whole GPU (lora_demod_spec_recomputed() counts them).
    certify_list<SF, T>(a, f, q, valid, l);
  }
}

// The certification test of one speculative symbol s (certify_list's, derivation at
// k_est_fast<SPEC = 2>) for a frame whose exact and speculative rates are rmax apart by
// drate, |t_off| = tabs.
template <int SF>
__device__ __forceinline__ bool spec_certified(double d, double wmax, int s, double rmax, double drate, double tabs) {
  constexpr int N = 1 << SF;
  constexpr int T = N >= 16 ? N / 16 : 1;
  const double u = 1.0 / 16777216.0;
  const double E = (8.0 * SF + 42.0) * u;
  const double e_spec = 36.0 * u * rmax * T + 16.0 * (1.87e-7 + 1.4143 * kHwSinCosErr) + 2.6e-6 + 9.6e-7;
  const double n1 = 2.0 * N * wmax;
  const double L = (double)(s + 1) * N + tabs;
  const double e_ref = u * rmax * (L + 2.0 * N);
  const double B = n1 * (drate * N + e_ref + e_spec + 2.0 * E);
  return d > 4.0 * B + 0x1p-60;
}

// Appends the wave's lanes with `rej` set to the reject list as (f, code): one returning
// atomic per wave on the workgroup's stripe (wave-uniform call).
__device__ __forceinline__ void fix_list_append(const KArgs& a, bool rej, int64_t f, uint32_t code) {
  const uint64_t m = __ballot(rej);
  if (m) {  // wave-uniform
    const int lane = (int)__lane_id();
    const int first = __builtin_ctzll(m);
    const int stripe = (int)(blockIdx.x % kFixStripes);
    unsigned base = 0;
    if (lane == first) base = atomicAdd(a.fix_count + 16 * stripe, (unsigned)__popcll(m));
    base = (unsigned)__shfl((int)base, first, 64);
    if (rej) {
      const size_t slot = base + (unsigned)__popcll(m & ((1ull << lane) - 1));
      uint32_t* list = a.fix_list + 2 * (size_t)stripe * (size_t)a.fix_cap;
      list[2 * slot] = (uint32_t)f;
      list[2 * slot + 1] = code;
    }
  }
}

// k_cert_raw: the certification of LORA_MODE_RAW's symbol pass (k_spec_demod SPM 2), one
// thread per symbol: no offsets, no rotation (its factors are exactly 1), no rescaling, so
// only the transforms' rounding bounds the argmax margin (spec_certified with rate 0); the
// rejected symbols are listed for k_spec_fix.
template <int SF>
__global__ void __launch_bounds__(256) k_cert_raw(KArgs a, int64_t frames) {
  const int tot = a.total;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = i < frames * tot;
  const int64_t f = valid ? i / tot : 0;
  const int s = valid ? (int)(i - f * tot) : 0;
  bool rej = false;
  if (valid) {
    const uint2 e = reinterpret_cast<const uint2*>(a.spec_marg)[f * tot + s];
    rej = !spec_certified<SF>((double)__uint_as_float(e.x), (double)__uint_as_float(e.y), s, 0.0, 0.0, 0.0);
  }
  fix_list_append(a, rej, f, (uint32_t)s);
}

// k_spec_fix: the pipeline's fourth launch.  Every data symbol the certification
// rejected (k_est_fast<SPEC = 2>'s list: frame, data symbol) recomputed exactly with the
// frame's exact offsets a.fp[f] (LoRaDemod.cpp:137-175), and every rejected sync word
// (data symbol 0xFFFFFFFF: symbols 0 and 1, LoRaDemod.cpp:177-192), one T-lane group per
// entry, the
// list spread over the whole grid - a frame with many rejected symbols no longer holds its
// certify workgroup while the others idle.  Entry i goes to workgroup i % grid, so a short
// list still spreads over every CU (slot g of round r: i = blockIdx.x + grid (r SPW + g)).
template <int SF, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
k_spec_fix(KArgs a, int rowc, int64_t grid) {
  using G = Geo<SF>;
  constexpr int T = G::T, SPW = G::SPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint64_t red[4];
  const int tid = threadIdx.x;
  const int g = SPW == 1 ? 0 : tid / T;
  const int l = tid % T;
  // the stripes' counts (every lane loads them: 16 scalar-uniform loads) and their sum
  int64_t count = 0;
  unsigned cnt[kFixStripes];
#pragma unroll
  for (int t = 0; t < kFixStripes; ++t) {
    cnt[t] = __builtin_nontemporal_load(a.fix_count + 16 * t);
    count += cnt[t];
  }
  if (blockIdx.x == 0 && tid == 0 && count > 0) atomicAdd(a.spec_fix, (unsigned)count);
  cf* row = reinterpret_cast<cf*>(smem) + (size_t)g * rowc;
  for (int64_t r0 = 0; (int64_t)blockIdx.x + grid * r0 < count; r0 += SPW) {  // workgroup-uniform
    const int64_t i = (int64_t)blockIdx.x + grid * (r0 + g);
    const bool valid = i < count;
    int64_t k = valid ? i : count - 1;  // spare slots mirror the last entry
    // entry k of the concatenated stripes
    int t = 0;
#pragma unroll
    for (int u = 0; u < kFixStripes - 1; ++u)
      if (t == u && k >= (int64_t)cnt[u]) {
        k -= cnt[u];
        ++t;
      }
    const uint32_t* list = a.fix_list + 2 * (size_t)t * (size_t)a.fix_cap;
    const int64_t f = list[2 * k];
    const uint32_t j = list[2 * k + 1];
    const bool sync = j == 0xFFFFFFFFu;  // the sync word: symbols 0 and 1
    const FrameParams q = a.fp[f];
    const cf* __restrict__ x = a.iq + f * a.frame_stride;
    // the lane index opaque per entry (k_est_fast: no lane addresses hoisted out of the loop)
    int lo = l;
    asm volatile("" : "+v"(lo));
    // (LORA_MODE_RAW: entry j is the frame's symbol j itself, every symbol an output)
    const int js = (a.mode == LORA_MODE_RAW ? 0 : 2) + (int)j;
    const uint32_t i0 = exact_symbol<SF, MODE>(a, x, q, sync ? 0 : js, row, lo, tid, red);
    // a second transform when any group of the workgroup holds a sync entry (uniform, so
    // the transform's barriers match); the others repeat theirs
    const bool any_sync = G::WAVE_LOCAL ? __any(sync) : __syncthreads_or(sync);
    uint32_t i1 = 0;
    if (any_sync) i1 = exact_symbol<SF, MODE>(a, x, q, sync ? 1 : js, row, lo, tid, red);
    if (l == 0 && valid) {
      if (!sync) {
        if (a.syms) a.syms[f * a.sym_stride + j] = (uint16_t)i0;
      } else if (a.sync) {
        const unsigned shift = a.sf > 4 ? a.sf - 4 : 0;
        a.sync[f] = (uint8_t)((((i0 >> shift) & 0x0f) << 4) | ((i1 >> shift) & 0x0f));
      }
    }
  }
}

template <int SF>
int row_complex() {
  return lds_row<SF>();
}

// ---- the speculative pipeline's estimate kernels, one lane group per symbol -----------
// k_est_split<SF, MODE>: stage 0 (the pre-pass) of the pipeline for LEGACY osr-1
// unwindowed frames at SF 6-9 (2T <= 64 lanes per frame: a wave holds 64 / 2T frames).
// The work and the arithmetic are k_est_fast<SF, MODE, 1>'s; the layout differs: symbols
// 0 and 1 of a frame go to two lane groups side by side (the offset estimate's two
// transforms and detector tails, then the two sync symbols, run concurrently on different
// lanes instead of one after the other in one group).  Twice the waves with half the
// registers each: the pre-pass is a latency-bound chain per frame (SF7: 13.7 vs 15-18 us).
// The same split of stage 2 (exact estimate + certification) measured slower - 47.7 vs
// 28-35 us, its certification state needs the registers - and was removed.
template <int SF, int MODE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4)))
k_est_split(KArgs a, int64_t frames, int rowc) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P;
  constexpr int FPW = 64 / (2 * T);  // frames per wave (= block)
  static_assert(2 * T <= 64 && P == 16, "SF 6-9");
  constexpr bool dech = MODE == 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ FrameParams sp[FPW];
  __shared__ float tail[FPW][2][4];  // per frame and symbol: index, fractional index, phase, -
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid < kFixStripes) a.fix_count[16 * tid] = 0;  // the certification's reject list
  const int g2 = tid / T;     // lane group: frame slot fg, symbol sym
  const int fg = g2 >> 1;
  const int sym = g2 & 1;
  const int l = tid % T;      // lane within the group
  const int l2 = tid % (2 * T);  // lane within the frame's two groups
  const int64_t f0 = (int64_t)blockIdx.x * FPW + fg;
  const bool valid = f0 < frames;
  const int64_t f = valid ? f0 : frames - 1;
  const cf* __restrict__ x = a.iq + f * a.frame_stride;
  cf* row = reinterpret_cast<cf*>(smem) + (size_t)g2 * rowc;
  // reduce over the frame's 2T lanes (the two groups of a frame are adjacent)
  auto frame_max = [&](float v) {
#pragma unroll
    for (int o = T; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
  };
  // LoRaDemod.cpp:59-77 normalises by the frame's maximum, known only after the symbol
  // pass.  The pre-pass guesses it: the maximum over symbols 0/1, which for a frame of
  // constant envelope is the frame's (every noiseless SF7 frame dechirps to 1 + 2^-23 in
  // both sync windows).  Its estimate is computed on the samples normalised by that guess
  // (unscaled when the guess is <= 1), exactly as the reference would with that maximum;
  // stage 2 takes it as the exact estimate when the frame's maximum gives the same scale
  // (k_cert_split), and the symbol pass's speculation is unaffected either way.
  FrameParams q;
  {
    // LoRaDemod.cpp:79-123 (osr 1: one phase per symbol) for symbol `sym` of the frame
    cf in[P], z[P];
    gather_points<SF>(a, x + (int64_t)sym * N, l, 1, N, 0, 1, dech, 1.0f, in);
    float mo = 0.0f;  // max(|I|,|Q|) over symbols 0/1 (this group's gathers)
#pragma unroll
    for (int k = 0; k < P; ++k) mo = amax3(mo, in[k]);
    asm volatile("" : "+v"(mo));
    const float m01 = frame_max(mo);
    const int scaled = m01 > 1.0f;
    const float scale = scaled ? 1.0f / m01 : 1.0f;
    if (scaled) {
#pragma unroll
      for (int k = 0; k < P; ++k) in[k] = cscale(in[k], scale);
    }
    rotate_place<SF, false>(in, z, 0.0f, 0.0f, a.hann != 0, a.win, l);
    uint64_t key = fft_key<SF, true>(z, row, l, a);
    key = group_max(key, T);
    if (l == 0) {
      // LoRaDetector.hpp:60-71 tail on the winning bin, and arg(bin) (LoRaDemod.cpp:124)
      const uint32_t idx = key_index(key);
      const uint32_t im1 = idx > 0 ? idx - 1 : N - 1, ip1 = idx < (uint32_t)N - 1 ? idx + 1 : 0;
      const cf L = row[lds_slot<SF>((int)im1)], R = row[lds_slot<SF>((int)ip1)], B = row[lds_slot<SF>((int)idx)];
      // best over the (single) osr phase from best_p = -1e30 (LoRaDemod.cpp:86-101):
      // taken exactly when |X|^2 > 0 (detect_findex)
      const float fi = detect_findex(key_value(key), L, R);
      const bool take = key_value(key) > 0.0f;
      tail[fg][sym][0] = take ? (float)idx : 0.0f;
      tail[fg][sym][1] = take ? fi : 0.0f;
      tail[fg][sym][2] = lm_atan2f(take ? B.im : 0.0f, take ? B.re : 0.0f);
    }
    wave_sync();
    if (l2 == 0) {
      // LoRaDemod.cpp:105-135 in the reference's order: symbol 0's terms, then symbol 1's
      float sum_index = 0.0f, phase_diff = 0.0f;
      sum_index += tail[fg][0][0] + tail[fg][0][1];
      sum_index += tail[fg][1][0] + tail[fg][1][1];
      float d = tail[fg][1][2] - tail[fg][0][2];
      while (d > PI_F) d -= 2.0f * PI_F;
      while (d < -PI_F) d += 2.0f * PI_F;
      phase_diff += d;
      const float avg_index = sum_index / 2.0f;
      const float cfo_coarse = avg_index / (float)N;
      const float cfo_fine = (phase_diff / 1.0f) / (2.0f * PI_F * (float)N);
      const float cfo = cfo_coarse + cfo_fine;
      const float frac = avg_index - floorf(avg_index + 0.5f);
      const float avg_t = (float)0u / 2.0f;
      const float toff = avg_t - frac * (float)N * 1.0f;
      FrameParams qe;
      qe.cfo = cfo;
      qe.toff = toff;
      qe.t_off = (int)roundf(toff);
      qe.rate = -2.0f * PI_F * cfo / (float)N;
      qe.scale = scale;
      qe.scaled = scaled;
      qe.pad0 = qe.pad1 = 0;
      sp[fg] = qe;
      if (valid) a.fp_spec[f] = qe;
    }
    wave_sync();
    q = sp[fg];
    {
      // the samples outside every data-symbol window of these offsets: [0, 2N) came with
      // the gathers above; a positive t_off's [2N, 2N + t_off) and the frame's tail here
      int64_t b2, bl;
      int cg;
      sym_base(2, N, a.frame_len, q.t_off, b2, cg);
      sym_base(a.total - 1, N, a.frame_len, q.t_off, bl, cg);
      const int64_t xend = bl + N;
      float m = mo;
      for (int64_t j = 2 * (int64_t)N + l2; j < b2; j += 2 * T) {
        cf v = x[j];
        if (dech) v = cmul(v, a.down[j % N]);
        m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
      }
      for (int64_t j = xend + l2; j < a.frame_len; j += 2 * T) {
        cf v = x[j];
        if (dech) v = cmul(v, a.down[j % N]);
        m = fmaxf(m, fmaxf(fabsf(v.re), fabsf(v.im)));
      }
      m = frame_max(m);
      if (l2 == 0 && valid) a.spec_max[f] = __float_as_uint(m);
      // the sync word waits for the exact offsets (k_est_fast<SPEC = 2>)
    }
  }
}

// k_cert_split<SF, MODE>: stage 2 of the pipeline (k_est_fast<SF, MODE, 2>'s work) for SF
// 6-9 in k_est_split's layout: symbols 0 and 1 of a frame on two lane groups side by side.
// Per frame: the maximum assembled from the pre-pass slot and the data windows' maxima,
// the exact estimate on the normalised samples (LoRaDemod.cpp:59-135) - the pre-pass's
// when its guessed scale is the frame's (no samples read), else recomputed - the outputs,
// then the certification of every speculative symbol over the frame's 2T lanes
// (certify_list).
template <int SF, int MODE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4)))
k_cert_split(KArgs a, int64_t frames, int rowc) {
  using G = Geo<SF>;
  constexpr int N = G::N, T = G::T, P = G::P;
  constexpr int FPW = 64 / (2 * T);  // frames per wave (= block)
  static_assert(2 * T <= 64 && P == 16, "SF 6-9");
  constexpr bool dech = MODE == 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ FrameParams sp[FPW];
  __shared__ float tail[FPW][2][4];  // per frame and symbol: index, fractional index, phase, -
  const int tid = threadIdx.x;
  const int g2 = tid / T;  // lane group: frame slot fg, symbol sym
  const int fg = g2 >> 1;
  const int sym = g2 & 1;
  const int l = tid % T;          // lane within the group
  const int l2 = tid % (2 * T);   // lane within the frame's two groups
  const int64_t f0 = (int64_t)blockIdx.x * FPW + fg;
  const bool valid = f0 < frames;
  const int64_t f = valid ? f0 : frames - 1;
  const cf* __restrict__ x = a.iq + f * a.frame_stride;
  cf* row = reinterpret_cast<cf*>(smem) + (size_t)g2 * rowc;
  const int per = a.total - 2;
  // LoRaDemod.cpp:59-67 the frame's maximum: the pre-pass's slot (the samples outside the
  // data windows) and each data window's, over the frame's 2T lanes
  const FrameParams qg = load_fp(a.fp_spec + f);
  float maxv = l2 == 0 ? __uint_as_float(a.maxbits[f]) : 0.0f;
  {
    const float2* __restrict__ mg = reinterpret_cast<const float2*>(a.spec_marg) + f * a.total + 2;
#pragma unroll 4
    for (int j = l2; j < per; j += 2 * T) maxv = fmaxf(maxv, mg[j].y);
#pragma unroll
    for (int o = T; o > 0; o >>= 1) maxv = fmaxf(maxv, __shfl_xor(maxv, o, 64));
  }
  const int scaled = maxv > 1.0f;
  const float scale = scaled ? 1.0f / maxv : 1.0f;
  // A frame whose maximum gives the scale the pre-pass guessed (no rescaling either way, or
  // the same 1/max) has the pre-pass estimate as its exact one: identical inputs and
  // arithmetic.  A wave of such frames takes it as it is (and reads no samples); any other
  // computes the exact estimate for all its frames (a guessed frame's equals the pre-pass's).
  const bool guessed = scaled ? (qg.scaled != 0 && qg.scale == scale) : qg.scaled == 0;
  if (__builtin_amdgcn_readfirstlane(__ballot(!guessed) == 0)) {
    if (l2 == 0) {
      store_fp(sp + fg, qg);
      if (valid) {
        store_fp(a.fp + f, qg);
        if (a.cfo) a.cfo[f] = qg.cfo;
        if (a.toff) a.toff[f] = qg.toff;
        if (a.max_amp) a.max_amp[f] = maxv;
      }
    }
  } else {
    {
      // the group's symbol, dechirped (e2e_chain_test.cpp:88-93), then normalised
      // (LoRaDemod.cpp:68-77, gather_points' order)
      cf in[P], z[P];
      gather_points<SF>(a, x + (int64_t)sym * N, l, 1, N, 0, 1, dech, 1.0f, in);
      if (scaled) {
#pragma unroll
        for (int q = 0; q < P; ++q) in[q] = cscale(in[q], scale);
      }
      // LoRaDemod.cpp:79-123 (osr 1: one phase per symbol) for symbol `sym` of the frame
      rotate_place<SF, false>(in, z, 0.0f, 0.0f, a.hann != 0, a.win, l);
      uint64_t key = fft_key<SF, true>(z, row, l, a);
      key = group_max(key, T);
      if (l == 0) {
        // LoRaDetector.hpp:60-71 tail on the winning bin, and arg(bin) (LoRaDemod.cpp:124)
        const uint32_t idx = key_index(key);
        const uint32_t im1 = idx > 0 ? idx - 1 : N - 1, ip1 = idx < (uint32_t)N - 1 ? idx + 1 : 0;
        const cf L = row[lds_slot<SF>((int)im1)], R = row[lds_slot<SF>((int)ip1)], B = row[lds_slot<SF>((int)idx)];
        // best over the (single) osr phase from best_p = -1e30 (LoRaDemod.cpp:86-101):
        // taken exactly when |X|^2 > 0 (detect_findex)
        const float fi = detect_findex(key_value(key), L, R);
        const bool take = key_value(key) > 0.0f;
        tail[fg][sym][0] = take ? (float)idx : 0.0f;
        tail[fg][sym][1] = take ? fi : 0.0f;
        tail[fg][sym][2] = lm_atan2f(take ? B.im : 0.0f, take ? B.re : 0.0f);
      }
      wave_sync();
    }
    if (l2 == 0) {
      // LoRaDemod.cpp:105-135 in the reference's order: symbol 0's terms, then symbol 1's
      float sum_index = 0.0f, phase_diff = 0.0f;
      sum_index += tail[fg][0][0] + tail[fg][0][1];
      sum_index += tail[fg][1][0] + tail[fg][1][1];
      float d = tail[fg][1][2] - tail[fg][0][2];
      while (d > PI_F) d -= 2.0f * PI_F;
      while (d < -PI_F) d += 2.0f * PI_F;
      phase_diff += d;
      const float avg_index = sum_index / 2.0f;
      const float cfo_coarse = avg_index / (float)N;
      const float cfo_fine = (phase_diff / 1.0f) / (2.0f * PI_F * (float)N);
      const float cfo = cfo_coarse + cfo_fine;
      const float frac = avg_index - floorf(avg_index + 0.5f);
      const float avg_t = (float)0u / 2.0f;
      const float toff = avg_t - frac * (float)N * 1.0f;
      FrameParams qe;
      qe.cfo = cfo;
      qe.toff = toff;
      qe.t_off = (int)roundf(toff);
      qe.rate = -2.0f * PI_F * cfo / (float)N;
      qe.scale = scale;
      qe.scaled = scaled;
      qe.pad0 = qe.pad1 = 0;
      sp[fg] = qe;
      if (valid) {
        a.fp[f] = qe;
        if (a.cfo) a.cfo[f] = cfo;
        if (a.toff) a.toff[f] = toff;
        if (a.max_amp) a.max_amp[f] = maxv;
      }
    }
  }
  wave_sync();
  const FrameParams q = sp[fg];
  certify_list<SF, 2 * T>(a, f, q, valid, l2);
}

template <int SF, int MODE>
bool launch_est_split(const KArgs& a, int64_t frames, hipStream_t st) {
  using G = Geo<SF>;
  constexpr int FPW = 64 / (2 * G::T);
  const int rowc = row_complex<SF>();
  const size_t lds = sizeof(cf) * (size_t)(2 * FPW) * rowc;
  const int64_t grid = (frames + FPW - 1) / FPW;
  launch(k_est_split<SF, MODE>, dim3((unsigned)grid), dim3(64), lds, st, a, frames, rowc);
  return true;
}


template <int SF, int MODE>
bool launch_cert_split(const KArgs& a, int64_t frames, hipStream_t st) {
  using G = Geo<SF>;
  constexpr int FPW = 64 / (2 * G::T);
  const int rowc = row_complex<SF>();
  const size_t lds = sizeof(cf) * (size_t)(2 * FPW) * rowc;
  const int64_t grid = (frames + FPW - 1) / FPW;
  launch(k_cert_split<SF, MODE>, dim3((unsigned)grid), dim3(64), lds, st, a, frames, rowc);
  return true;
}

template <int SF, int MODE, int SPEC = 0>
bool launch_est_mode(const KArgs& a, int64_t frames, hipStream_t st) {
  using G = Geo<SF>;
  constexpr int T = G::T;
  constexpr int BLOCK = T >= 64 ? 256 : 64;
  constexpr int SPB = BLOCK / T;
  const int rowc = row_complex<SF>();
  const size_t lds = G::NPASS == 1 ? 16 : sizeof(cf) * (size_t)SPB * rowc * (EstGeo<SF>::PAIR && MODE <= 1 ? 2 : 1);
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_est_fast<SF, MODE, SPEC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return false;
  const int64_t grid = (frames + SPB - 1) / SPB;
  launch(k_est_fast<SF, MODE, SPEC>, dim3((unsigned)grid), dim3(BLOCK), lds, st, a, frames, rowc);
  return true;
}

template <int SF>
bool launch_est_sf(const KArgs& a, int64_t frames, hipStream_t st) {
  const bool simple = a.mode == LORA_MODE_LEGACY && a.osr == 1 && !a.hann;
  if (simple && a.dechirp) return launch_est_mode<SF, 0>(a, frames, st);
  if (simple) return launch_est_mode<SF, 1>(a, frames, st);
  return launch_est_mode<SF, 2>(a, frames, st);
}

template <int SF, int MODE, bool FAST = false, bool SPEC = false>
bool launch_mode(const KArgs& a, int s0, int64_t work, hipStream_t st) {
  using G = Geo<SF>;
  const int rowc = row_complex<SF>();
  const size_t lds = G::NPASS == 1 ? 16 : sizeof(cf) * ((size_t)G::SPW * rowc + demod_twl_entries<SF, SPEC>());
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_demod_fast<SF, MODE, FAST, SPEC>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return false;
  const int64_t grid = (work + G::SPW - 1) / G::SPW;
  launch(k_demod_fast<SF, MODE, FAST, SPEC>, dim3((unsigned)grid), dim3(256), lds, st, a, s0, work,
                     rowc);
  return true;
}

constexpr int kSpecWgPerCu = 4;
// Persistent grid of the speculative demod: kSpecWgPerCu workgroups per CU (the LDS rows
// allow four at every SF), or one per group when there are fewer groups.
int device_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

template <int SF, int MODE, bool HANN, int OSRV, int SPM = 0>
bool launch_spec_demod_w(const KArgs& a, int64_t frames, hipStream_t st) {
  using G = Geo<SF>;
  const int rowc = row_complex<SF>();
  const size_t lds = spec_lds_bytes<SF>();
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_spec_demod<SF, MODE, HANN, OSRV, SPM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return false;
  // the kernel's blocks: SPB symbols of one frame (see k_spec_demod), BPG per workgroup round
  constexpr int SPB = G::WAVE_LOCAL ? 64 / G::T : G::SPW, BPG = G::WAVE_LOCAL ? 4 : 1;
  const int per = a.total - (SPM == 2 ? 0 : 2);
  const int64_t blocks = frames * (int64_t)((per + SPB - 1) / SPB) + (SPM != 0 ? 0 : (2 * frames + SPB - 1) / SPB);
  const int64_t groups = (blocks + BPG - 1) / BPG;
  // persistent: the wave-local geometries, and every prefetching one (PF3: SF 10-12)
  const bool persist = G::WAVE_LOCAL || (G::NPASS == 3 && a.osr == 1);
  const int64_t cap = persist ? (int64_t)device_cus() * kSpecWgPerCu : groups;
  const int64_t grid = groups < cap ? groups : cap;
  launch(k_spec_demod<SF, MODE, HANN, OSRV, SPM>, dim3((unsigned)grid), dim3(256), lds, st, a, frames, rowc, grid);
  return true;
}
// the Hann window (LoRaDemod.cpp:158-160) and oversampling as instantiations of their own:
// the unwindowed osr-1 kernels keep no per-point branch
template <int SF, int MODE>
bool launch_spec_demod(const KArgs& a, int64_t frames, hipStream_t st) {
  if (a.osr > 1) {
    if (a.hann) return launch_spec_demod_w<SF, MODE, true, 0>(a, frames, st);
    if (a.osr == 2) return launch_spec_demod_w<SF, MODE, false, 2>(a, frames, st);
    if (a.osr == 4) return launch_spec_demod_w<SF, MODE, false, 4>(a, frames, st);
    return launch_spec_demod_w<SF, MODE, false, 0>(a, frames, st);
  }
  return a.hann ? launch_spec_demod_w<SF, MODE, true, 1>(a, frames, st)
                : launch_spec_demod_w<SF, MODE, false, 1>(a, frames, st);
}

// k_spec_fix's grid: one workgroup per CU (or fewer when the frames hold fewer data
// symbols); it reads the list's length on the device, so the launch does not wait for it.
template <int SF, int MODE>
bool launch_spec_fix(const KArgs& a, int64_t frames, hipStream_t st) {
  using G = Geo<SF>;
  const int rowc = row_complex<SF>();
  const size_t lds = sizeof(cf) * (size_t)G::SPW * rowc;
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_spec_fix<SF, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return false;
  const int64_t most = (frames * (int64_t)(a.total - 1) + G::SPW - 1) / G::SPW;
  const int64_t cap = (int64_t)device_cus();  // (one per CU: an empty list costs a smaller ramp)
  const int64_t grid = std::max<int64_t>(1, std::min(most, cap));
  launch(k_spec_fix<SF, MODE>, dim3((unsigned)grid), dim3(256), lds, st, a, rowc, grid);
  return true;
}

// The speculative pipeline's four launches for SF 6-12, MODE 0/1 (see lora_capi.hip).
template <int SF>
bool launch_spec_sf(const KArgs& a, int64_t frames, int stage, hipStream_t st) {
  if constexpr (SF < 6) {
    return false;
  } else {
    if (a.mode == LORA_MODE_RAW) {
      // the detector alone (osr 1, SF 6-9: at SF 10-12 this instantiation spills): the symbol
      // pass over every symbol, its certification, the recompute (the frame parameters are
      // zero: no offsets, no rescaling)
      if constexpr (SF > 9) {
        return false;
      } else {
        if (stage == 1) {
          if (a.hann)
            return a.dechirp ? launch_spec_demod_w<SF, 0, true, 1, 2>(a, frames, st)
                             : launch_spec_demod_w<SF, 1, true, 1, 2>(a, frames, st);
          return a.dechirp ? launch_spec_demod_w<SF, 0, false, 1, 2>(a, frames, st)
                           : launch_spec_demod_w<SF, 1, false, 1, 2>(a, frames, st);
        }
        if (stage == 2) {
          const int64_t n = frames * (int64_t)a.total;
          launch(k_cert_raw<SF>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, frames);
          return true;
        }
        if (stage == 3) return launch_spec_fix<SF, 2>(a, frames, st);
        return false;
      }
    }
    if (a.mode == LORA_MODE_API) {
      // lora_phy::demodulate (osr 1): the exact estimate with the sync word (the three-launch
      // path's kernel), the symbol pass with the exact offsets (down-chirp from table phase
      // 0, no sync blocks), the certification with no rate difference, the recompute
      if (stage == 0) return launch_est_mode<SF, 2, 0>(a, frames, st);
      if (stage == 1)
        return a.hann ? launch_spec_demod_w<SF, 0, true, 1, 1>(a, frames, st)
                      : launch_spec_demod_w<SF, 0, false, 1, 1>(a, frames, st);
      if (stage == 2) return launch_est_mode<SF, 2, 2>(a, frames, st);
      return launch_spec_fix<SF, 2>(a, frames, st);
    }
    if (a.osr > 1) {  // oversampled frames: the estimate stages at run-time osr (MODE 2)
      if (stage == 0) return launch_est_mode<SF, 2, 1>(a, frames, st);
      if (stage == 1)
        return a.dechirp ? launch_spec_demod<SF, 0>(a, frames, st) : launch_spec_demod<SF, 1>(a, frames, st);
      if (stage == 2) return launch_est_mode<SF, 2, 2>(a, frames, st);
      return launch_spec_fix<SF, 2>(a, frames, st);
    }
    if constexpr (SF <= 9) {
      if (stage == 0) return a.dechirp ? launch_est_split<SF, 0>(a, frames, st) : launch_est_split<SF, 1>(a, frames, st);
      if (stage == 2)
        return a.dechirp ? launch_cert_split<SF, 0>(a, frames, st) : launch_cert_split<SF, 1>(a, frames, st);
    }
    if (stage == 3) return a.dechirp ? launch_spec_fix<SF, 0>(a, frames, st) : launch_spec_fix<SF, 1>(a, frames, st);
    if (stage == 0) return a.dechirp ? launch_est_mode<SF, 0, 1>(a, frames, st) : launch_est_mode<SF, 1, 1>(a, frames, st);
    if (stage == 1)
      return a.dechirp ? launch_spec_demod<SF, 0>(a, frames, st) : launch_spec_demod<SF, 1>(a, frames, st);
    return a.dechirp ? launch_est_mode<SF, 0, 2>(a, frames, st) : launch_est_mode<SF, 1, 2>(a, frames, st);
  }
}

template <int SF>
bool launch_sf(const KArgs& a, int s0, int64_t work, hipStream_t st) {
  const bool simple = a.mode == LORA_MODE_LEGACY && a.osr == 1 && !a.hann;
  if (a.mode == LORA_MODE_RAW) return launch_mode<SF, 3>(a, s0, work, st);
  if (a.fast_rot) {  // LORA_PRECISION_FAST (include/lora_mi355x.h)
    if (simple && a.dechirp) return launch_mode<SF, 0, true>(a, s0, work, st);
    if (simple) return launch_mode<SF, 1, true>(a, s0, work, st);
    return launch_mode<SF, 2, true>(a, s0, work, st);
  }
  if (simple && a.dechirp) return launch_mode<SF, 0>(a, s0, work, st);
  if (simple) return launch_mode<SF, 1>(a, s0, work, st);
  return launch_mode<SF, 2>(a, s0, work, st);
}

}  // namespace


bool launch_spec(const KArgs& a, int64_t frames, int stage, hipStream_t st) {
  switch (a.sf) {
    case 6: return launch_spec_sf<6>(a, frames, stage, st);
    case 7: return launch_spec_sf<7>(a, frames, stage, st);
    case 8: return launch_spec_sf<8>(a, frames, stage, st);
    case 9: return launch_spec_sf<9>(a, frames, stage, st);
    case 10: return launch_spec_sf<10>(a, frames, stage, st);
    case 11: return launch_spec_sf<11>(a, frames, stage, st);
    case 12: return launch_spec_sf<12>(a, frames, stage, st);
    default: return false;
  }
}

bool launch_est_fast(const KArgs& a, int64_t frames, hipStream_t st) {
  if (a.total < 2 || a.est_only || a.mode == LORA_MODE_RAW) return false;
  switch (a.sf) {
    case 2: return launch_est_sf<2>(a, frames, st);
    case 3: return launch_est_sf<3>(a, frames, st);
    case 4: return launch_est_sf<4>(a, frames, st);
    case 5: return launch_est_sf<5>(a, frames, st);
    case 6: return launch_est_sf<6>(a, frames, st);
    case 7: return launch_est_sf<7>(a, frames, st);
    case 8: return launch_est_sf<8>(a, frames, st);
    case 9: return launch_est_sf<9>(a, frames, st);
    case 10: return launch_est_sf<10>(a, frames, st);
    case 11: return launch_est_sf<11>(a, frames, st);
    case 12: return launch_est_sf<12>(a, frames, st);
    default: return false;
  }
}

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
