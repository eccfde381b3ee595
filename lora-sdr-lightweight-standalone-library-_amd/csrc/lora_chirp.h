// lora_chirp.h — the frequency sequence of genChirp (ChirpGenerator.hpp:105-132) in closed
// form, for the modulator's frame kernel (lora_capi.hip k_mod_frame) and its host check
// (tests/native/chirp_seg_check.cpp).  Host and device code.
//
// genChirp's per-sample recurrence is  f = fl(f + fStep); if (f > fMax) f = fl(f - span);
// phase = fl(phase + f)  (all fp32).  The frequency part does not depend on the phase, and
// it is piecewise arithmetic: while |f| stays in one binade [2^e, 2^(e+1)) of one sign, f
// is a multiple of that binade's ulp u, so fl(f + fStep) = f + RN_u(fStep) - a constant
// step d (with round-half-even ties only possible in the one binade where fStep is an odd
// multiple of u/2; there the first rounded step lands on an even multiple of u and every
// later step then has the same increment, so a run anchored one step into the binade has a
// constant d in every case).  A chirp's n steps therefore split into runs
// f_k = base + (k - k0) * d (both products and sums exact: every value is a multiple of u
// below 2^(e+1)) and single steps where the binade changes or the frequency wraps.  The
// runs are found once per chirp (chirp_segments, a few dozen per chirp); any sample's
// frequency then follows from its run, so the frame kernel fills a chirp's frequencies in
// parallel and leaves only the phase additions sequential.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LC_FN __host__ __device__ static inline
#else
#define LC_FN static inline
#endif

#pragma STDC FP_CONTRACT OFF
#ifdef __clang__
#pragma clang fp contract(off)
#endif

namespace lora {

// The chirp's constants as genChirp computes them (ChirpGenerator.hpp:107-109, double
// expressions rounded to float).
struct ChirpConst {
  float fMin, fMax, fStep, span;  // span = fMax - fMin (fp32, ChirpGenerator.hpp:120)
};

// A run of the frequency sequence: for steps k in [k0, k0 + len) (k = 1 is the first
// sample), f_k = base + (float)(k - k0) * d exactly.  A single step is len 1, d 0.
struct ChirpSeg {
  int32_t k0, len;
  float base, d;
};

// One step of the recurrence (ChirpGenerator.hpp:119-120).
LC_FN float chirp_fstep(float f, const ChirpConst& c) {
  f = f + c.fStep;
  if (f > c.fMax) f = f - c.span;
  return f;
}

LC_FN uint32_t lc_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}

// sign and exponent field (one binade of one sign), or -1 for zero / denormals
LC_FN int lc_binade(float f) {
  const uint32_t b = lc_bits(f);
  const int e = (int)((b >> 23) & 0xff);
  return (e == 0 || e == 0xff) ? -1 : (int)(b >> 23);
}

// 2^(e+1) for the binade [2^e, 2^(e+1)) of |f| (f normal): built from the exponent bits
LC_FN double lc_top(float f) {
  const uint64_t e = (lc_bits(f) >> 23) & 0xff;  // biased: 2^(e - 127 + 1) = double exponent e - 127 + 1 + 1023
  const uint64_t d = (e + 897u) << 52;
  double t;
  __builtin_memcpy(&t, &d, 8);
  return t;
}

// Runs of one chirp of n steps from f_init (the value before the first step, fl(fMin + f0)).
// Writes at most cap segments; returns the count, or -1 if cap was too small.
LC_FN int chirp_segments(float f_init, int n, const ChirpConst& c, ChirpSeg* seg, int cap) {
  int cnt = 0;
  int k = 0;
  float f = f_init;
  const double fs = (double)c.fStep;
  while (k < n) {
    // one step on its own: it may change the binade or wrap
    const float prev = f;
    f = chirp_fstep(f, c);
    ++k;
    if (cnt == cap) return -1;
    seg[cnt++] = ChirpSeg{k, 1, f, 0.0f};
    // a run needs its anchor one step into a binade (prev and f in the same binade, no
    // wrap between them), then the next step in it too to read the increment
    if (k >= n || lc_binade(f) < 0 || lc_binade(f) != lc_binade(prev) || !(f > prev)) continue;
    const float f2 = chirp_fstep(f, c);
    if (lc_binade(f2) != lc_binade(f) || !(f2 > f)) continue;
    const float d = f2 - f;  // exact: both in one binade
    // steps j = 1..L from the anchor: v_j = f + j d, valid while the exact v_{j-1} + fStep
    // stays in the anchor's binade and v_j does not wrap (v_j <= fMax)
    const double fd = (double)f, dd = (double)d;
    const double top = lc_top(f);
    auto ok = [&](int64_t j) {
      const double vprev = fd + (double)(j - 1) * dd, v = fd + (double)j * dd;
      const bool in_bin = f > 0.0f ? (vprev + fs < top) : (vprev + fs <= -top * 0.5);
      return in_bin && v <= (double)c.fMax;
    };
    // candidate from the bounds (one reciprocal: the estimate may be off by one either way),
    // then corrected by the exact conditions (monotone in j)
    double lim = (double)(n - k);
    const double inv = 1.0 / dd;
    if (f > 0.0f) {
      const double a = (top - fs - fd) * inv + 1.0, b = ((double)c.fMax - fd) * inv;
      lim = a < lim ? a : lim;
      lim = b < lim ? b : lim;
    } else {
      const double a = (-top * 0.5 - fs - fd) * inv + 1.0;
      lim = a < lim ? a : lim;
    }
    int64_t L = lim > 0.0 ? (int64_t)lim : 0;
    while (L > 0 && !ok(L)) --L;
    while (L < n - k && ok(L + 1)) ++L;
    if (L <= 0) continue;
    if (cnt == cap) return -1;
    seg[cnt++] = ChirpSeg{k + 1, (int32_t)L, f + d, d};
    f = f + (float)L * d;
    k += (int)L;
  }
  return cnt;
}

// Runs per chirp at most, for any osr 1-4 and bandwidth (tests/native/chirp_seg_check
// finds at most 6 SF + 8 over every start frequency a symbol < N or a sync nibble gives).
LC_FN constexpr int chirp_seg_cap(int sf) { return 7 * sf + 8; }

// f_k from a chirp's runs (s: the run holding k)
LC_FN float chirp_seg_f(const ChirpSeg& s, int k) { return s.base + (float)(k - s.k0) * s.d; }

}  // namespace lora
