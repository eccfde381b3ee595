// lora_libm.h — glibc-2.35-faithful single-precision transcendentals, usable from
// host C/C++ and from HIP device code (gfx950).
//
// Why this exists: the reference demodulator (src/phy/LoRaDemod.cpp) is plain C++
// compiled for x86-64 and links glibc's libm.  Its outputs (symbol indices, CFO,
// time offset) depend on the exact bits of
//   * sincosf  — per-sample CFO rotation, LoRaDemod.cpp:151-157 (gcc fuses the
//                std::cos/std::sin pair into one sincosf call),
//   * atan2f   — std::arg of the peak bin in the offset estimate, LoRaDemod.cpp:114,
//   * hypotf   — std::abs of the neighbour bins in LoRaDetector.hpp:66-67 (cabsf),
//   * log10f   — the detector power in LoRaDetector.hpp:63-64 (compared across
//                osr phases in LoRaDemod.cpp:101).
// The GPU must therefore evaluate the *same algorithms* as glibc, not "an accurate
// sinf".  These are restatements of the published algorithms glibc 2.35 uses:
//   * sincosf / logf: the Arm optimized-routines double-precision kernels, in the
//     x86-64 "FMA" multiarch build that glibc's IFUNC selects on any CPU with
//     FMA+AVX2 (every contraction site below is an explicit fma()).
//   * atan2f / atanf / log10f: the fdlibm single-precision code (no FMA).
//   * hypotf: glibc 2.35's (float)sqrt((double)x*x + (double)y*y).
// Coefficients are the values glibc ships (they are the published constants of the
// respective algorithms).  tests/test_libm_host.py checks every function here
// against the host libm bit-for-bit over tens of millions of inputs.
//
// Contraction must be OFF wherever this header is compiled (hipcc defaults to
// -ffp-contract=fast-honor-pragmas; the pragma below pins it).
//
// Third-party notices for the algorithms and constants restated here:
//
//   sincosf, logf (Arm optimized-routines, as shipped in glibc 2.35):
//     Copyright (c) 2018-2019, Arm Limited.
//     SPDX-License-Identifier: MIT (optimized-routines; glibc carries it under
//     LGPL-2.1-or-later)
//
//   atanf, atan2f, log10f (fdlibm, as shipped in glibc 2.35 sysdeps/ieee754/flt-32):
//     Conversion to float by Ian Lance Taylor, Cygnus Support, ian@cygnus.com.
//     ====================================================
//     Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//
//     Developed at SunPro, a Sun Microsystems, Inc. business.
//     Permission to use, copy, modify, and distribute this
//     software is freely granted, provided that this notice
//     is preserved.
//     ====================================================
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define LM_FN __host__ __device__ static inline
#else
#include <math.h>
#define LM_FN static inline
#endif

#pragma STDC FP_CONTRACT OFF
#ifdef __clang__
#pragma clang fp contract(off)
#endif

LM_FN uint32_t lm_asuint(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
LM_FN float lm_asfloat(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
LM_FN uint64_t lm_asuint64(double f) { uint64_t u; __builtin_memcpy(&u, &f, 8); return u; }
LM_FN double lm_asdouble(uint64_t u) { double f; __builtin_memcpy(&f, &u, 8); return f; }
LM_FN double lm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// ---------------------------------------------------------------------------
// sincosf (Arm optimized-routines algorithm, glibc 2.35 x86-64 FMA build)
// ---------------------------------------------------------------------------
// Polynomial table in glibc's field order {c0,c1,s1,c2,s2,c3,s3,c4}; quadrants with
// n&2 use the same table with the cosine coefficients negated, which yields exactly
// the negated cosine (fma/mul are sign-symmetric under round-to-nearest-even).
#define LM_SC_HPI_INV 0x1.45f306dc9c883p+23 /* 2/pi * 2^24 */
#define LM_SC_HPI 0x1.921fb54442d18p+0      /* pi/2 */
#define LM_SC_C0 1.0
#define LM_SC_C1 (-0x1.ffffffd0c621cp-2)
#define LM_SC_S1 (-0x1.555545995a603p-3)
#define LM_SC_C2 0x1.55553e1068f19p-5
#define LM_SC_S2 0x1.1107605230bc4p-7
#define LM_SC_C3 (-0x1.6c087e89a359dp-10)
#define LM_SC_S3 (-0x1.994eb3774cf24p-13)
#define LM_SC_C4 0x1.99343027bf8c3p-16
#define LM_PI63 0x1.921fb54442d18p-62 /* pi * 2^-63 */

// Bits of 4/pi used by the large-argument reduction (glibc __inv_pio4).
#if defined(__HIPCC__) || defined(__HIP__)
__device__ __constant__ static const uint32_t lm_inv_pio4_dev[24] = {
#else
static const uint32_t lm_inv_pio4_host[24] = {
#endif
    0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
    0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
    0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
    0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};

#if defined(__HIPCC__) || defined(__HIP__)
#if defined(__HIP_DEVICE_COMPILE__)
#define LM_INV_PIO4 lm_inv_pio4_dev
#else
static const uint32_t lm_inv_pio4_host[24] = {
    0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
    0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
    0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
    0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
#define LM_INV_PIO4 lm_inv_pio4_host
#endif
#else
#define LM_INV_PIO4 lm_inv_pio4_host
#endif

LM_FN uint32_t lm_abstop12(float x) { return (lm_asuint(x) >> 20) & 0x7ff; }

// The shared polynomial: x is the sign-adjusted reduced argument, x2 = x*x.
// Returns (s, c) before the quadrant swap; `negc` negates c (table 1).
LM_FN void lm_sincosf_poly(double x, double x2, int negc, float* s_out, float* c_out) {
  const double x3 = x2 * x;
  const double x4 = x2 * x2;
  const double x5 = x2 * x3;
  const double x6 = x2 * x4;
  const double s1 = lm_fma(x2, LM_SC_S3, LM_SC_S2);
  const double c2 = lm_fma(x2, LM_SC_C4, LM_SC_C3);
  const double c1 = lm_fma(x2, LM_SC_C1, LM_SC_C0);
  const double s = lm_fma(x3, LM_SC_S1, x);
  const double c = lm_fma(x4, LM_SC_C2, c1);
  const float sf = (float)lm_fma(s1, x5, s);
  float cf = (float)lm_fma(c2, x6, c);
  if (negc) cf = -cf;
  *s_out = sf;
  *c_out = cf;
}

// sincosf(y) -> (*sinp, *cosp).  Finite inputs only (the demodulator never feeds
// inf/NaN phases; NaN in -> NaN out is preserved).
LM_FN void lm_sincosf(float y, float* sinp, float* cosp) {
  double x = (double)y;
  const uint32_t top = lm_abstop12(y);
  float s, c;
  if (top < 0x3f4u) {  // |y| < pi/4
    if (top < 0x398u) {  // |y| < 2^-12
      *sinp = y;
      *cosp = 1.0f;
      return;
    }
    lm_sincosf_poly(x, x * x, 0, &s, &c);
    *sinp = s;
    *cosp = c;
    return;
  }
  int n;
  int nq;  // quadrant used for sign/table selection
  if (top < 0x42fu) {  // |y| < 120: reduce_fast
    const double r = x * LM_SC_HPI_INV;
    n = (((int32_t)r) + 0x800000) >> 24;
    x = lm_fma(-(double)n, LM_SC_HPI, x);
    nq = n;
  } else if (top < 0x7f8u) {  // reduce_large (Payne-Hanek with 4/pi bits)
    uint32_t xi = lm_asuint(y);
    const int sign = (int)(xi >> 31);
    const uint32_t* arr = &LM_INV_PIO4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t nn = (res0 + (1ull << 61)) >> 62;
    res0 -= nn << 62;
    x = (double)(int64_t)res0 * LM_PI63;
    n = (int)nn;
    nq = n + sign;
  } else {  // inf / NaN
    const float nanv = y - y;
    *sinp = nanv;
    *cosp = nanv;
    return;
  }
  const double xs = (nq & 1) ^ ((nq >> 1) & 1) ? -x : x;  // sign[nq&3] = {1,-1,-1,1}
  lm_sincosf_poly(xs, x * x, (nq & 2) != 0, &s, &c);
  if (n & 1) {
    *sinp = c;
    *cosp = s;
  } else {
    *sinp = s;
    *cosp = c;
  }
}

// Branch-free form of lm_sincosf for |y| < 120 (abstop12 < 0x42f).  glibc's |y| < pi/4
// path equals its reduce_fast path with n = 0 (fma(-0, hpi, x) == x), and its
// |y| < 2^-12 shortcut (y, 1.0f) equals the polynomial's rounding there except for
// the sign of -0; so one straight-line sequence reproduces all three.  Checked exhaustively against glibc
// (tests/test_libm_host.py).
LM_FN void lm_sincosf_fast(float y, float* sinp, float* cosp) {
  const double x = (double)y;
  const double r = x * LM_SC_HPI_INV;
  const int n = (((int32_t)r) + 0x800000) >> 24;
  const double xr = lm_fma(-(double)n, LM_SC_HPI, x);
  const double xs = ((n ^ (n >> 1)) & 1) ? -xr : xr;
  float s, c;
  lm_sincosf_poly(xs, xr * xr, (n & 2) != 0, &s, &c);
  const float sv = (n & 1) ? c : s;
  *sinp = (y == 0.0f) ? y : sv;  // keep the sign of -0 (glibc's tiny path returns y)
  *cosp = (n & 1) ? s : c;
}

// K-way lockstep version of lm_sincosf_fast (identical arithmetic per element).  The
// element chains are written interleaved so the compiler keeps K independent DP
// dependency chains in flight instead of one long serial chain per point.
template <int K>
LM_FN void lm_sincosf_fast_k(const float* y, float* sinp, float* cosp) {
  double x[K], xr[K], xs[K], x2[K], x3[K], x4[K], x5[K], x6[K];
  int n[K];
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = (double)y[k];
#pragma unroll
  for (int k = 0; k < K; ++k) n[k] = (((int32_t)(x[k] * LM_SC_HPI_INV)) + 0x800000) >> 24;
#pragma unroll
  for (int k = 0; k < K; ++k) xr[k] = lm_fma(-(double)n[k], LM_SC_HPI, x[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    xs[k] = ((n[k] ^ (n[k] >> 1)) & 1) ? -xr[k] : xr[k];
    x2[k] = xr[k] * xr[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    x3[k] = x2[k] * xs[k];
    x4[k] = x2[k] * x2[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    x5[k] = x2[k] * x3[k];
    x6[k] = x2[k] * x4[k];
  }
  double s1[K], c2[K], c1[K], sp[K], cp[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    s1[k] = lm_fma(x2[k], LM_SC_S3, LM_SC_S2);
    c2[k] = lm_fma(x2[k], LM_SC_C4, LM_SC_C3);
    c1[k] = lm_fma(x2[k], LM_SC_C1, LM_SC_C0);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    sp[k] = lm_fma(x3[k], LM_SC_S1, xs[k]);
    cp[k] = lm_fma(x4[k], LM_SC_C2, c1[k]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float sf = (float)lm_fma(s1[k], x5[k], sp[k]);
    float cf = (float)lm_fma(c2[k], x6[k], cp[k]);
    if (n[k] & 2) cf = -cf;
    const float sv = (n[k] & 1) ? cf : sf;
    sinp[k] = (y[k] == 0.0f) ? y[k] : sv;
    cosp[k] = (n[k] & 1) ? sf : cf;
  }
}

// lm_sincosf_fast_k for callers that only need the rotation's magnitude-relevant
// bits (the demodulator's argmax): identical except that sin(-0) may come out +0
// (glibc returns -0).  A zero's sign never changes |X|^2 of any bin, so symbol
// indices are unaffected.  The quadrant sign of the reduced argument is applied by
// flipping its sign bit instead of a select.
template <int K>
LM_FN void lm_sincosf_fast_k_nz(const float* y, float* sinp, float* cosp) {
  double xs[K], x2[K], x3[K], x4[K], x5[K], x6[K];
  int n[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double x = (double)y[k];
    n[k] = (((int32_t)(x * LM_SC_HPI_INV)) + 0x800000) >> 24;
    const double xr = lm_fma(-(double)n[k], LM_SC_HPI, x);
    const uint64_t flip = (uint64_t)((uint32_t)(n[k] ^ (n[k] >> 1)) & 1u) << 63;
    xs[k] = lm_asdouble(lm_asuint64(xr) ^ flip);  // sign[nq & 3] = {1,-1,-1,1}
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    x2[k] = xs[k] * xs[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    x3[k] = x2[k] * xs[k];
    x4[k] = x2[k] * x2[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    x5[k] = x2[k] * x3[k];
    x6[k] = x2[k] * x4[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double s1 = lm_fma(x2[k], LM_SC_S3, LM_SC_S2);
    const double c2 = lm_fma(x2[k], LM_SC_C4, LM_SC_C3);
    const double c1 = lm_fma(x2[k], LM_SC_C1, LM_SC_C0);
    const double sp = lm_fma(x3[k], LM_SC_S1, xs[k]);
    const double cp = lm_fma(x4[k], LM_SC_C2, c1);
    const float sf = (float)lm_fma(s1, x5[k], sp);
    float cf = (float)lm_fma(c2, x6[k], cp);
    if (n[k] & 2) cf = -cf;
    sinp[k] = (n[k] & 1) ? cf : sf;
    cosp[k] = (n[k] & 1) ? sf : cf;
  }
}

// Branch-free lm_sincosf for every input (same results, including -0, inf and NaN):
// both of glibc's argument reductions are evaluated - reduce_fast (|y| < 120, which
// also reproduces the |y| < pi/4 and tiny paths, see lm_sincosf_fast) and the
// Payne-Hanek reduce_large - and selected per element, then one polynomial.  For a
// wave whose phases straddle 120 or lie beyond it (large CFO, long frames, the
// modulator's in-chirp phase) this replaces lm_sincosf's divergent branches.
LM_FN void lm_sincosf_bf(float y, float* sinp, float* cosp) {
  const uint32_t top = lm_abstop12(y);
  const double x = (double)y;
  // reduce_fast
  const int nf = (((int32_t)(x * LM_SC_HPI_INV)) + 0x800000) >> 24;
  const double xf = lm_fma(-(double)nf, LM_SC_HPI, x);
  // reduce_large (valid for finite |y| >= 120; computed regardless, selected below)
  uint32_t xi = lm_asuint(y);
  const int sign = (int)(xi >> 31);
  const uint32_t* arr = &LM_INV_PIO4[(xi >> 26) & 15];
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffffu) | 0x800000u;
  xi <<= shift;
  uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
  const uint64_t res1 = (uint64_t)xi * arr[4];
  const uint64_t res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t nn = (res0 + (1ull << 61)) >> 62;
  res0 -= nn << 62;
  const double xl = (double)(int64_t)res0 * LM_PI63;
  const bool large = top >= 0x42fu;
  const double xr = large ? xl : xf;
  const int n = large ? (int)nn : nf;
  const int nq = large ? (int)nn + sign : nf;
  const double xs = ((nq ^ (nq >> 1)) & 1) ? -xr : xr;
  float sv, cv;
  lm_sincosf_poly(xs, xr * xr, (nq & 2) != 0, &sv, &cv);
  float so = (n & 1) ? cv : sv;
  float co = (n & 1) ? sv : cv;
  if (y == 0.0f) so = y;  // sin(-0) = -0 (glibc's tiny path)
  if (top >= 0x7f8u) so = co = y - y;  // inf / NaN
  *sinp = so;
  *cosp = co;
}

// True when lm_sincosf_fast is exact for y.
LM_FN int lm_sincosf_fast_ok(float y) { return lm_abstop12(y) < 0x42fu; }

// lm_sincosf_bf's large-argument branch alone: exact for finite |y| >= 120
// (lm_sincosf_large_ok), where glibc takes reduce_large - the same integer Payne-Hanek
// reduction and polynomial, without evaluating reduce_fast and selecting.
LM_FN int lm_sincosf_large_ok(float y) {
  const uint32_t top = lm_abstop12(y);
  return top >= 0x42fu && top < 0x7f8u;
}
LM_FN void lm_sincosf_large(float y, float* sinp, float* cosp) {
  uint32_t xi = lm_asuint(y);
  const int sign = (int)(xi >> 31);
  const uint32_t* arr = &LM_INV_PIO4[(xi >> 26) & 15];
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffffu) | 0x800000u;
  xi <<= shift;
  uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
  const uint64_t res1 = (uint64_t)xi * arr[4];
  const uint64_t res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t nn = (res0 + (1ull << 61)) >> 62;
  res0 -= nn << 62;
  const double xr = (double)(int64_t)res0 * LM_PI63;
  const int n = (int)nn;
  const int nq = (int)nn + sign;
  const double xs = ((nq ^ (nq >> 1)) & 1) ? -xr : xr;
  float sv, cv;
  lm_sincosf_poly(xs, xr * xr, (nq & 2) != 0, &sv, &cv);
  *sinp = (n & 1) ? cv : sv;
  *cosp = (n & 1) ? sv : cv;
}

// ---------------------------------------------------------------------------
// hypotf (glibc 2.35): exact double sum of squares, double sqrt, round to float.
// ---------------------------------------------------------------------------
LM_FN float lm_hypotf(float x, float y) {
  const double dx = (double)x, dy = (double)y;
  return (float)__builtin_sqrt(dx * dx + dy * dy);
}

// ---------------------------------------------------------------------------
// atanf / atan2f (fdlibm single precision, as built into glibc 2.35 libm)
// ---------------------------------------------------------------------------
LM_FN float lm_atanf(float x) {
  const float atanhi0 = lm_asfloat(0x3eed6338u), atanhi1 = lm_asfloat(0x3f490fdau),
              atanhi2 = lm_asfloat(0x3f7b985eu), atanhi3 = lm_asfloat(0x3fc90fdau);
  const float atanlo0 = lm_asfloat(0x31ac3769u), atanlo1 = lm_asfloat(0x33222168u),
              atanlo2 = lm_asfloat(0x33140fb4u), atanlo3 = lm_asfloat(0x33a22168u);
  const float aT0 = lm_asfloat(0x3eaaaaabu), aT1 = lm_asfloat(0xbe4ccccdu),
              aT2 = lm_asfloat(0x3e124925u), aT3 = lm_asfloat(0xbde38e38u),
              aT4 = lm_asfloat(0x3dba2e6eu), aT5 = lm_asfloat(0xbd9d8795u),
              aT6 = lm_asfloat(0x3d886b35u), aT7 = lm_asfloat(0xbd6ef16bu),
              aT8 = lm_asfloat(0x3d4bda59u), aT9 = lm_asfloat(0xbd15a221u),
              aT10 = lm_asfloat(0x3c8569d7u);
  const uint32_t hx = lm_asuint(x);
  const uint32_t ix = hx & 0x7fffffffu;
  int id;
  if (ix >= 0x4c000000u) {  // |x| >= 2^25
    if (ix > 0x7f800000u) return x + x;  // NaN
    return ((int32_t)hx > 0) ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000u) {  // |x| < 0.4375
    if (ix < 0x31000000u) {  // |x| < 2^-29
      if (1.0e30f + x > 1.0f) return x;
    }
    id = -1;
  } else {
    x = __builtin_fabsf(x);
    if (ix < 0x3f980000u) {      // |x| < 1.1875
      if (ix < 0x3f300000u) {    // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    } else {
      if (ix < 0x401c0000u) {  // |x| < 2.4375
        id = 2;
        x = (x - 1.5f) / (1.0f + 1.5f * x);
      } else {  // 2.4375 <= |x| < 2^25
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  const float z = x * x;
  const float w = z * z;
  const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  const float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  const float zz = hi - ((x * (s1 + s2) - lo) - x);
  return ((int32_t)hx < 0) ? -zz : zz;
}

LM_FN float lm_atan2f(float y, float x) {
  const float tiny = 1.0e-30f;
  const float pi_o_4 = lm_asfloat(0x3f490fdbu);
  const float pi_o_2 = lm_asfloat(0x3fc90fdbu);
  const float pi = lm_asfloat(0x40490fdbu);
  const float pi_lo = lm_asfloat(0xb3bbbd2eu);
  const uint32_t hx = lm_asuint(x), hy = lm_asuint(y);
  const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;  // NaN
  if (hx == 0x3f800000u) return lm_atanf(y);                // x = 1.0
  const int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));  // 2*sign(x)+sign(y)
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return ((int32_t)hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000u) {
    if (iy == 0x7f800000u) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000u) return ((int32_t)hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int32_t k = ((int32_t)iy - (int32_t)ix) >> 23;
  float z;
  if (k > 60) {
    z = pi_o_2 + 0.5f * pi_lo;  // |y/x| > 2^60
  } else if ((int32_t)hx < 0 && k < -60) {
    z = 0.0f;  // |y|/x < -2^60
  } else {
    z = lm_atanf(__builtin_fabsf(y / x));
  }
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---------------------------------------------------------------------------
// logf (Arm optimized-routines, glibc 2.35 x86-64 FMA build) and log10f (fdlibm
// wrapper that calls logf).
// ---------------------------------------------------------------------------
LM_FN void lm_logf_tab(int i, double* invc, double* logc) {
  // {invc, logc} for the 16 subintervals of [0x3f330000, 2*0x3f330000).
  const uint64_t T[16][2] = {
      {0x3ff661ec79f8f3beull, 0xbfd57bf7808caadeull}, {0x3ff571ed4aaf883dull, 0xbfd2bef0a7c06ddbull},
      {0x3ff49539f0f010b0ull, 0xbfd01eae7f513a67ull}, {0x3ff3c995b0b80385ull, 0xbfcb31d8a68224e9ull},
      {0x3ff30d190c8864a5ull, 0xbfc6574f0ac07758ull}, {0x3ff25e227b0b8ea0ull, 0xbfc1aa2bc79c8100ull},
      {0x3ff1bb4a4a1a343full, 0xbfba4e76ce8c0e5eull}, {0x3ff12358f08ae5baull, 0xbfb1973c5a611cccull},
      {0x3ff0953f419900a7ull, 0xbfa252f438e10c1eull}, {0x3ff0000000000000ull, 0x0000000000000000ull},
      {0x3fee608cfd9a47acull, 0x3faaa5aa5df25984ull}, {0x3feca4b31f026aa0ull, 0x3fbc5e53aa362eb4ull},
      {0x3feb2036576afce6ull, 0x3fc526e57720db08ull}, {0x3fe9c2d163a1aa2dull, 0x3fcbc2860d224770ull},
      {0x3fe886e6037841edull, 0x3fd1058bc8a07ee1ull}, {0x3fe767dcf5534862ull, 0x3fd4043057b6ee09ull}};
  *invc = lm_asdouble(T[i][0]);
  *logc = lm_asdouble(T[i][1]);
}

LM_FN float lm_logf(float x) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = lm_asdouble(0xbfd00ea348b88334ull);
  const double A1 = lm_asdouble(0x3fd5575b0be00b6aull);
  const double A2 = lm_asdouble(0xbfdffffef20a4123ull);
  uint32_t ix = lm_asuint(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -__builtin_inff();  // log(+-0) = -inf
    if (ix == 0x7f800000u) return x;            // log(inf) = inf
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);  // NaN
    ix = lm_asuint(x * 8388608.0f);  // subnormal: normalise
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & (0x1ffu << 23));
  double invc, logc;
  lm_logf_tab(i, &invc, &logc);
  const double z = (double)lm_asfloat(iz);
  const double r = lm_fma(z, invc, -1.0);
  const double y0 = lm_fma((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = lm_fma(A1, r, A2);
  y = lm_fma(A0, r2, y);
  y = lm_fma(y, r2, y0 + r);
  return (float)y;
}

LM_FN float lm_log10f(float x) {
  const float two25 = 33554432.0f;
  const float ivln10 = lm_asfloat(0x3ede5bd9u);
  const float log10_2hi = lm_asfloat(0x3e9a2080u);
  const float log10_2lo = lm_asfloat(0x355427dbu);
  int32_t hx = (int32_t)lm_asuint(x);
  int32_t k = 0;
  if (hx < 0x00800000) {
    if ((hx & 0x7fffffff) == 0) return -two25 / 0.0f;  // -inf
    if (hx < 0) return (x - x) / (x - x);                // NaN
    k -= 25;
    x *= two25;
    hx = (int32_t)lm_asuint(x);
  }
  if (hx >= 0x7f800000) return x + x;
  k += (hx >> 23) - 127;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
  const float y = (float)(k + i);
  x = lm_asfloat((uint32_t)hx);
  const float z = y * log10_2lo + ivln10 * lm_logf(x);
  return z + y * log10_2hi;
}
