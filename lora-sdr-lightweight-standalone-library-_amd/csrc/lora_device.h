// lora_device.h — device building blocks shared by the demod/mod kernels (gfx950).
//
// Arithmetic contract: every fp32 operation below is one IEEE operation in the same
// order as the reference's x86-64 build (no FMA contraction — the file pins
// `fp contract(off)` and the library is compiled with -ffp-contract=off), so the
// FFT values, magnitudes and argmax are bit-identical to kissfft<float> /
// LoRaDetector<float> (include/lora_phy/kissfft.hh, LoRaDetector.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lora_libm.h"

#pragma clang fp contract(off)

namespace lora {

// float(M_PI), the reference's `float(M_PI)` (phy.cpp:40, LoRaDemod.cpp)
constexpr float PI_F = 3.14159265358979323846f;

struct alignas(8) cf {  // 8-byte aligned: one 64-bit LDS / global access per value
  float re, im;
};

// Per-frame results of the offset estimate, consumed by every symbol of the frame.
struct FrameParams {
  float cfo, toff, rate, scale;
  int t_off, scaled, pad0, pad1;
};
// Field by field: a whole-struct copy between global and LDS memory was lowered through a
// 32-byte scratch buffer (k_cert_split, k_est_fast<..., 2>).
__device__ __forceinline__ FrameParams load_fp(const FrameParams* p) {
  FrameParams q;
  q.cfo = p->cfo;
  q.toff = p->toff;
  q.rate = p->rate;
  q.scale = p->scale;
  q.t_off = p->t_off;
  q.scaled = p->scaled;
  q.pad0 = p->pad0;
  q.pad1 = p->pad1;
  return q;
}
__device__ __forceinline__ void store_fp(FrameParams* p, const FrameParams& q) {
  p->cfo = q.cfo;
  p->toff = q.toff;
  p->rate = q.rate;
  p->scale = q.scale;
  p->t_off = q.t_off;
  p->scaled = q.scaled;
  p->pad0 = q.pad0;
  p->pad1 = q.pad1;
}

// std::complex<float> product as GCC lowers it: (ac - bd, ad + bc).
__device__ __forceinline__ cf cmul(cf a, cf b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
// ---- packed fp32 complex arithmetic (v_pk_*_f32: both components in one instruction) ----
// A complex value is a VGPR pair (re, im); op_sel / op_sel_hi pick which half of each source
// feeds the low / high lane and neg_lo / neg_hi negate it, so swaps and the j-rotations of
// the butterflies cost nothing.  A packed instruction issues at about 0.58 of the scalar
// fp32 rate while doing two operations (tools/micro/valu_rate.hip).  Every operation is
// one IEEE fp32 operation (an fma rounds once), so pk_cmul_ref below is bit-identical to
// cmul; the others are used only by the certified speculative demod, whose rounding bound
// covers them (lora_demod_fast.hip, certify_list).
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f pk(cf a) { return __builtin_bit_cast(v2f, a); }
__device__ __forceinline__ cf unpk(v2f a) { return __builtin_bit_cast(cf, a); }
// a * w with the reference's roundings: (fl(ar wr) - fl(ai wi), fl(ai wr) + fl(ar wi)) = cmul
// Each helper's dependent instructions sit in ONE asm statement: the hazard recognizer
// cannot see inside an inline asm, so it pads every asm that reads a VGPR the previous asm
// just wrote with an s_nop - one per complex product when each instruction was its own
// statement (110 s_nops per symbol in the SF12 symbol pass's loop).  Back to back, the
// hardware interlocks these VALU -> VALU dependences itself (the compiler's own packed code
// carries no wait states there).  "=&v": the result is written before the last input read.
__device__ __forceinline__ cf pk_cmul_ref(cf a, cf w) {
  v2f p, q, r;
  asm("v_pk_mul_f32 %1, %3, %4 op_sel_hi:[1,0]\n\t"                                   // (ar wr, ai wr)
      "v_pk_mul_f32 %2, %3, %4 op_sel:[0,1]\n\t"                                      // (ar wi, ai wi)
      "v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
      : "=v"(r), "=&v"(p), "=&v"(q)
      : "v"(pk(a)), "v"(pk(w)));
  return unpk(r);
}
// a * w: (fma(-ai, wi, fl(ar wr)), fma(ar, wi, fl(ai wr)))
__device__ __forceinline__ v2f pk_cmul(v2f a, v2f w) {
  v2f t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(r), "=&v"(t)
      : "v"(a), "v"(w));
  return r;
}
// two independent products a0 * w0, a1 * w1 (pk_cmul's operations) in one asm statement:
// one hazard pad per pair instead of one per product, the halves interleaved
__device__ __forceinline__ void pk_cmul2(v2f a0, v2f w0, v2f a1, v2f w1, v2f& r0, v2f& r1) {
  v2f t0, t1;
  asm("v_pk_mul_f32 %2, %4, %5 op_sel_hi:[1,0]\n\t"
      "v_pk_mul_f32 %3, %6, %7 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %4, %5, %2 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
      "v_pk_fma_f32 %1, %6, %7, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=&v"(r0), "=v"(r1), "=&v"(t0), "=&v"(t1)
      : "v"(a0), "v"(w0), "v"(a1), "v"(w1));
}
// two steps of a product recurrence, r0 = a * w, r1 = r0 * w (pk_cmul's operations), in one
// asm statement
__device__ __forceinline__ void pk_cmul_chain2(v2f a, v2f w, v2f& r0, v2f& r1) {
  v2f t0, t1;
  asm("v_pk_mul_f32 %2, %4, %5 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %4, %5, %2 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
      "v_pk_mul_f32 %3, %0, %5 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %1, %0, %5, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=&v"(r0), "=v"(r1), "=&v"(t0), "=&v"(t1)
      : "v"(a), "v"(w));
}
// c + a * w: (fma(-ai, wi, fma(ar, wr, cr)), fma(ar, wi, fma(ai, wr, ci)))
__device__ __forceinline__ v2f pk_cfma(v2f a, v2f w, v2f c) {
  v2f t, r;
  asm("v_pk_fma_f32 %1, %2, %3, %4 op_sel_hi:[1,0,1]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(r), "=&v"(t)
      : "v"(a), "v"(w), "v"(c));
  return r;
}
__device__ __forceinline__ v2f pk_add(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2f pk_sub(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a - j b = (ar + bi, ai - br) and a + j b = (ar - bi, ai + br)
__device__ __forceinline__ v2f pk_sub_j(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2f pk_add_j(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// 2 a - b and b - 2 a (one fma per component)
__device__ __forceinline__ v2f pk_twice_minus(v2f a, v2f b) {
  v2f r;
  asm("v_pk_fma_f32 %0, %1, 2.0, %2 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2f pk_minus_twice(v2f b, v2f a) {
  v2f r;
  asm("v_pk_fma_f32 %0, %1, -2.0, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// FMA = true: the product with fused multiply-adds (fewer roundings, not the reference's
// arithmetic), packed: only for the speculative demod, whose symbols are certified against
// a rounding bound (lora_demod_fast.hip, certify_list).
template <bool FMA>
__device__ __forceinline__ cf cmul_t(cf a, cf b) {
  if constexpr (FMA)
    return unpk(pk_cmul(pk(a), pk(b)));
  else
    return cmul(a, b);
}
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf cscale(cf a, float s) { return {a.re * s, a.im * s}; }

// kissfft.hh:164-185 kf_bfly4 (forward) on F[0], F[m], F[2m], F[3m].
// FMA (certified path): the same outputs from twelve packed operations -
//   A = f0 + w2 f2, B = 2 f0 - A (= f0 - w2 f2), P = w3 f3, C = P + w1 f1, D = C - 2 P
//   (= w1 f1 - w3 f3); f0 = A + C, f2 = A - C, f1 = B - j D, f3 = B + j D
// (kissfft's 3 products and 8 sums: 28 scalar operations).  Per component the rounding
// error of an output is at most 6 u (|f0| + |f1| + |f2| + |f3|) (D's error is C's minus twice
// P's plus one rounding: 5 u (|f1| + |f3|)), within the bound's 8 u per radix-2 level.
template <bool FMA = false>
__device__ __forceinline__ void bfly4(cf& f0, cf& f1, cf& f2, cf& f3, cf w1, cf w2, cf w3) {
  if constexpr (FMA) {
    // pk_cfma(f2, w2, f0) = A, pk_cmul(f3, w3) = P, pk_twice_minus(f0, A) = B,
    // pk_cfma(f1, w1, P) = C, pk_minus_twice(C, P) = D, then pk_add / pk_sub / pk_sub_j /
    // pk_add_j - the same twelve instructions, in one asm statement (no hazard padding
    // between them; see pk_cmul_ref), the two products' halves interleaved
    v2f x0 = pk(f0), x1 = pk(f1), x2 = pk(f2), x3 = pk(f3), A, B, P, C, D;
    asm("v_pk_fma_f32 %4, %2, %9, %0 op_sel_hi:[1,0,1]\n\t"
        "v_pk_mul_f32 %6, %3, %10 op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %4, %2, %9, %4 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
        "v_pk_fma_f32 %6, %3, %10, %6 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
        "v_pk_fma_f32 %7, %1, %11, %6 op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %5, %0, 2.0, %4 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 %7, %1, %11, %7 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
        "v_pk_fma_f32 %8, %6, -2.0, %7 op_sel_hi:[1,0,1]\n\t"
        "v_pk_add_f32 %0, %4, %7\n\t"
        "v_pk_add_f32 %2, %4, %7 neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %1, %5, %8 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %3, %5, %8 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
        : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=&v"(A), "=&v"(B), "=&v"(P), "=&v"(C), "=&v"(D)
        : "v"(pk(w2)), "v"(pk(w3)), "v"(pk(w1)));
    f0 = unpk(x0);
    f1 = unpk(x1);
    f2 = unpk(x2);
    f3 = unpk(x3);
    return;
  }
  const cf s0 = cmul_t<FMA>(f1, w1);
  const cf s1 = cmul_t<FMA>(f2, w2);
  const cf s2 = cmul_t<FMA>(f3, w3);
  const cf s5 = csub(f0, s1);
  const cf a0 = cadd(f0, s1);
  const cf s3 = cadd(s0, s2);
  cf s4 = csub(s0, s2);
  s4 = cf{s4.im, -s4.re};
  f2 = csub(a0, s3);
  f0 = cadd(a0, s3);
  f1 = cadd(s5, s4);
  f3 = csub(s5, s4);
}

// bfly4 with w1 = w2 = w3 = (1, 0), the multiplies skipped: identical outputs up to
// the sign of zero components (argmax-only callers, see pass_regs).  PK: the same sums as
// packed adds (bit-identical; the certified path's transforms use it).
template <bool PK = false>
__device__ __forceinline__ void bfly4_unit(cf& f0, cf& f1, cf& f2, cf& f3) {
  if constexpr (PK) {
    // s5 = f0 - f2, a0 = f0 + f2, s3 = f1 + f3, s4 = f1 - f3; f2 = a0 - s3, f0 = a0 + s3,
    // f1 = s5 - j s4 = s5 + (s4.im, -s4.re), f3 = s5 + j s4 (one asm statement, as bfly4)
    v2f x0 = pk(f0), x1 = pk(f1), x2 = pk(f2), x3 = pk(f3), s5, a0, s3, s4;
    asm("v_pk_add_f32 %4, %0, %2 neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %5, %0, %2\n\t"
        "v_pk_add_f32 %6, %1, %3\n\t"
        "v_pk_add_f32 %7, %1, %3 neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %2, %5, %6 neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %0, %5, %6\n\t"
        "v_pk_add_f32 %1, %4, %7 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %3, %4, %7 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
        : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=&v"(s5), "=&v"(a0), "=&v"(s3), "=&v"(s4));
    f0 = unpk(x0);
    f1 = unpk(x1);
    f2 = unpk(x2);
    f3 = unpk(x3);
    return;
  }
  const cf s5 = csub(f0, f2);
  const cf a0 = cadd(f0, f2);
  const cf s3 = cadd(f1, f3);
  cf s4 = csub(f1, f3);
  s4 = cf{s4.im, -s4.re};
  f2 = csub(a0, s3);
  f0 = cadd(a0, s3);
  f1 = cadd(s5, s4);
  f3 = csub(s5, s4);
}

// bfly2 with w = (1, 0), the multiply skipped (argmax-only callers, see bfly4_unit).
template <bool PK = false>
__device__ __forceinline__ void bfly2_unit(cf& f0, cf& f1) {
  if constexpr (PK) {
    const v2f a = pk(f0), t = pk(f1);
    f1 = unpk(pk_sub(a, t));
    f0 = unpk(pk_add(a, t));
    return;
  }
  const cf a = f0, t = f1;
  f1 = csub(a, t);
  f0 = cadd(a, t);
}

// kissfft.hh:155-162 kf_bfly2 (forward).
template <bool FMA = false>
__device__ __forceinline__ void bfly2(cf& f0, cf& f1, cf w) {
  if constexpr (FMA) {  // A = f0 + w f1 (pk_cfma), B = 2 f0 - A (pk_twice_minus): one asm
    v2f x0 = pk(f0), x1 = pk(f1), A;
    asm("v_pk_fma_f32 %2, %1, %3, %0 op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %2, %1, %3, %2 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]\n\t"
        "v_pk_fma_f32 %1, %0, 2.0, %2 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]"
        : "+v"(x0), "+v"(x1), "=&v"(A)
        : "v"(pk(w)));
    f1 = unpk(x1);
    f0 = unpk(A);
    return;
  }
  const cf t = cmul_t<FMA>(f1, w);
  const cf a = f0;
  f1 = csub(a, t);
  f0 = cadd(a, t);
}

// Cooperative in-place DIT FFT of G transforms of N = 2^sf points held in LDS in
// kissfft's leaf order (A[rev[i]] = x[i]).  Stages run bottom-up exactly as
// kf_work's recursion unwinds: the radix-2 stage (odd sf) first with m = 1, then
// radix-4 stages with m = 1|2, 4|8, ...  Twiddle for butterfly k of a stage of block
// size M is tw[q*k*(N/M)] (kissfft.hh:158,169-171).
__device__ __forceinline__ void fft_lds(cf* A, int sf, int G, const cf* __restrict__ tw, int tid,
                                        int nthreads) {
  const int N = 1 << sf;
  int M = 1;
  if (sf & 1) {
    const cf w0 = tw[0];
    for (int b = tid; b < (G * N) >> 1; b += nthreads) {
      cf a = A[2 * b], c = A[2 * b + 1];
      bfly2(a, c, w0);
      A[2 * b] = a;
      A[2 * b + 1] = c;
    }
    M = 2;
    __syncthreads();
  }
  for (M *= 4; M <= N; M *= 4) {
    const int m = M >> 2;
    const int fs = N / M;
    const int nb = (G * N) >> 2;
    for (int b = tid; b < nb; b += nthreads) {
      const int sym = b >> (sf - 2);
      const int bb = b & ((N >> 2) - 1);
      const int blk = bb / m;
      const int k = bb - blk * m;
      cf* p = A + sym * N + blk * M + k;
      cf f0 = p[0], f1 = p[m], f2 = p[2 * m], f3 = p[3 * m];
      bfly4(f0, f1, f2, f3, tw[k * fs], tw[2 * k * fs], tw[3 * k * fs]);
      p[0] = f0;
      p[m] = f1;
      p[2 * m] = f2;
      p[3 * m] = f3;
    }
    __syncthreads();
  }
}

// Packed argmax key: |X|^2 bits in the high word (non-negative floats order like
// their bits; NaN and 0 map to 0, matching the strict '>' scan from maxValue = 0 in
// LoRaDetector.hpp:46-58), bit-inverted index in the low word so that max() picks
// the LOWEST index among equal magnitudes (first max wins).
__device__ __forceinline__ uint64_t argmax_key(cf v, uint32_t idx) {
  const float m2 = v.re * v.re + v.im * v.im;
  const float val = (m2 > 0.0f) ? m2 : 0.0f;
  return ((uint64_t)__float_as_uint(val) << 32) | (uint32_t)(~idx);
}
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t key_index(uint64_t k) { return ~(uint32_t)k; }
__device__ __forceinline__ float key_value(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t lo2 = __shfl_xor(lo, mask, 64), hi2 = __shfl_xor(hi, mask, 64);
  return ((uint64_t)hi2 << 32) | lo2;
}

// Reduce a key over aligned groups of T lanes (T a power of two <= 64).
__device__ __forceinline__ uint64_t group_max(uint64_t k, int T) {
  for (int s = T >> 1; s > 0; s >>= 1) k = umax64(k, shfl_xor64(k, s));
  return k;
}

// LoRaDetector.hpp:66-71: the fractional index alone.  Single-phase estimates (osr 1) use
// the power only through LoRaDemod.cpp:97's `p > best_p` against best_p = -1e30, which
// holds exactly when fund2 > 0 (20 log10(sqrt(fund2)) - power_scale is finite for every
// positive fund2, -inf for 0, NaN for NaN), so they skip the log10f.
__device__ __forceinline__ float detect_findex(float fund2, cf L, cf R) {
  const float fundamental = sqrtf(fund2);
  const float left = lm_hypotf(L.re, L.im);
  const float right = lm_hypotf(R.re, R.im);
  const double demon = (2.0 * (double)fundamental) - (double)right - (double)left;
  return demon == 0.0 ? 0.0f : (float)(0.5 * (double)(right - left) / demon);
}

// LoRaDetector.hpp:60-71 for the winning bin: power p and fractional index.
// `fund2` = max |X|^2, `L`/`R` = the neighbour bins (wrap-around).
__device__ __forceinline__ void detect_tail(float fund2, cf L, cf R, float power_scale,
                                            float* p_out, float* findex_out) {
  const float fundamental = sqrtf(fund2);
  *p_out = 20.0f * lm_log10f(fundamental) - power_scale;
  const float left = lm_hypotf(L.re, L.im);
  const float right = lm_hypotf(R.re, R.im);
  const double demon = (2.0 * (double)fundamental) - (double)right - (double)left;
  if (demon == 0.0)
    *findex_out = 0.0f;
  else
    *findex_out = (float)(0.5 * (double)(right - left) / demon);
}

}  // namespace lora
