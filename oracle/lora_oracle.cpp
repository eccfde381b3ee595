// lora_oracle.cpp — CPU restatement of the reference LoRa PHY hot path.
//
// *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker /
// CPU baseline.  The product path (lora_phy_amd + liblora_mi355x.so) never calls it.
//
// Every function restates one reference routine (cited as file:line relative to the
// reference checkout) with the same fp32 operation order, so that compiled with
// g++ -O2 -ffp-contract=off against the same glibc it reproduces the reference's
// outputs bit-for-bit.  Parity of this restatement with the reference itself is
// pinned by tests/test_oracle_vs_reference.py (compiled reference in oracle/_ref,
// this container only) and by the committed golden fixtures in tests/golden/.
//
// Complex arithmetic is written out explicitly: GCC lowers std::complex<float>
// products to (ac-bd, ad+bc) with no FMA on x86-64, which is what cmul() does.
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>
#include <random>

namespace {

struct cf {
  float re, im;
};
static inline cf cmul(cf a, cf b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
static inline cf cadd(cf a, cf b) { return {a.re + b.re, a.im + b.im}; }
static inline cf csub(cf a, cf b) { return {a.re - b.re, a.im - b.im}; }
static inline cf cscale(cf a, float s) { return {a.re * s, a.im * s}; }

const float PI_F = float(M_PI);
constexpr int MAX_N = 4096;  // kissfft.hh:34

// ChirpGenerator.hpp:105-132 (genChirp).  fMin/fMax/fStep are evaluated in double
// and narrowed to float, the recurrence runs in float, std::polar -> sincosf.
int gen_chirp(cf* out, int N, int osr, int NN, float f0, bool down, float ampl, float& phase,
              float bw_scale) {
  const float fMin = -M_PI * bw_scale / osr;
  const float fMax = M_PI * bw_scale / osr;
  const float fStep = (2 * M_PI * bw_scale) / (N * osr * osr);
  float f = fMin + f0;
  int i;
  for (i = 0; i < NN; i++) {
    f += fStep;
    if (f > fMax) f -= (fMax - fMin);
    if (down)
      phase -= f;
    else
      phase += f;
    float s, c;
    sincosf(phase, &s, &c);
    out[i] = {ampl * c, ampl * s};
  }
  phase -= std::floor(phase / (2 * M_PI)) * 2 * M_PI;
  return i;
}

// kissfft.hh:71-98 (init): twiddles exp(j*i*phinc) with phinc in float, and the
// radix plan "4 while divisible, then 2, then odd".
struct FftPlan {
  int nfft = 0;
  int stages = 0;
  int radix[32];
  int remain[32];
  cf tw[MAX_N];
};

void fft_plan_init(FftPlan& p, int nfft) {
  p.nfft = nfft;
  const float phinc = -2 * std::acos((float)-1) / nfft;
  for (int i = 0; i < nfft; ++i) {
    std::complex<float> t = std::exp(std::complex<float>(0, i * phinc));
    p.tw[i] = {t.real(), t.imag()};
  }
  int n = nfft, r = 4;
  p.stages = 0;
  do {
    while (n % r) {
      r = (r == 4) ? 2 : (r == 2) ? 3 : r + 2;
      if (r * r > n) r = n;
    }
    n /= r;
    p.radix[p.stages] = r;
    p.remain[p.stages] = n;
    ++p.stages;
  } while (n > 1);
}

// kissfft.hh:155-162 (kf_bfly2), forward.
void bfly2(const FftPlan& p, cf* F, size_t fs, int m) {
  for (int k = 0; k < m; ++k) {
    cf t = cmul(F[m + k], p.tw[k * fs]);
    F[m + k] = csub(F[k], t);
    F[k] = cadd(F[k], t);
  }
}

// kissfft.hh:164-185 (kf_bfly4), forward (negative_if_inverse = 1).
void bfly4(const FftPlan& p, cf* F, size_t fs, size_t m) {
  for (size_t k = 0; k < m; ++k) {
    cf s0 = cmul(F[k + m], p.tw[k * fs]);
    cf s1 = cmul(F[k + 2 * m], p.tw[k * fs * 2]);
    cf s2 = cmul(F[k + 3 * m], p.tw[k * fs * 3]);
    cf s5 = csub(F[k], s1);
    F[k] = cadd(F[k], s1);
    cf s3 = cadd(s0, s2);
    cf s4 = csub(s0, s2);
    s4 = {s4.im, -s4.re};
    F[k + 2 * m] = csub(F[k], s3);
    F[k] = cadd(F[k], s3);
    F[k + m] = cadd(s5, s4);
    F[k + 3 * m] = csub(s5, s4);
  }
}

// kissfft.hh:106-143 (kf_work): recursive decimation in time.  Only radix 4 and 2
// occur for N = 2^SF; other radices are rejected by the callers (SF 2..12).
void fft_work(const FftPlan& p, int stage, cf* out, const cf* f, size_t fs) {
  const int r = p.radix[stage];
  const int m = p.remain[stage];
  cf* beg = out;
  cf* end = out + r * m;
  if (m == 1) {
    do {
      *out = *f;
      f += fs;
    } while (++out != end);
  } else {
    do {
      fft_work(p, stage + 1, out, f, fs * r);
      f += fs;
    } while ((out += m) != end);
  }
  if (r == 2)
    bfly2(p, beg, fs, m);
  else
    bfly4(p, beg, fs, m);
}

void fft(const FftPlan& p, const cf* in, cf* out) { fft_work(p, 0, out, in, 1); }

// LoRaDetector.hpp:39-74 (detect): strict '>' argmax over |X|^2 (lowest index wins),
// power in dB, and the neighbour-magnitude fractional index.
size_t detect(const FftPlan& p, const cf* in, cf* out, float power_scale, float& power,
              float& fIndex) {
  const size_t N = (size_t)p.nfft;
  fft(p, in, out);
  size_t maxIndex = 0;
  float maxValue = 0;
  for (size_t i = 0; i < N; i++) {
    const float mag2 = out[i].re * out[i].re + out[i].im * out[i].im;
    if (mag2 > maxValue) {
      maxIndex = i;
      maxValue = mag2;
    }
  }
  const float fundamental = std::sqrt(maxValue);
  power = 20 * std::log10(fundamental) - power_scale;
  const cf L = out[maxIndex > 0 ? maxIndex - 1 : N - 1];
  const cf R = out[maxIndex < N - 1 ? maxIndex + 1 : 0];
  const float left = hypotf(L.re, L.im);
  const float right = hypotf(R.re, R.im);
  const double demon = (2.0 * fundamental) - right - left;
  if (demon == 0.0)
    fIndex = 0.0f;
  else
    fIndex = 0.5 * (right - left) / demon;
  return maxIndex;
}

struct DemodState {
  unsigned sf = 0;
  size_t N = 0;
  bool hann = false;
  float window[MAX_N];
  float power_scale = 0;
  FftPlan plan;
  cf fin[MAX_N];
  cf fout[MAX_N];
};

// LoRaDemod.cpp:10-32 (lora_demod_init): window + plan.
void demod_init(DemodState& st, unsigned sf, bool hann) {
  st.sf = sf;
  st.N = size_t(1) << sf;
  st.hann = hann;
  for (size_t i = 0; i < st.N; ++i)
    st.window[i] = hann ? 0.5f - 0.5f * std::cos(2.0f * PI_F * static_cast<float>(i) /
                                                 (static_cast<float>(st.N) - 1.0f))
                        : 1.0f;
  fft_plan_init(st.plan, (int)st.N);
  st.power_scale = 20 * std::log10(st.N);  // LoRaDetector.hpp:30 (double -> float)
}

struct Estimate {
  float cfo = 0, time_offset = 0;
};

// Shared 2-symbol offset estimate.  LoRaDemod.cpp:79-135 (legacy, with the
// "p == best_p && idx < best_idx" tie rule) and phy.cpp:97-145 (API twin, plain
// "p > best_p").  `nsym` is min(total,2) for the legacy path and the symbol count
// of the estimate window for the API path.
Estimate estimate(DemodState& st, const cf* x, size_t nsym, unsigned osr, bool tie_rule) {
  const size_t N = st.N, step = N * osr;
  float sum_index = 0.0f, phase_diff = 0.0f, prev_phase = 0.0f;
  bool have_prev = false;
  unsigned sum_t = 0;
  for (size_t s = 0; s < nsym; ++s) {
    const cf* base = x + s * step;
    float best_p = -1e30f, best_fi = 0.0f;
    size_t best_idx = 0;
    unsigned best_t = 0;
    cf best_bin = {0.0f, 0.0f};
    for (unsigned t = 0; t < osr; ++t) {
      for (size_t i = 0; i < N; ++i) {
        cf v = base[t + i * osr];
        if (st.hann) v = cscale(v, st.window[i]);
        st.fin[i] = v;
      }
      float pw, fi;
      const size_t idx = detect(st.plan, st.fin, st.fout, st.power_scale, pw, fi);
      if (pw > best_p || (tie_rule && pw == best_p && idx < best_idx)) {
        best_p = pw;
        best_idx = idx;
        best_fi = fi;
        best_t = t;
        best_bin = st.fout[idx];
      }
    }
    sum_t += best_t;
    sum_index += static_cast<float>(best_idx) + best_fi;
    const float phase = std::atan2(best_bin.im, best_bin.re);
    if (have_prev) {
      float d = phase - prev_phase;
      while (d > PI_F) d -= 2.0f * PI_F;
      while (d < -PI_F) d += 2.0f * PI_F;
      phase_diff += d;
    }
    prev_phase = phase;
    have_prev = true;
  }
  Estimate e;
  const float avg_index = sum_index / static_cast<float>(nsym);
  const float cfo_coarse = avg_index / static_cast<float>(N);
  float cfo_fine = 0.0f;
  if (nsym > 1)
    cfo_fine = (phase_diff / static_cast<float>(nsym - 1)) / (2.0f * PI_F * static_cast<float>(N));
  e.cfo = cfo_coarse + cfo_fine;
  const float frac = avg_index - std::floor(avg_index + 0.5f);
  const float avg_t = static_cast<float>(sum_t) / static_cast<float>(nsym);
  e.time_offset = avg_t - frac * static_cast<float>(N) * static_cast<float>(osr);
  return e;
}

// LoRaDemod.cpp:49-195 (lora_demodulate).  Returns the symbol count (total-2 with a
// sync pair, else total), or 0 when rescaling is needed but scratch_len is short
// (LoRaDemod.cpp:69-71).
size_t lora_demodulate(DemodState& st, const cf* samples, size_t count, uint16_t* out_syms,
                       unsigned osr, uint8_t* out_sync, size_t scratch_len, std::vector<cf>& scratch,
                       float* out_cfo, float* out_toff) {
  const size_t N = st.N, step = N * osr;
  const size_t total = count / step;
  const bool have_sync = total >= 2;
  const cf* x = samples;
  float max_amp = 0.0f;
  for (size_t i = 0; i < count; ++i) {
    const float m = std::max(std::fabs(samples[i].re), std::fabs(samples[i].im));
    if (m > max_amp) max_amp = m;
  }
  if (max_amp > 1.0f) {
    if (scratch_len < count) return 0;
    const float scale = 1.0f / max_amp;
    scratch.resize(count);
    for (size_t i = 0; i < count; ++i) scratch[i] = cscale(samples[i], scale);
    x = scratch.data();
  }
  const size_t est_syms = std::min(total, size_t(2));
  const Estimate e = estimate(st, x, est_syms, osr, true);
  if (out_cfo) *out_cfo = e.cfo;
  if (out_toff) *out_toff = e.time_offset;

  const int t_off = static_cast<int>(std::round(e.time_offset));
  const float rate = -2.0f * PI_F * e.cfo / static_cast<float>(N);
  uint16_t sw0 = 0, sw1 = 0;
  size_t out_idx = 0;
  for (size_t s = 0; s < total; ++s) {
    size_t base = s * step;
    if (t_off > 0) {
      if (base + size_t(t_off) + step <= count) base += size_t(t_off);
    } else if (t_off < 0) {
      const size_t off = size_t(-t_off);
      if (off <= base) base -= off;
    }
    const float start =
        rate * (static_cast<float>(s * N) + static_cast<float>(t_off) / static_cast<float>(osr));
    for (size_t i = 0; i < N; ++i) {
      const float ph = start + rate * static_cast<float>(i);
      float sn, cs;
      sincosf(ph, &sn, &cs);
      cf v = cmul(x[base + i * osr], cf{cs, sn});
      if (st.hann) v = cscale(v, st.window[i]);
      st.fin[i] = v;
    }
    float pw, fi;
    const uint16_t idx = (uint16_t)detect(st.plan, st.fin, st.fout, st.power_scale, pw, fi);
    if (have_sync && s == 0)
      sw0 = idx;
    else if (have_sync && s == 1)
      sw1 = idx;
    else
      out_syms[out_idx++] = idx;
  }
  if (out_sync) {
    if (have_sync) {
      const unsigned shift = st.sf > 4 ? st.sf - 4 : 0;
      *out_sync = (uint8_t)((((sw0 >> shift) & 0x0f) << 4) | ((sw1 >> shift) & 0x0f));
    } else {
      *out_sync = 0;
    }
  }
  return have_sync ? out_idx : total;
}

// LoRaMod.cpp:8-41 (lora_modulate).
size_t lora_modulate(const uint16_t* syms, size_t count, cf* out, unsigned sf, unsigned osr,
                     float bw_scale, float amplitude, uint8_t sync) {
  const size_t N = size_t(1) << sf, step = N * osr;
  float phase = 0.0f;
  amplitude = std::max(-1.0f, std::min(1.0f, amplitude));
  const unsigned shift = sf > 4 ? sf - 4 : 0;
  const uint16_t sw0 = (uint16_t)((sync >> 4) << shift);
  const uint16_t sw1 = (uint16_t)((sync & 0x0f) << shift);
  const float den = float(N) * static_cast<float>(osr);
  const float f0 = (2.0f * PI_F * sw0 * bw_scale) / den;
  gen_chirp(out, (int)N, (int)osr, (int)step, f0, false, amplitude, phase, bw_scale);
  const float f1 = (2.0f * PI_F * sw1 * bw_scale) / den;
  gen_chirp(out + step, (int)N, (int)osr, (int)step, f1, false, amplitude, phase, bw_scale);
  for (size_t s = 0; s < count; ++s) {
    const float freq = (2.0f * PI_F * syms[s] * bw_scale) / den;
    gen_chirp(out + (s + 2) * step, (int)N, (int)osr, (int)step, freq, false, amplitude, phase,
              bw_scale);
  }
  return (count + 2) * step;
}

// phy.cpp:78-145 (estimate_offsets) on the raw samples of the first 2 symbols.
// phy.cpp:178-239 (demodulate): fused per-symbol downchirp (osr 1 generator), CFO
// rotation, window; returns total-2 or -1.
long api_demodulate(DemodState& st, unsigned osr, float bw_scale, const cf* iq, size_t count,
                    uint16_t* syms, size_t cap, uint8_t* out_sync, float* out_cfo, float* out_toff) {
  const size_t N = st.N, step = N * osr;
  if (count % step != 0) return -1;
  const size_t total = count / step;
  if (total < 2) return -1;
  const size_t num = total - 2;
  if (num > cap) return -1;
  const size_t est_samples = std::min(count, step * 2);
  const Estimate e = estimate(st, iq, est_samples / step, osr, false);
  if (out_cfo) *out_cfo = e.cfo;
  if (out_toff) *out_toff = e.time_offset;
  const int t_off = static_cast<int>(std::round(e.time_offset));
  const float rate = -2.0f * PI_F * e.cfo / static_cast<float>(N);
  static thread_local cf down[MAX_N];
  uint16_t sw0 = 0, sw1 = 0;
  for (size_t s = 0; s < total; ++s) {
    float tmp = 0.0f;
    gen_chirp(down, (int)N, 1, (int)N, 0.0f, true, 1.0f, tmp, bw_scale);
    size_t base = s * step;
    if (t_off > 0) {
      if (base + size_t(t_off) + step <= count) base += size_t(t_off);
    } else if (t_off < 0) {
      const size_t off = size_t(-t_off);
      if (off <= base) base -= off;
    }
    const float start =
        rate * (static_cast<float>(s * N) + static_cast<float>(t_off) / static_cast<float>(osr));
    for (size_t i = 0; i < N; ++i) {
      const float ph = start + rate * static_cast<float>(i);
      float sn, cs;
      sincosf(ph, &sn, &cs);
      cf v = cmul(cmul(iq[base + i * osr], down[i]), cf{cs, sn});
      if (st.hann) v = cscale(v, st.window[i]);
      st.fin[i] = v;
    }
    float pw, fi;
    const uint16_t idx = (uint16_t)detect(st.plan, st.fin, st.fout, st.power_scale, pw, fi);
    if (s == 0)
      sw0 = idx;
    else if (s == 1)
      sw1 = idx;
    else
      syms[s - 2] = idx;
  }
  const unsigned shift = st.sf > 4 ? st.sf - 4 : 0;
  if (out_sync) *out_sync = (uint8_t)((((sw0 >> shift) & 0x0f) << 4) | ((sw1 >> shift) & 0x0f));
  return (long)num;
}

// phy.cpp:147-176 (compensate_offsets), in place.
void compensate_offsets(unsigned sf, unsigned osr, float cfo, float to, cf* x, size_t count) {
  const size_t N = size_t(1) << sf;
  const float rate = -2.0f * PI_F * cfo / (static_cast<float>(N) * static_cast<float>(osr));
  for (size_t n = 0; n < count; ++n) {
    const float ph = rate * static_cast<float>(n);
    float sn, cs;
    sincosf(ph, &sn, &cs);
    x[n] = cmul(x[n], cf{cs, sn});
  }
  const int offset = static_cast<int>(std::round(to));
  if (offset > 0 && size_t(offset) < count) {
    for (size_t n = count; n-- > size_t(offset);) x[n] = x[n - size_t(offset)];
    for (size_t n = 0; n < size_t(offset); ++n) x[n] = {0.0f, 0.0f};
  } else if (offset < 0 && size_t(-offset) < count) {
    const size_t off = size_t(-offset);
    for (size_t n = 0; n + off < count; ++n) x[n] = x[n + off];
    for (size_t n = count - off; n < count; ++n) x[n] = {0.0f, 0.0f};
  }
}

// ---- LoRaCodes.hpp restatements (host-side chain) ----
uint8_t enc_h84(uint8_t x) {  // LoRaCodes.hpp:229-242
  const unsigned d0 = x & 1, d1 = (x >> 1) & 1, d2 = (x >> 2) & 1, d3 = (x >> 3) & 1;
  uint8_t b = x & 0xf;
  b |= (d0 ^ d1 ^ d2) << 4;
  b |= (d1 ^ d2 ^ d3) << 5;
  b |= (d0 ^ d1 ^ d3) << 6;
  b |= (d0 ^ d2 ^ d3) << 7;
  return b;
}
uint8_t dec_h84(uint8_t b, bool& err, bool& bad) {  // LoRaCodes.hpp:250-281
  const unsigned b0 = b & 1, b1 = (b >> 1) & 1, b2 = (b >> 2) & 1, b3 = (b >> 3) & 1;
  const unsigned b4 = (b >> 4) & 1, b5 = (b >> 5) & 1, b6 = (b >> 6) & 1, b7 = (b >> 7) & 1;
  const unsigned p = (b0 ^ b1 ^ b2 ^ b4) | ((b1 ^ b2 ^ b3 ^ b5) << 1) | ((b0 ^ b1 ^ b3 ^ b6) << 2) |
                     ((b0 ^ b2 ^ b3 ^ b7) << 3);
  if (p) err = true;
  switch (p) {
    case 0xD: return (b ^ 1) & 0xf;
    case 0x7: return (b ^ 2) & 0xf;
    case 0xB: return (b ^ 4) & 0xf;
    case 0xE: return (b ^ 8) & 0xf;
    case 0x0: case 0x1: case 0x2: case 0x4: case 0x8: return b & 0xf;
    default: bad = true; return b & 0xf;
  }
}

}  // namespace

// ============================ C ABI (ctypes) ===================================
extern "C" {

int orc_gen_chirp(float* out_iq, int N, int osr, int NN, float f0, int down, float ampl,
                  float* phase, float bw_scale) {
  return gen_chirp(reinterpret_cast<cf*>(out_iq), N, osr, NN, f0, down != 0, ampl, *phase, bw_scale);
}

// Forward FFT exactly as kissfft<float> (N = 2^k, 4 <= N <= 4096).
int orc_fft(const float* in_iq, float* out_iq, int N) {
  static thread_local FftPlan p;
  if (p.nfft != N) fft_plan_init(p, N);
  fft(p, reinterpret_cast<const cf*>(in_iq), reinterpret_cast<cf*>(out_iq));
  return 0;
}

// Twiddle table of the forward plan (kissfft.hh:24-29) and the factor list.
int orc_fft_twiddles(float* out_iq, int N) {
  FftPlan p;
  fft_plan_init(p, N);
  std::memcpy(out_iq, p.tw, sizeof(cf) * N);
  return p.stages;
}

size_t orc_lora_modulate(const uint16_t* syms, size_t count, float* out_iq, unsigned sf,
                         unsigned osr, float bw_scale, float amplitude, uint8_t sync) {
  return lora_modulate(syms, count, reinterpret_cast<cf*>(out_iq), sf, osr, bw_scale, amplitude, sync);
}

// Caller-side dechirp of e2e_chain_test.cpp:85-93: y[j] = x[j] * down[j % (N*osr)]
// for the whole symbols, with down = genChirp(N, osr, N*osr, 0, down=true, 1).
void orc_dechirp(const float* in_iq, float* out_iq, size_t count, unsigned sf, unsigned osr,
                 float bw_scale) {
  const size_t N = size_t(1) << sf, step = N * osr;
  std::vector<cf> down(step);
  float phase = 0.0f;
  gen_chirp(down.data(), (int)N, (int)osr, (int)step, 0.0f, true, 1.0f, phase, bw_scale);
  const cf* x = reinterpret_cast<const cf*>(in_iq);
  cf* y = reinterpret_cast<cf*>(out_iq);
  for (size_t j = 0; j < count; ++j) y[j] = cmul(x[j], down[j % step]);
}

// One lora_demodulate call (single frame).  hann: 0/1.  Returns produced symbols.
size_t orc_lora_demodulate(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                           uint16_t* out_syms, uint8_t* out_sync, float* out_cfo, float* out_toff,
                           size_t scratch_len) {
  static thread_local DemodState st;
  static thread_local std::vector<cf> scratch;
  if (st.sf != sf || st.hann != (hann != 0) || st.N == 0) demod_init(st, sf, hann != 0);
  return lora_demodulate(st, reinterpret_cast<const cf*>(iq), count, out_syms, osr, out_sync,
                         scratch_len, scratch, out_cfo, out_toff);
}

// Batched frames [F][frame_len] with optional fused dechirp, over `threads` host
// threads (frames striped).  sym_stride entries per frame in out_syms.
void orc_demod_frames(const float* iq, size_t frames, size_t frame_len, unsigned sf, int hann,
                      unsigned osr, int dechirp, float bw_scale, uint16_t* out_syms,
                      size_t sym_stride, uint8_t* out_sync, float* out_cfo, float* out_toff,
                      int64_t* out_count, int threads) {
  if (threads < 1) threads = 1;
  auto worker = [&](int tid) {
    DemodState* st = new DemodState();
    demod_init(*st, sf, hann != 0);
    std::vector<cf> scratch, dech(dechirp ? frame_len : 0), down;
    const size_t N = size_t(1) << sf, step = N * osr;
    if (dechirp) {
      down.resize(step);
      float ph = 0.0f;
      gen_chirp(down.data(), (int)N, (int)osr, (int)step, 0.0f, true, 1.0f, ph, bw_scale);
    }
    for (size_t f = (size_t)tid; f < frames; f += (size_t)threads) {
      const cf* x = reinterpret_cast<const cf*>(iq) + f * frame_len;
      if (dechirp) {
        for (size_t j = 0; j < frame_len; ++j) dech[j] = cmul(x[j], down[j % step]);
        x = dech.data();
      }
      uint8_t sync = 0;
      float cfo = 0, toff = 0;
      const size_t n = lora_demodulate(*st, x, frame_len, out_syms + f * sym_stride, osr, &sync,
                                       frame_len, scratch, &cfo, &toff);
      if (out_sync) out_sync[f] = sync;
      if (out_cfo) out_cfo[f] = cfo;
      if (out_toff) out_toff[f] = toff;
      if (out_count) out_count[f] = (int64_t)n;
    }
    delete st;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
}

// LORA_MODE_RAW checker: the detector primitive alone per whole symbol
// (LoRaDetector.hpp:39-58 on the (caller-dechirped, e2e_chain_test.cpp:88-93) and
// windowed samples; no normalisation, estimate or rotation) - the demodulator of
// tests/awgn_sweep.py:262-265 in fp32.  Returns the number of symbols.
size_t orc_raw_demod(const float* iq, size_t count, unsigned sf, int hann, unsigned osr, int dechirp,
                     float bw_scale, uint16_t* out_syms) {
  static thread_local DemodState st;
  if (st.sf != sf || st.hann != (hann != 0) || st.N == 0) demod_init(st, sf, hann != 0);
  if (osr == 0) osr = 1;
  const size_t N = st.N, step = N * osr, total = count / step;
  std::vector<cf> down;
  if (dechirp) {
    down.resize(step);
    float ph = 0.0f;
    gen_chirp(down.data(), (int)N, (int)osr, (int)step, 0.0f, true, 1.0f, ph, bw_scale);
  }
  const cf* x = reinterpret_cast<const cf*>(iq);
  for (size_t s = 0; s < total; ++s) {
    for (size_t i = 0; i < N; ++i) {
      const size_t j = s * step + i * osr;
      cf v = x[j];
      if (dechirp) v = cmul(v, down[j % step]);
      st.fin[i] = cscale(v, st.window[i]);
    }
    float p, fi;
    out_syms[s] = (uint16_t)detect(st.plan, st.fin, st.fout, st.power_scale, p, fi);
  }
  return total;
}

long orc_api_demodulate(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                        float bw_scale, uint16_t* syms, size_t cap, uint8_t* out_sync,
                        float* out_cfo, float* out_toff) {
  static thread_local DemodState st;
  if (st.sf != sf || st.hann != (hann != 0) || st.N == 0) demod_init(st, sf, hann != 0);
  return api_demodulate(st, osr, bw_scale, reinterpret_cast<const cf*>(iq), count, syms, cap,
                        out_sync, out_cfo, out_toff);
}

void orc_estimate_offsets(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                          float* out_cfo, float* out_toff) {
  static thread_local DemodState st;
  if (st.sf != sf || st.hann != (hann != 0) || st.N == 0) demod_init(st, sf, hann != 0);
  const size_t step = (size_t(1) << sf) * osr;
  if (count == 0 || count / step == 0) return;  // phy.cpp:81,87
  const Estimate e = estimate(st, reinterpret_cast<const cf*>(iq), count / step, osr, false);
  *out_cfo = e.cfo;
  *out_toff = e.time_offset;
}

void orc_compensate_offsets(float* iq, size_t count, unsigned sf, unsigned osr, float cfo, float to) {
  compensate_offsets(sf, osr, cfo, to, reinterpret_cast<cf*>(iq), count);
}

// LoRaEncoder.cpp:8-19 / LoRaDecoder.cpp:8-19.
size_t orc_lora_encode(const uint8_t* bytes, size_t n, uint16_t* out) {
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    out[k++] = enc_h84(bytes[i] >> 4);
    out[k++] = enc_h84(bytes[i] & 0x0f);
  }
  return k;
}
size_t orc_lora_decode(const uint16_t* syms, size_t n, uint8_t* out) {
  size_t k = 0;
  for (size_t i = 0; i + 1 < n; i += 2) {
    bool e = false, b = false;
    const uint8_t hi = dec_h84((uint8_t)syms[i], e, b) & 0x0f;
    e = b = false;
    const uint8_t lo = dec_h84((uint8_t)syms[i + 1], e, b) & 0x0f;
    out[k++] = (uint8_t)((hi << 4) | lo);
  }
  return k;
}

// awgn_sweep_gtest.cpp:52-108 restated without gtest: for each packet, payload
// bytes rng()&0xFF, encode, modulate (osr 1, amplitude 1, sync 0x12), add
// normal_distribution<float>(0, sigma/sqrt2) noise (re then im per sample) from the
// same std::mt19937(0) stream, shared across profiles.  Writes the noisy raw IQ of
// every packet back to back and the payloads.
size_t orc_awgn_gtest_frames(const unsigned* sfs, const float* bw_scales, int nprof, int packets,
                             int payload_size, double snr_db, float* out_iq, uint8_t* out_payload) {
  std::mt19937 rng(0);
  size_t off = 0, poff = 0;
  for (int p = 0; p < nprof; ++p) {
    const size_t N = size_t(1) << sfs[p];
    for (int k = 0; k < packets; ++k) {
      std::vector<uint8_t> payload(payload_size);
      for (auto& b : payload) b = static_cast<uint8_t>(rng() & 0xFF);
      std::vector<uint16_t> syms(payload_size * 2);
      const size_t ns = orc_lora_encode(payload.data(), payload.size(), syms.data());
      const size_t count = (ns + 2) * N;
      std::vector<cf> s(count);
      lora_modulate(syms.data(), ns, s.data(), sfs[p], 1, bw_scales[p], 1.0f, 0x12);
      const double sigma = std::pow(10.0, -snr_db / 20.0);
      std::normal_distribution<float> noise(0.0f, static_cast<float>(sigma / std::sqrt(2.0)));
      for (auto& v : s) {
        // Same statement shape as awgn_sweep_gtest.cpp:80 so g++ picks the same
        // (unspecified) argument evaluation order for the two draws.
        const std::complex<float> n(noise(rng), noise(rng));
        v.re += n.real();
        v.im += n.imag();
      }
      if (out_iq) std::memcpy(out_iq + 2 * off, s.data(), sizeof(cf) * count);
      if (out_payload) std::memcpy(out_payload + poff, payload.data(), payload.size());
      off += count;
      poff += payload.size();
    }
  }
  return off;
}

}  // extern "C"
