// Host check of csrc/lora_libm.h against this machine's glibc, bit for bit.
// Test infrastructure (tests/test_libm_host.py builds and runs it).
//
//   libm_check <stride> <threads>
// sincosf: every `stride`-th float bit pattern (all signs and exponents), fast path
// variants over |y| < 120; atan2f / hypotf / log10f / logf over a hashed sample.
// Prints one line per function: "<name> <checked> <mismatches>".
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

#include "../../lora-sdr-lightweight-standalone-library-_amd/csrc/lora_libm.h"

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float flt(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
static bool same(float a, float b) { return bits(a) == bits(b) || (isnan(a) && isnan(b)); }

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 97;
  const int T = argc > 2 ? atoi(argv[2]) : 4;
  std::atomic<uint64_t> n_sc{0}, bad_sc{0}, n_fast{0}, bad_fast{0}, bad_fastk{0}, bad_nz{0}, bad_bf{0}, n_lg{0}, bad_lgr{0};
  std::atomic<uint64_t> n_o{0}, bad_at{0}, bad_hy{0}, bad_lg{0}, bad_l10{0};
  auto work = [&](int t) {
    uint64_t c_sc = 0, b_sc = 0, c_f = 0, b_f = 0, b_fk = 0, b_nz = 0, b_bf = 0, c_lg = 0, b_lgr = 0;
    for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += (uint64_t)T * stride) {
      const float y = flt((uint32_t)u);
      float s, c, s2, c2;
      sincosf(y, &s, &c);
      lm_sincosf(y, &s2, &c2);
      ++c_sc;
      if (!same(s, s2) || !same(c, c2)) ++b_sc;
      lm_sincosf_bf(y, &s2, &c2);
      if (!same(s, s2) || !same(c, c2)) ++b_bf;
      if (lm_sincosf_large_ok(y)) {
        ++c_lg;
        lm_sincosf_large(y, &s2, &c2);
        if (!same(s, s2) || !same(c, c2)) ++b_lgr;
      }
      if (lm_sincosf_fast_ok(y)) {
        ++c_f;
        lm_sincosf_fast(y, &s2, &c2);
        if (!same(s, s2) || !same(c, c2)) ++b_f;
        float yk[2] = {y, -y}, sk[2], ck[2];
        lm_sincosf_fast_k<2>(yk, sk, ck);
        if (!same(s, sk[0]) || !same(c, ck[0])) ++b_fk;
        lm_sincosf_fast_k_nz<2>(yk, sk, ck);
        // _nz: equal except the sign of a zero sine
        const bool sin_ok = same(s, sk[0]) || (s == 0.0f && sk[0] == 0.0f);
        if (!sin_ok || !same(c, ck[0])) ++b_nz;
      }
    }
    n_sc += c_sc; bad_sc += b_sc; n_fast += c_f; bad_fast += b_f; bad_fastk += b_fk; bad_nz += b_nz;
    bad_bf += b_bf;
    n_lg += c_lg;
    bad_lgr += b_lgr;
    uint64_t c_o = 0, b_a = 0, b_h = 0, b_l = 0, b_10 = 0;
    for (uint64_t i = t; i < 4000000; i += T) {
      const uint64_t h = mix(i * 0x9e3779b97f4a7c15ull + 12345);
      const float a = flt((uint32_t)h), b = flt((uint32_t)(h >> 32));
      ++c_o;
      if (!same(atan2f(a, b), lm_atan2f(a, b))) ++b_a;
      if (!same(hypotf(a, b), lm_hypotf(a, b))) ++b_h;
      if (!same(logf(fabsf(a)), lm_logf(fabsf(a)))) ++b_l;
      if (!same(log10f(fabsf(b)), lm_log10f(fabsf(b)))) ++b_10;
    }
    n_o += c_o; bad_at += b_a; bad_hy += b_h; bad_lg += b_l; bad_l10 += b_10;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  printf("sincosf %llu %llu\n", (unsigned long long)n_sc, (unsigned long long)bad_sc);
  printf("sincosf_bf %llu %llu\n", (unsigned long long)n_sc, (unsigned long long)bad_bf);
  printf("sincosf_large %llu %llu\n", (unsigned long long)n_lg, (unsigned long long)bad_lgr);
  printf("sincosf_fast %llu %llu\n", (unsigned long long)n_fast, (unsigned long long)bad_fast);
  printf("sincosf_fast_k %llu %llu\n", (unsigned long long)n_fast, (unsigned long long)bad_fastk);
  printf("sincosf_fast_k_nz %llu %llu\n", (unsigned long long)n_fast, (unsigned long long)bad_nz);
  printf("atan2f %llu %llu\n", (unsigned long long)n_o, (unsigned long long)bad_at);
  printf("hypotf %llu %llu\n", (unsigned long long)n_o, (unsigned long long)bad_hy);
  printf("logf %llu %llu\n", (unsigned long long)n_o, (unsigned long long)bad_lg);
  printf("log10f %llu %llu\n", (unsigned long long)n_o, (unsigned long long)bad_l10);
  return 0;
}
