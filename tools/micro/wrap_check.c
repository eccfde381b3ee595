// Host check behind lora_capi.hip mf_wrap: floor(p / (2 pi)) against floor(p * (1 / (2 pi))) in
// double for every finite float p (all 2^32 bit patterns).  gcc -O2 -fopenmp wrap_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <omp.h>
int main(void) {
  const double d = 2 * M_PI, inv = 1.0 / d;
  float minbad = INFINITY; uint64_t nbad = 0;
#pragma omp parallel for reduction(min:minbad) reduction(+:nbad) schedule(static)
  for (int64_t u = 0; u < (1ll << 32); ++u) {
    uint32_t b = (uint32_t)u; float p; memcpy(&p, &b, 4);
    if (!isfinite(p)) continue;
    const double q1 = floor((double)p / d), q2 = floor((double)p * inv);
    if (q1 != q2) { nbad++; if (fabsf(p) < minbad) minbad = fabsf(p); }
  }
  printf("inv=%.17g mismatches=%llu smallest |p| mismatching=%.9g (2^%.3f)\n", inv, (unsigned long long)nbad, minbad, log2(minbad));
  return 0;
}
