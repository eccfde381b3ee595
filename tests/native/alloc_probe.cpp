// Host allocations (global operator new, as counted by the reference's
// tests/alloc_tracker.h) made by each drop-in call and by each HIP step of one
// lora_demodulate, on the GPU.  Prints one JSON line; tests/test_gpu_dropin.py records
// it next to the reference's own no_alloc_test run.  Built by the package Makefile.
#include <hip/hip_runtime.h>
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <vector>

#include "../../include/lora_mi355x.h"

static std::atomic<size_t> g_news{0};
void* operator new(size_t n) {
  g_news.fetch_add(1, std::memory_order_relaxed);
  if (void* p = std::malloc(n ? n : 1)) return p;
  throw std::bad_alloc();
}
void* operator new[](size_t n) {
  g_news.fetch_add(1, std::memory_order_relaxed);
  if (void* p = std::malloc(n ? n : 1)) return p;
  throw std::bad_alloc();
}
void operator delete(void* p) noexcept { std::free(p); }
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete(void* p, size_t) noexcept { std::free(p); }
void operator delete[](void* p, size_t) noexcept { std::free(p); }

struct Count {
  size_t start = g_news.load();
  size_t get() const { return g_news.load() - start; }
};

int main() {
  const unsigned sf = 7;
  const size_t N = size_t(1) << sf;
  const uint16_t syms[5] = {0, 1, 12, 34, 56};  // no_alloc_test.cpp:35
  const size_t count = (5 + 2) * N;
  std::vector<std::complex<float>> samples(count), dechirped(count), scratch(count), down(N);
  std::vector<uint16_t> demod(5);
  size_t mod1, mod2, init, dem[3], steps[4];
  {
    Count c;
    lora_phy::lora_modulate(syms, 5, samples.data(), sf, 1, lora_phy::bandwidth::bw_125, 1.0f, 0x12);
    mod1 = c.get();
  }
  {
    Count c;
    lora_phy::lora_modulate(syms, 5, samples.data(), sf, 1, lora_phy::bandwidth::bw_125, 1.0f, 0x12);
    mod2 = c.get();
  }
  float ph = 0.0f;
  genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, 1.0f);
  for (size_t i = 0; i < count; ++i) dechirped[i] = samples[i] * down[i % N];
  lora_phy::lora_demod_workspace ws{};
  {
    Count c;
    lora_phy::lora_demod_init(&ws, sf, lora_phy::window_type::window_none, scratch.data(), scratch.size());
    init = c.get();
  }
  const bool aql = ws.gpu.aql != nullptr;  // frames dispatched on the private AQL queue
  const int aql_status = ws.gpu.aql_status;
  bool ok = true;
  for (int k = 0; k < 3; ++k) {
    Count c;
    const size_t got = lora_phy::lora_demodulate(&ws, dechirped.data(), count, demod.data(), 1, nullptr);
    dem[k] = c.get();
    ok = ok && got == 5;
    for (int i = 0; i < 5; ++i) ok = ok && demod[i] == syms[i];
  }
  // the HIP steps of one call, separately: pinned H2D copy, the kernels, D2H, sync
  {
    void *dev = nullptr, *host = nullptr;
    hipStream_t st = nullptr;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    (void)hipMalloc(&dev, 1 << 20);
    (void)hipHostMalloc(&host, 1 << 20, hipHostMallocDefault);
    lora_demod_params p{sf, 1, 125000, LORA_WINDOW_NONE, 0, LORA_MODE_LEGACY, 0, LORA_PRECISION_EXACT};
    lora_demod_plan* plan = nullptr;
    lora_demod_plan_create(&p, &plan);
    unsigned char* d = static_cast<unsigned char*>(dev);
    lora_demod_outputs o{reinterpret_cast<uint16_t*>(d + 65536), 5, d + 66560, reinterpret_cast<float*>(d + 66816),
                         reinterpret_cast<float*>(d + 67072), reinterpret_cast<float*>(d + 67328)};
    const size_t wsb = lora_demod_workspace_bytes(plan, 1, (int64_t)count);
    for (int warm = 0; warm < 2; ++warm) {
      size_t c0 = g_news.load();
      (void)hipMemcpyAsync(dev, host, count * 8, hipMemcpyHostToDevice, st);
      size_t c1 = g_news.load();
      lora_demod_batch(plan, reinterpret_cast<const float*>(dev), 1, (int64_t)count, (int64_t)count, &o,
                       d + 131072, wsb, st);
      size_t c2 = g_news.load();
      (void)hipMemcpyAsync(host, d + 65536, 10, hipMemcpyDeviceToHost, st);
      size_t c3 = g_news.load();
      (void)hipStreamSynchronize(st);
      size_t c4 = g_news.load();
      steps[0] = c1 - c0;
      steps[1] = c2 - c1;
      steps[2] = c3 - c2;
      steps[3] = c4 - c3;
    }
    lora_demod_plan_destroy(plan);
    (void)hipFree(dev);
    (void)hipHostFree(host);
    (void)hipStreamDestroy(st);
  }
  lora_phy::lora_demod_free(&ws);
  std::printf("{\"dropin_status\": %d, ", lora_phy_dropin_status());
  std::printf("\"roundtrip_ok\": %s, \"aql_queue\": %s, \"aql_status\": %d, \"lora_modulate_first\": %zu, \"lora_modulate_second\": %zu, "
              "\"lora_demod_init\": %zu, \"lora_demodulate\": [%zu, %zu, %zu], \"hip_steps_second_call\": "
              "{\"memcpy_h2d_pinned\": %zu, \"lora_demod_batch\": %zu, \"memcpy_d2h_pinned\": %zu, "
              "\"stream_sync\": %zu}}\n",
              ok ? "true" : "false", aql ? "true" : "false", aql_status, mod1, mod2, init, dem[0], dem[1], dem[2], steps[0], steps[1], steps[2], steps[3]);
  return ok ? 0 : 1;
}
