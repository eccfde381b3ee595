// Where a drop-in packet's time goes: performance_test.cpp:103-121's loop (lora_modulate,
// the caller's dechirp, lora_demodulate per packet, host buffers) with each phase timed,
// and - with LORA_MI355X_AQL_PROFILE=1 - the private AQL queue's timeline of each call
// (doorbell -> packet start/end -> the host seeing the completion).  Prints one JSON line
// per spreading factor (medians over the timed packets).  Built by the package Makefile;
// tests/test_gpu_dropin.py runs it beside the reference's own performance_test.
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/lora_mi355x.h"

namespace {

double median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// one call's AQL timeline, appended as JSON: [[start, end], ...], seen
std::string timeline() {
  double t[64];
  const int n = lora_aql_last_profile(t, 64);
  if (n <= 0) return "null";
  const int k = (int)t[0];
  std::string s = "{\"packets\": [";
  char buf[96];
  for (int i = 0; i < k; ++i) {
    std::snprintf(buf, sizeof buf, "%s[%.2f, %.2f]", i ? ", " : "", t[1 + 2 * i], t[2 + 2 * i]);
    s += buf;
  }
  std::snprintf(buf, sizeof buf, "], \"seen\": %.2f}", t[1 + 2 * k]);
  return s + buf;
}

}  // namespace

int main(int argc, char** argv) {
  const int packets = argc > 1 ? std::atoi(argv[1]) : 300;
  const int warm = 20;
  for (unsigned sf : {7u, 8u, 9u, 12u}) {
    const size_t N = size_t(1) << sf;
    std::vector<uint8_t> payload(32);
    for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)i;
    std::vector<uint16_t> symbols(64);
    const size_t ns = lora_phy::lora_encode(payload.data(), payload.size(), symbols.data(), sf);
    const size_t count = (ns + 2) * N;
    std::vector<std::complex<float>> samples(count), dechirped(count), scratch(count), down(N);
    std::vector<uint16_t> demod(ns);
    float ph = 0.0f;
    genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, 1.0f);
    lora_phy::lora_demod_workspace ws{};
    lora_phy::lora_demod_init(&ws, sf, lora_phy::window_type::window_none, scratch.data(), scratch.size());
    const int n = sf >= 12 ? std::max(packets / 10, 20) : packets;
    std::vector<double> tm, td, tdm, tall, phs[8];
    std::string mod_tl = "null", dem_tl = "null";
    bool ok = true;
    for (int p = 0; p < warm + n; ++p) {
      const double t0 = now_us();
      lora_phy::lora_modulate(symbols.data(), ns, samples.data(), sf, 1, lora_phy::bandwidth::bw_125, 1.0f, 0x12);
      const double t1 = now_us();
      if (p == warm + n - 1) mod_tl = timeline();
      const double t2 = now_us();
      for (size_t s = 0; s < ns + 2; ++s)
        for (size_t i = 0; i < N; ++i) dechirped[s * N + i] = samples[s * N + i] * down[i];
      const double t3 = now_us();
      lora_phy::lora_demodulate(&ws, dechirped.data(), count, demod.data(), 1, nullptr);
      const double t4 = now_us();
      if (p == warm + n - 1) dem_tl = timeline();
      if (p >= warm) {
        double b[8];
        lora_phy_dropin_last_timing(b);
        for (int k = 0; k < 8; ++k) phs[k].push_back(b[k]);
        tm.push_back(t1 - t0);
        td.push_back(t3 - t2);
        tdm.push_back(t4 - t3);
        tall.push_back((t1 - t0) + (t3 - t2) + (t4 - t3));
      }
      for (size_t i = 0; i < ns; ++i) ok = ok && demod[i] == symbols[i] % N;  // codewords >= N wrap
    }
    lora_phy::lora_demod_free(&ws);
    std::printf(
        "{\"sf\": %u, \"packets\": %d, \"symbols_ok\": %s, \"modulate_us\": %.2f, \"dechirp_us\": %.2f, "
        "\"demodulate_us\": %.2f, \"packet_us\": %.2f, \"pps\": %.1f, "
        "\"demodulate_phases_us\": {\"copy_in\": %.2f, \"host_logic\": %.2f, \"aql_run\": %.2f, \"copy_out\": %.2f}, "
        "\"modulate_phases_us\": {\"copy_in\": %.2f, \"host_logic\": %.2f, \"aql_run\": %.2f, \"copy_out\": %.2f}, "
        "\"modulate_aql\": %s, \"demodulate_aql\": %s}\n",
        sf, n, ok ? "true" : "false", median(tm), median(td), median(tdm), median(tall), 1e6 / median(tall),
        median(phs[0]), median(phs[1]), median(phs[2]), median(phs[3]), median(phs[4]), median(phs[5]), median(phs[6]),
        median(phs[7]), mod_tl.c_str(), dem_tl.c_str());
    std::fflush(stdout);
  }
  return 0;
}
