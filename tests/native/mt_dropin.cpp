// Two host threads through the C++ drop-in at once (include/lora_mi355x_phy.hpp): each thread
// initialises its own legacy workspace with the same spreading factor and window - so the two
// share the load-time runtime's plan and AQL queue (lora_phy_dropin.hip serialises them on the
// runtime's lock) - and demodulates its own noisy frames (different payloads, delays and
// amplitudes) `iters` times, every result compared with what the same thread computed alone
// before the threads started.  `mixed`: thread t at SF 7 + t (two plans, the one shared
// queue), each call preceded by a lora_modulate of the thread's packet compared with its
// first modulation.  Prints one JSON line; tests/test_gpu_dropin.py runs it.
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

namespace {

struct Frame {
  std::vector<std::complex<float>> dech, scratch, iq;
  std::vector<uint16_t> tx;
  std::vector<uint16_t> symbols;
  uint8_t sync = 0;
  float cfo = 0.0f, toff = 0.0f;
  size_t count = 0;
};

// a dechirped frame of `nsym` data symbols: payload seed, a delay of `delay` samples, noise
Frame make_frame(unsigned sf, unsigned seed, int delay, float amp, float noise) {
  const size_t N = size_t(1) << sf;
  std::vector<uint8_t> payload(16);
  for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)(seed * 31 + i * 7);
  std::vector<uint16_t> symbols(2 * payload.size() + 8);
  const size_t nsym = lora_phy::lora_encode(payload.data(), payload.size(), symbols.data(), sf);
  const size_t count = (nsym + 2) * N;
  std::vector<std::complex<float>> iq(count), down(N);
  lora_phy::lora_modulate(symbols.data(), nsym, iq.data(), sf, 1, lora_phy::bandwidth::bw_125, amp, 0x12);
  float ph = 0.0f;
  genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, lora_phy::bw_scale(lora_phy::bandwidth::bw_125));
  std::mt19937 rng(seed);
  std::normal_distribution<float> g(0.0f, noise);
  Frame fr;
  fr.count = count;
  fr.dech.resize(count);
  fr.scratch.resize(count);
  for (size_t j = 0; j < count; ++j) {
    const size_t src = j >= (size_t)delay ? j - delay : 0;
    fr.dech[j] = (iq[src] + std::complex<float>(g(rng), g(rng))) * down[j % N];
  }
  fr.symbols.resize(nsym);
  fr.iq = iq;
  fr.tx.assign(symbols.begin(), symbols.begin() + nsym);
  return fr;
}

bool demod(Frame& fr, unsigned sf, std::vector<uint16_t>& out, uint8_t& sync, float& cfo, float& toff) {
  lora_phy::lora_demod_workspace ws{};
  lora_phy::lora_demod_init(&ws, sf, lora_phy::window_type::window_none, fr.scratch.data(), fr.scratch.size());
  out.assign(fr.symbols.size(), 0);
  const size_t got = lora_phy::lora_demodulate(&ws, fr.dech.data(), fr.count, out.data(), 1, &sync);
  cfo = ws.metrics.cfo;
  toff = ws.metrics.time_offset;
  lora_phy::lora_demod_free(&ws);
  return got == fr.symbols.size();
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const bool mixed = argc > 2 && std::strcmp(argv[2], "mixed") == 0;
  constexpr int kThreads = 2, kFrames = 4;
  unsigned sfs[kThreads];
  std::vector<Frame> frames[kThreads];
  for (int t = 0; t < kThreads; ++t) {
    sfs[t] = mixed ? 7 + t : 7;
    for (int k = 0; k < kFrames; ++k)
      frames[t].push_back(make_frame(sfs[t], 100 * t + k, 3 * k + t, 1.0f + 0.5f * k, 0.3f + 0.1f * t));
  }
  // each frame alone first (the expected outputs)
  for (int t = 0; t < kThreads; ++t)
    for (Frame& fr : frames[t])
      if (!demod(fr, sfs[t], fr.symbols, fr.sync, fr.cfo, fr.toff)) return 2;
  std::atomic<long> calls{0}, bad{0};
  auto work = [&](int t) {
    std::vector<uint16_t> out;
    std::vector<std::complex<float>> iq;
    for (int i = 0; i < iters; ++i) {
      Frame& fr = frames[t][i % kFrames];
      if (mixed) {
        iq.assign(fr.iq.size(), std::complex<float>(0.0f, 0.0f));
        lora_phy::lora_modulate(fr.tx.data(), fr.tx.size(), iq.data(), sfs[t], 1, lora_phy::bandwidth::bw_125,
                                1.0f + 0.5f * (float)(i % kFrames), 0x12);
        if (std::memcmp(iq.data(), fr.iq.data(), iq.size() * sizeof(iq[0])) != 0) ++bad;
      }
      uint8_t sync = 0;
      float cfo = 0.0f, toff = 0.0f;
      const bool ok = demod(fr, sfs[t], out, sync, cfo, toff);
      ++calls;
      if (!ok || out != fr.symbols || sync != fr.sync || std::memcmp(&cfo, &fr.cfo, 4) != 0 ||
          std::memcmp(&toff, &fr.toff, 4) != 0)
        ++bad;
    }
  };
  std::thread th[kThreads];
  for (int t = 0; t < kThreads; ++t) th[t] = std::thread(work, t);
  for (auto& x : th) x.join();
  std::printf("{\"threads\": %d, \"calls\": %ld, \"mismatches\": %ld}\n", kThreads, calls.load(), bad.load());
  return bad.load() == 0 ? 0 : 1;
}
