// The reference's workspace API (<lora_phy/phy.hpp>, phy.cpp:26-261) through the C++
// drop-in, with runners/rx_runner.cpp:102-122's call sequence: init -> demodulate ->
// decode -> get_last_metrics, then estimate_offsets and compensate_offsets on the same
// frame; and tx_runner.cpp's encode -> modulate.  Built by the package Makefile against
// liblora_mi355x.so; tests/test_gpu_dropin.py runs it on the GPU and compares with the
// reference's outputs (tests/golden/golden.json["api"]) and the oracle.
//   rx_dropin rx <sf> <osr> <hann 0|1> <in.iq> <compensated_out.iq>
//   rx_dropin tx <sf> <osr> <payload hex> <out.iq>
// IQ files are interleaved float32 (rx_runner.cpp:72-79, tx_runner.cpp:133-138).
#include <lora_phy/phy.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace lora_phy;

static uint32_t fbits(float v) {
  uint32_t b;
  std::memcpy(&b, &v, 4);
  return b;
}

static int rx(unsigned sf, unsigned osr, bool hann, const char* in, const char* out) {
  std::FILE* fh = std::fopen(in, "rb");
  if (!fh) return 2;
  std::vector<std::complex<float>> samples;
  std::complex<float> v;
  while (std::fread(&v, sizeof(v), 1, fh) == 1) samples.push_back(v);
  std::fclose(fh);
  const size_t N = size_t(1) << sf;
  const size_t symbol_count = samples.size() / N;
  // rx_runner.cpp:93-107
  std::vector<uint16_t> symbols(symbol_count);
  std::vector<std::complex<float>> fft_in(N), fft_out(N * osr);
  std::vector<float> window(N);
  lora_workspace ws{};
  ws.symbol_buf = symbols.data();
  ws.fft_in = fft_in.data();
  ws.fft_out = fft_out.data();
  ws.window = window.data();
  lora_params params{};
  params.sf = sf;
  params.osr = osr;
  params.window = hann ? window_type::window_hann : window_type::window_none;
  params.sync_word = 0x34;
  if (init(&ws, &params) != 0) return 3;
  const ssize_t demod_syms = demodulate(&ws, samples.data(), samples.size(), symbols.data(), symbols.size());
  if (demod_syms < 0) return 4;
  std::vector<uint8_t> decoded(demod_syms / 2 + 1);
  const ssize_t decoded_bytes = decode(&ws, symbols.data(), demod_syms, decoded.data(), decoded.size());
  const lora_metrics* m = get_last_metrics(&ws);
  std::printf("{\"ret\": %zd, \"sync\": %u, \"cfo_bits\": %u, \"toff_bits\": %u, \"decoded_bytes\": %zd, "
              "\"crc_ok\": %d, \"window0\": %u, \"window_mid\": %u, \"symbols\": [",
              demod_syms, ws.sync_word, fbits(m->cfo), fbits(m->time_offset), decoded_bytes, m->crc_ok ? 1 : 0,
              fbits(window[0]), fbits(window[N / 2]));
  for (ssize_t i = 0; i < demod_syms; ++i) std::printf("%s%u", i ? ", " : "", symbols[i]);
  std::printf("]");
  // estimate_offsets over every whole symbol, then compensate_offsets in place (phy.cpp:78-176)
  estimate_offsets(&ws, samples.data(), samples.size());
  std::printf(", \"est_cfo_bits\": %u, \"est_toff_bits\": %u}\n", fbits(m->cfo), fbits(m->time_offset));
  compensate_offsets(&ws, samples.data(), samples.size());
  std::FILE* fo = std::fopen(out, "wb");
  if (!fo) return 5;
  std::fwrite(samples.data(), sizeof(samples[0]), samples.size(), fo);
  std::fclose(fo);
  reset(&ws);
  return (m->cfo == 0.0f && m->time_offset == 0.0f && !m->crc_ok) ? 0 : 6;
}

static int tx(unsigned sf, unsigned osr, const char* hex, const char* out) {
  std::vector<uint8_t> payload;
  for (size_t i = 0; hex[i] && hex[i + 1]; i += 2) {
    char b[3] = {hex[i], hex[i + 1], 0};
    payload.push_back((uint8_t)std::strtoul(b, nullptr, 16));
  }
  lora_workspace ws{};
  lora_params params{};
  params.sf = sf;
  params.osr = osr;
  params.sync_word = 0x12;
  if (init(&ws, &params) != 0) return 3;
  std::vector<uint16_t> symbols(payload.size() * 2);
  const ssize_t ns = encode(&ws, payload.data(), payload.size(), symbols.data(), symbols.size());
  if (ns < 0) return 4;
  if (encode(&ws, payload.data(), payload.size(), symbols.data(), symbols.size() - 1) != -1) return 7;
  const size_t cap = (size_t(ns) + 2) * (size_t(1) << sf) * osr;
  std::vector<std::complex<float>> iq(cap);
  const ssize_t produced = modulate(&ws, symbols.data(), ns, iq.data(), cap);
  if (produced != (ssize_t)cap) return 5;
  if (modulate(&ws, symbols.data(), ns, iq.data(), cap - 1) != -1) return 8;
  std::FILE* fo = std::fopen(out, "wb");
  if (!fo) return 6;
  std::fwrite(iq.data(), sizeof(iq[0]), iq.size(), fo);
  std::fclose(fo);
  std::printf("{\"nsym\": %zd, \"samples\": %zd, \"symbols\": [", ns, produced);
  for (ssize_t i = 0; i < ns; ++i) std::printf("%s%u", i ? ", " : "", symbols[i]);
  std::printf("]}\n");
  return 0;
}

// A legacy workspace initialised twice without lora_demod_free (the reference's init
// overwrites every field): SF12 for long frames, then SF7 for a short frame; the SF7
// round trip must be exact (no stale plan, no undersized device buffer).
static int reinit() {
  const uint16_t syms[6] = {3, 77, 0, 127, 64, 12};
  const unsigned sf = 7;
  const size_t N = 128, n = (6 + 2) * N;
  std::vector<std::complex<float>> iq(n), dech(n), down(N), scratch(66 * 4096);
  lora_demod_workspace ws{};
  lora_demod_init(&ws, 12, window_type::window_hann, scratch.data(), scratch.size());
  lora_demod_init(&ws, sf, window_type::window_none, scratch.data(), 40);
  lora_modulate(syms, 6, iq.data(), sf, 1, bandwidth::bw_125, 1.0f, 0x12);
  float ph = 0.0f;
  genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, 1.0f);
  for (size_t i = 0; i < n; ++i) dech[i] = iq[i] * down[i % N] * 0.5f;  // no rescale: scratch not needed
  std::vector<uint16_t> out(6);
  uint8_t sync = 0;
  const size_t got = lora_demodulate(&ws, dech.data(), n, out.data(), 1, &sync);
  lora_demod_free(&ws);
  std::printf("{\"reinit_count\": %zu, \"sync\": %u, \"symbols\": [%u, %u, %u, %u, %u, %u]}\n", got, sync, out[0],
              out[1], out[2], out[3], out[4], out[5]);
  for (int i = 0; i < 6; ++i)
    if (out[i] != syms[i]) return 2;
  return got == 6 && sync == 0x12 ? 0 : 3;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::strcmp(argv[1], "reinit") == 0) return reinit();
  if (argc >= 7 && std::strcmp(argv[1], "rx") == 0)
    return rx((unsigned)std::atoi(argv[2]), (unsigned)std::atoi(argv[3]), std::atoi(argv[4]) != 0, argv[5], argv[6]);
  if (argc >= 6 && std::strcmp(argv[1], "tx") == 0)
    return tx((unsigned)std::atoi(argv[2]), (unsigned)std::atoi(argv[3]), argv[4], argv[5]);
  std::fprintf(stderr, "usage: rx_dropin rx <sf> <osr> <hann> <in.iq> <out.iq> | tx <sf> <osr> <hex> <out.iq>\n");
  return 1;
}
