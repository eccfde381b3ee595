// ref_shim.cpp — C ABI over the *reference* library, for validating the oracle.
//
// *** TEST INFRASTRUCTURE ONLY. ***  Built by oracle/Makefile together with the
// reference's own sources where they lie (/root/reference/src/phy/*.cpp, headers in
// /root/reference/include) into oracle/_ref/liblora_ref.so.  Nothing here is
// copied from the reference: these wrappers only marshal plain pointers into the
// reference's public API (include/lora_phy/phy.hpp:102-215, ChirpGenerator.hpp,
// kissfft.hh, LoRaCodes.hpp) so that Python tests can call it through ctypes.
// Built only in the build container (the reference sources do not exist on the GPU
// box); the built .so travels with the repo snapshot, where bench.py's cpu_baseline
// times ref_demod_frames - the reference's own lora_demodulate - on the host cores.
#include <lora_phy/phy.hpp>
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/LoRaCodes.hpp>
#include <lora_phy/kissfft.hh>

#include <complex>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

using cpx = std::complex<float>;

extern "C" {

int ref_gen_chirp(float* out, int N, int osr, int NN, float f0, int down, float ampl, float* phase,
                  float bw_scale) {
  return genChirp(reinterpret_cast<cpx*>(out), N, osr, NN, f0, down != 0, ampl, *phase, bw_scale);
}

int ref_fft(const float* in, float* out, int N) {
  static kissfft_plan<float> plan;
  kissfft<float>::init(plan, N, false);
  kissfft<float> f(plan);
  f.transform(reinterpret_cast<const cpx*>(in), reinterpret_cast<cpx*>(out));
  return plan.stages;
}

size_t ref_lora_modulate(const uint16_t* syms, size_t count, float* out, unsigned sf, unsigned osr,
                         unsigned bw_hz, float amplitude, uint8_t sync) {
  return lora_phy::lora_modulate(syms, count, reinterpret_cast<cpx*>(out), sf, osr,
                                 static_cast<lora_phy::bandwidth>(bw_hz), amplitude, sync);
}

size_t ref_lora_demodulate(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                           uint16_t* out_syms, uint8_t* out_sync, float* out_cfo, float* out_toff,
                           size_t scratch_len) {
  static lora_phy::lora_demod_workspace ws;
  std::vector<cpx> scratch(scratch_len ? scratch_len : 1);
  lora_phy::lora_demod_init(&ws, sf,
                            hann ? lora_phy::window_type::window_hann
                                 : lora_phy::window_type::window_none,
                            scratch_len ? scratch.data() : nullptr, scratch_len);
  ws.metrics = lora_phy::lora_metrics{};
  size_t n = lora_phy::lora_demodulate(&ws, reinterpret_cast<const cpx*>(iq), count, out_syms, osr,
                                       out_sync);
  if (out_cfo) *out_cfo = ws.metrics.cfo;
  if (out_toff) *out_toff = ws.metrics.time_offset;
  lora_phy::lora_demod_free(&ws);
  return n;
}

struct ApiWs {
  std::vector<uint16_t> symbol_buf;
  std::vector<cpx> fft_in, fft_out;
  std::vector<float> window;
  lora_phy::lora_workspace ws;
};

static void api_init(ApiWs& a, unsigned sf, int hann, unsigned osr, unsigned bw_hz) {
  const size_t N = size_t(1) << sf;
  a.symbol_buf.assign(N, 0);
  a.fft_in.assign(N, cpx());
  a.fft_out.assign(N * (osr ? osr : 1), cpx());
  a.window.assign(N, 0.0f);
  a.ws = lora_phy::lora_workspace{};
  a.ws.symbol_buf = a.symbol_buf.data();
  a.ws.fft_in = a.fft_in.data();
  a.ws.fft_out = a.fft_out.data();
  a.ws.window = a.window.data();
  lora_phy::lora_params p;
  p.sf = sf;
  p.bw = static_cast<lora_phy::bandwidth>(bw_hz);
  p.osr = osr;
  p.window = hann ? lora_phy::window_type::window_hann : lora_phy::window_type::window_none;
  lora_phy::init(&a.ws, &p);
}

long ref_api_demodulate(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                        unsigned bw_hz, uint16_t* syms, size_t cap, uint8_t* out_sync,
                        float* out_cfo, float* out_toff) {
  static ApiWs a;
  api_init(a, sf, hann, osr, bw_hz);
  long r = (long)lora_phy::demodulate(&a.ws, reinterpret_cast<const cpx*>(iq), count, syms, cap);
  if (out_sync) *out_sync = a.ws.sync_word;
  const lora_phy::lora_metrics* m = lora_phy::get_last_metrics(&a.ws);
  if (out_cfo) *out_cfo = m->cfo;
  if (out_toff) *out_toff = m->time_offset;
  return r;
}

long ref_api_modulate(const uint16_t* syms, size_t count, unsigned sf, unsigned osr, unsigned bw_hz,
                      uint8_t sync, float* out, size_t cap) {
  static ApiWs a;
  api_init(a, sf, 0, osr, bw_hz);
  a.ws.sync_word = sync;
  return (long)lora_phy::modulate(&a.ws, syms, count, reinterpret_cast<cpx*>(out), cap);
}

void ref_estimate_offsets(const float* iq, size_t count, unsigned sf, int hann, unsigned osr,
                          float* out_cfo, float* out_toff) {
  static ApiWs a;
  api_init(a, sf, hann, osr, 125000);
  lora_phy::estimate_offsets(&a.ws, reinterpret_cast<const cpx*>(iq), count);
  *out_cfo = a.ws.metrics.cfo;
  *out_toff = a.ws.metrics.time_offset;
}

void ref_compensate_offsets(float* iq, size_t count, unsigned sf, unsigned osr, float cfo, float to) {
  static ApiWs a;
  api_init(a, sf, 0, osr, 125000);
  a.ws.metrics.cfo = cfo;
  a.ws.metrics.time_offset = to;
  lora_phy::compensate_offsets(&a.ws, reinterpret_cast<cpx*>(iq), count);
}

long ref_api_encode(const uint8_t* payload, size_t n, unsigned sf, uint16_t* syms, size_t cap) {
  static ApiWs a;
  api_init(a, sf, 0, 1, 125000);
  return (long)lora_phy::encode(&a.ws, payload, n, syms, cap);
}

long ref_api_decode(const uint16_t* syms, size_t n, uint8_t* payload, size_t cap, int* crc_ok) {
  static ApiWs a;
  api_init(a, 7, 0, 1, 125000);
  long r = (long)lora_phy::decode(&a.ws, syms, n, payload, cap);
  *crc_ok = a.ws.metrics.crc_ok ? 1 : 0;
  return r;
}

size_t ref_lora_encode(const uint8_t* b, size_t n, uint16_t* out, unsigned sf) {
  return lora_phy::lora_encode(b, n, out, sf);
}
size_t ref_lora_decode(const uint16_t* s, size_t n, uint8_t* out) {
  return lora_phy::lora_decode(s, n, out);
}

// LoRaCodes.hpp helpers, one call per element / buffer.
uint8_t ref_enc_h84(uint8_t x) { return encodeHamming84sx(x); }
uint8_t ref_dec_h84(uint8_t b, int* err, int* bad) {
  bool e = false, d = false;
  uint8_t r = decodeHamming84sx(b, e, d);
  *err = e;
  *bad = d;
  return r;
}
uint8_t ref_enc_h74(uint8_t x) { return encodeHamming74sx(x); }
uint8_t ref_dec_h74(uint8_t b, int* err) {
  bool e = false;
  uint8_t r = decodeHamming74sx(b, e);
  *err = e;
  return r;
}
uint8_t ref_enc_p54(uint8_t x) { return encodeParity54(x); }
uint8_t ref_chk_p54(uint8_t b, int* err) {
  bool e = false;
  uint8_t r = checkParity54(b, e);
  *err = e;
  return r;
}
uint8_t ref_enc_p64(uint8_t x) { return encodeParity64(x); }
uint8_t ref_chk_p64(uint8_t b, int* err) {
  bool e = false;
  uint8_t r = checkParity64(b, e);
  *err = e;
  return r;
}
uint16_t ref_gray2bin(uint16_t x) { return grayToBinary16(x); }
uint16_t ref_bin2gray(uint16_t x) { return binaryToGray16(x); }
uint8_t ref_checksum8(const uint8_t* p, size_t n) { return checksum8(p, n); }
uint8_t ref_header_checksum(const uint8_t* h) { return headerChecksum(h); }
uint16_t ref_sx1272_crc(const uint8_t* d, int n) { return sx1272DataChecksum(d, n); }
void ref_whiten_sx1232(uint8_t* b, uint16_t n) { SX1232RadioComputeWhitening(b, n); }
void ref_whiten_sx1272(uint8_t* b, uint16_t n, int bitofs, int rdd) {
  Sx1272ComputeWhitening(b, n, bitofs, rdd);
}
void ref_whiten_lfsr(uint8_t* b, uint16_t n, int bitofs, size_t rdd) {
  Sx1272ComputeWhiteningLfsr(b, n, bitofs, rdd);
}
void ref_interleave(const uint8_t* cw, size_t ncw, uint16_t* syms, size_t ppm, size_t rdd) {
  diagonalInterleaveSx(cw, ncw, syms, ppm, rdd);
}
void ref_deinterleave(const uint16_t* syms, size_t ns, uint8_t* cw, size_t ppm, size_t rdd) {
  diagonalDeterleaveSx(syms, ns, cw, ppm, rdd);
}
void ref_deinterleave2(const uint16_t* syms, size_t ns, uint8_t* cw, size_t ppm, size_t rdd) {
  diagonalDeterleaveSx2(syms, ns, cw, ppm, rdd);
}

// The body of awgn_sweep_gtest.cpp:52-108 re-expressed as a generator of the noisy
// raw IQ and payloads it feeds to the reference (no gtest available offline).
size_t ref_awgn_gtest_frames(const unsigned* sfs, const unsigned* bws, int nprof, int packets,
                             int payload_size, double snr_db, float* out_iq, uint8_t* out_payload) {
  std::mt19937 rng(0);
  size_t off = 0, poff = 0;
  for (int p = 0; p < nprof; ++p) {
    const size_t N = size_t(1) << sfs[p];
    for (int pkt = 0; pkt < packets; ++pkt) {
      std::vector<uint8_t> payload(payload_size);
      for (auto& b : payload) b = static_cast<uint8_t>(rng() & 0xFF);
      std::vector<uint16_t> symbols(payload_size * 2);
      size_t symbol_count =
          lora_phy::lora_encode(payload.data(), payload.size(), symbols.data(), sfs[p]);
      size_t sample_count = (symbol_count + 2) * N;
      std::vector<cpx> samples(sample_count);
      lora_phy::lora_modulate(symbols.data(), symbol_count, samples.data(), sfs[p], 1,
                              static_cast<lora_phy::bandwidth>(bws[p]), 1.0f, 0x12);
      double sigma = std::pow(10.0, -snr_db / 20.0);
      std::normal_distribution<float> noise(0.0f, static_cast<float>(sigma / std::sqrt(2.0)));
      for (auto& s : samples) {
        s += std::complex<float>(noise(rng), noise(rng));
      }
      if (out_iq) std::memcpy(out_iq + 2 * off, samples.data(), sizeof(cpx) * sample_count);
      if (out_payload) std::memcpy(out_payload + poff, payload.data(), payload.size());
      off += sample_count;
      poff += payload.size();
    }
  }
  return off;
}


// The reference's usage pattern (tests/e2e_chain_test.cpp:79-101) over F frames of
// frame_len samples: optional caller-side dechirp with a genChirp down-chirp table,
// then one lora_demodulate per frame with a caller-owned scratch buffer; `threads`
// workers each own a workspace (the reference is reentrant per workspace).
void ref_demod_frames(const float* iq, size_t frames, size_t frame_len, unsigned sf, int hann,
                      unsigned osr, int dechirp, float bw_scale, uint16_t* out_syms,
                      size_t sym_stride, uint8_t* out_sync, float* out_cfo, float* out_toff,
                      int64_t* out_count, int threads) {
  if (threads < 1) threads = 1;
  auto worker = [&](int tid) {
    auto* ws = new lora_phy::lora_demod_workspace();
    std::vector<cpx> scratch(frame_len ? frame_len : 1), dech(dechirp ? frame_len : 0);
    const size_t N = size_t(1) << sf, step = N * (osr ? osr : 1);
    std::vector<cpx> down(dechirp ? step : 0);
    if (dechirp) {
      float ph = 0.0f;
      genChirp(down.data(), (int)N, (int)(osr ? osr : 1), (int)step, 0.0f, true, 1.0f, ph, bw_scale);
    }
    lora_phy::lora_demod_init(ws, sf,
                              hann ? lora_phy::window_type::window_hann
                                   : lora_phy::window_type::window_none,
                              scratch.data(), scratch.size());
    for (size_t f = (size_t)tid; f < frames; f += (size_t)threads) {
      const cpx* x = reinterpret_cast<const cpx*>(iq) + f * frame_len;
      if (dechirp) {
        for (size_t j = 0; j < frame_len; ++j) dech[j] = x[j] * down[j % step];
        x = dech.data();
      }
      uint8_t sync = 0;
      ws->metrics = lora_phy::lora_metrics{};
      const size_t n = lora_phy::lora_demodulate(ws, x, frame_len, out_syms + f * sym_stride, osr,
                                                 &sync);
      if (out_sync) out_sync[f] = sync;
      if (out_cfo) out_cfo[f] = ws->metrics.cfo;
      if (out_toff) out_toff[f] = ws->metrics.time_offset;
      if (out_count) out_count[f] = (int64_t)n;
    }
    lora_phy::lora_demod_free(ws);
    delete ws;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
}

}  // extern "C"
