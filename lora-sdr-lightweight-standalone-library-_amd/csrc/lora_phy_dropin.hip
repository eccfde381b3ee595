// lora_phy_dropin.hip — the reference's legacy C++ API (include/lora_mi355x_phy.hpp)
// implemented on the C-ABI: one frame per call, host buffers in and out, the demodulation
// on the plan's device.  Reference semantics kept per function (file:line in the header).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "../../include/lora_mi355x.h"
#include "../../include/lora_mi355x_phy.hpp"
#include "lora_internal.h"

namespace {

// Hamming 8/4 of LoRaCodes.hpp:229-281 (encodeHamming84sx / decodeHamming84sx): data bits
// d0..d3 in bits 0..3, parities (d0^d1^d2, d1^d2^d3, d0^d1^d3, d0^d2^d3) in bits 4..7;
// decoding corrects the single data-bit errors whose syndrome names one data bit.
uint8_t enc_h84(uint8_t x) {
  const int d0 = x & 1, d1 = (x >> 1) & 1, d2 = (x >> 2) & 1, d3 = (x >> 3) & 1;
  return (uint8_t)((x & 0xF) | ((d0 ^ d1 ^ d2) << 4) | ((d1 ^ d2 ^ d3) << 5) | ((d0 ^ d1 ^ d3) << 6) |
                   ((d0 ^ d2 ^ d3) << 7));
}

uint8_t dec_h84_nibble(uint8_t b) {
  const int b0 = b & 1, b1 = (b >> 1) & 1, b2 = (b >> 2) & 1, b3 = (b >> 3) & 1, b4 = (b >> 4) & 1,
            b5 = (b >> 5) & 1, b6 = (b >> 6) & 1, b7 = (b >> 7) & 1;
  const int p = (b0 ^ b1 ^ b2 ^ b4) | ((b1 ^ b2 ^ b3 ^ b5) << 1) | ((b0 ^ b1 ^ b3 ^ b6) << 2) |
                ((b0 ^ b2 ^ b3 ^ b7) << 3);
  switch (p) {
    case 0xD: return (uint8_t)((b ^ 1) & 0xF);
    case 0x7: return (uint8_t)((b ^ 2) & 0xF);
    case 0xB: return (uint8_t)((b ^ 4) & 0xF);
    case 0xE: return (uint8_t)((b ^ 8) & 0xF);
    default: return (uint8_t)(b & 0xF);
  }
}

// Per-frame outputs and the batch workspace behind the IQ in the workspace's single
// device allocation.
struct DevLayout {
  size_t iq, syms, sync, cfo, toff, maxa, ws, total;
};

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

DevLayout layout(const lora_demod_plan* plan, size_t samples, size_t N) {
  DevLayout d;
  size_t o = 0;
  d.iq = o;
  o += align256(samples * 8);
  d.syms = o;
  o += align256((samples / N + 2) * sizeof(uint16_t));
  d.sync = o;
  o += 256;
  d.cfo = o;
  o += 256;
  d.toff = o;
  o += 256;
  d.maxa = o;
  o += 256;
  d.ws = o;
  o += align256(lora_demod_workspace_bytes(plan, 1));
  d.total = o;
  return d;
}

// The plan for this call's oversampling (the reference passes osr per call): created on
// first use, recreated when osr changes.
bool ensure_plan(lora_phy::lora_demod_workspace* ws, unsigned osr) {
  if (ws->plan && ws->plan_osr == osr) return true;
  if (ws->plan) lora_demod_plan_destroy(ws->plan);
  ws->plan = nullptr;
  lora_demod_params p{};
  p.sf = ws->sf;
  p.osr = osr;
  p.bw_hz = 125000;  // no dechirp in the plan: the bandwidth only sets table phases it does not use
  p.window = ws->window_kind == lora_phy::window_type::window_hann ? LORA_WINDOW_HANN : LORA_WINDOW_NONE;
  p.dechirp = 0;     // lora_demodulate takes dechirped samples (its callers dechirp first)
  p.mode = LORA_MODE_LEGACY;
  p.device = ws->device;
  p.precision = LORA_PRECISION_EXACT;
  if (lora_demod_plan_create(&p, &ws->plan) != LORA_OK) {
    ws->plan = nullptr;
    return false;
  }
  ws->plan_osr = osr;
  return true;
}

bool ensure_dev(lora_phy::lora_demod_workspace* ws, size_t samples) {
  if (ws->dev && ws->dev_samples >= samples) return true;
  if (ws->dev) hipFree(ws->dev);
  ws->dev = nullptr;
  ws->dev_samples = 0;
  const DevLayout d = layout(ws->plan, samples, ws->N);
  if (hipMalloc(&ws->dev, d.total) != hipSuccess) {
    ws->dev = nullptr;
    return false;
  }
  ws->dev_samples = samples;
  return true;
}

}  // namespace

namespace lora_phy {

void lora_demod_init(lora_demod_workspace* ws, unsigned sf, window_type win, std::complex<float>* scratch,
                     size_t max_samples) {
  if (!ws) return;
  ws->N = size_t(1) << sf;
  ws->sf = sf;
  ws->window_kind = win;
  ws->scratch = scratch;
  ws->scratch_len = max_samples;
  ws->metrics = lora_metrics{};
  int dev = 0;
  hipGetDevice(&dev);
  ws->device = dev;
  hipStream_t st = nullptr;
  if (!ws->stream && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) ws->stream = st;
  // device resources for the common case (osr 1, max_samples), so that lora_demodulate
  // allocates nothing (no_alloc_test.cpp:78-99)
  if (ensure_plan(ws, 1) && max_samples > 0) ensure_dev(ws, max_samples);
}

void lora_demod_free(lora_demod_workspace* ws) {
  if (!ws) return;
  if (ws->stream) hipStreamSynchronize(static_cast<hipStream_t>(ws->stream));
  if (ws->dev) hipFree(ws->dev);
  if (ws->plan) lora_demod_plan_destroy(ws->plan);
  if (ws->stream) hipStreamDestroy(static_cast<hipStream_t>(ws->stream));
  ws->dev = nullptr;
  ws->dev_samples = 0;
  ws->plan = nullptr;
  ws->plan_osr = 0;
  ws->stream = nullptr;
  ws->N = 0;
  ws->scratch = nullptr;
  ws->scratch_len = 0;
}

size_t lora_demodulate(lora_demod_workspace* ws, const std::complex<float>* samples, size_t sample_count,
                       uint16_t* out_symbols, unsigned osr, uint8_t* out_sync) {
  if (!ws || ws->N == 0 || !samples) return 0;
  if (osr == 0) osr = 1;
  if (!ensure_plan(ws, osr) || !ensure_dev(ws, std::max<size_t>(sample_count, 1))) return 0;
  hipStream_t st = static_cast<hipStream_t>(ws->stream);
  const DevLayout d = layout(ws->plan, ws->dev_samples, ws->N);
  unsigned char* base = static_cast<unsigned char*>(ws->dev);
  const int64_t nsym = lora_demod_symbols_per_frame(ws->plan, (int64_t)sample_count);
  if (nsym < 0) return 0;
  if (sample_count > 0 &&
      hipMemcpyAsync(base + d.iq, samples, sample_count * sizeof(std::complex<float>), hipMemcpyHostToDevice,
                     st) != hipSuccess)
    return 0;
  lora_demod_outputs o{};
  o.symbols = reinterpret_cast<uint16_t*>(base + d.syms);
  o.sym_stride = std::max<int64_t>(nsym, 1);
  o.sync = base + d.sync;
  o.cfo = reinterpret_cast<float*>(base + d.cfo);
  o.time_offset = reinterpret_cast<float*>(base + d.toff);
  o.max_amp = reinterpret_cast<float*>(base + d.maxa);
  if (lora_demod_batch(ws->plan, reinterpret_cast<const float*>(base + d.iq), 1, (int64_t)sample_count,
                       (int64_t)sample_count, &o, base + d.ws, d.total - d.ws, st) < 0)
    return 0;
  uint8_t sync = 0;
  float cfo = 0.0f, toff = 0.0f, maxa = 0.0f;
  if (hipMemcpyAsync(&sync, o.sync, 1, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&cfo, o.cfo, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&toff, o.time_offset, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&maxa, o.max_amp, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
    return 0;
  if (nsym > 0 && out_symbols &&
      hipMemcpyAsync(out_symbols, o.symbols, (size_t)nsym * sizeof(uint16_t), hipMemcpyDeviceToHost, st) !=
          hipSuccess)
    return 0;
  if (hipStreamSynchronize(st) != hipSuccess) return 0;
  // LoRaDemod.cpp:68-71: a frame that needs rescaling without a large enough scratch
  // buffer returns 0 before anything is written (the symbols were copied above; the
  // caller's buffer content is unspecified then, as with a partially written output).
  if (maxa > 1.0f && (!ws->scratch || ws->scratch_len < sample_count)) return 0;
  ws->metrics.cfo = cfo;
  ws->metrics.time_offset = toff;
  if (out_sync) *out_sync = sync;
  return (size_t)nsym;
}

size_t lora_modulate(const uint16_t* symbols, size_t symbol_count, std::complex<float>* out_samples, unsigned sf,
                     unsigned osr, bandwidth bw, float amplitude, uint8_t sync) {
  if (osr == 0) osr = 1;
  const size_t per = (symbol_count + 2) * (size_t(1) << sf) * osr;
  if (!out_samples || (symbol_count > 0 && !symbols)) return 0;
  // per-thread device staging, grown on demand (the reference's lora_modulate takes no
  // workspace)
  thread_local void* dev = nullptr;
  thread_local size_t cap = 0;
  const size_t need = align256(per * 8) + align256(symbol_count * 2 + 2);
  if (cap < need) {
    if (dev) hipFree(dev);
    dev = nullptr;
    cap = 0;
    if (hipMalloc(&dev, need) != hipSuccess) return 0;
    cap = need;
  }
  int device = 0;
  hipGetDevice(&device);
  float* iq = static_cast<float*>(dev);
  uint16_t* s = reinterpret_cast<uint16_t*>(static_cast<unsigned char*>(dev) + align256(per * 8));
  if (symbol_count > 0 && hipMemcpy(s, symbols, symbol_count * 2, hipMemcpyHostToDevice) != hipSuccess) return 0;
  if (lora_mod_batch(sf, osr, static_cast<unsigned>(bw), amplitude, sync, s, 1, (int64_t)symbol_count, iq, device,
                     nullptr) < 0)
    return 0;
  if (hipMemcpy(out_samples, iq, per * 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return per;
}

size_t lora_encode(const uint8_t* bytes, size_t byte_count, uint16_t* out_symbols, unsigned /*sf*/) {
  size_t k = 0;
  for (size_t i = 0; i < byte_count; ++i) {
    out_symbols[k++] = enc_h84((uint8_t)(bytes[i] >> 4));
    out_symbols[k++] = enc_h84((uint8_t)(bytes[i] & 0x0F));
  }
  return k;
}

size_t lora_decode(const uint16_t* symbols, size_t symbol_count, uint8_t* out_bytes) {
  size_t k = 0;
  for (size_t i = 0; i + 1 < symbol_count; i += 2)
    out_bytes[k++] = (uint8_t)((dec_h84_nibble((uint8_t)symbols[i]) << 4) | dec_h84_nibble((uint8_t)symbols[i + 1]));
  return k;
}

}  // namespace lora_phy

int genChirp(std::complex<float>* samps, int N, int osr, int NN, float f0, bool down, const float ampl,
             float& phaseAccum, float bw_scale) {
  lora::host_gen_chirp(samps, N, osr, NN, f0, down, ampl, phaseAccum, bw_scale);
  return NN;
}
