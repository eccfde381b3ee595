/*
 * lora_mi355x_phy.hpp — C++ drop-in for the reference's legacy demodulator API, over the
 * C-ABI of lora_mi355x.h (the same liblora_mi355x.so exports both).
 *
 * A caller written against the reference's <lora_phy/phy.hpp> legacy helpers and
 * <lora_phy/ChirpGenerator.hpp> genChirp (e.g. tests/e2e_chain_test.cpp:54-117) compiles
 * unchanged with -I<repo>/include/compat (whose lora_phy/phy.hpp and
 * lora_phy/ChirpGenerator.hpp only include this header) and links with -llora_mi355x.
 * The functions keep the reference's names, argument meaning and return values; the
 * demodulation runs on the GPU:
 *
 *   lora_demod_init / lora_demod_free     phy.hpp:190-194, LoRaDemod.cpp:10-47
 *   lora_demodulate                       phy.hpp:204-207, LoRaDemod.cpp:49-195
 *   lora_modulate                         phy.hpp:198-201, LoRaMod.cpp:8-41
 *   lora_encode / lora_decode             phy.hpp:210-215, LoRaEncoder.cpp / LoRaDecoder.cpp
 *   genChirp (float)                      ChirpGenerator.hpp:24-50
 *
 * Source-compatible, not binary-compatible: lora_demod_workspace has the reference's
 * name and the fields callers touch (N, window_kind, metrics, scratch, scratch_len), but
 * holds a device plan and device buffers instead of kissfft state.  Ownership follows
 * the reference: the caller owns the workspace object and the scratch buffer; the
 * device resources the workspace holds are created by lora_demod_init (sized by its
 * max_samples) and released by lora_demod_free.  lora_demodulate allocates only when a
 * call exceeds the max_samples given to init (or init was given none).  Host pointers in,
 * host pointers out; each call is synchronous like the reference's.  For batches of
 * frames already in device memory use lora_demod_batch (lora_mi355x.h) directly.
 */
#ifndef LORA_MI355X_PHY_HPP
#define LORA_MI355X_PHY_HPP

#include <cmath>
#include <complex>
#include <cstddef>
#include <cstdint>

struct lora_demod_plan;  // lora_mi355x.h

namespace lora_phy {

/* phy.hpp:29-32 */
enum class window_type {
  window_none,
  window_hann,
};

/* phy.hpp:37-41 */
enum class bandwidth : unsigned {
  bw_125 = 125000,
  bw_250 = 250000,
  bw_500 = 500000,
};

constexpr float bw_to_hz(bandwidth bw) { return static_cast<float>(static_cast<unsigned>(bw)); }
constexpr float bw_scale(bandwidth bw) { return bw_to_hz(bw) / 125000.0f; }

/* phy.hpp:65-69 */
struct lora_metrics {
  bool crc_ok{};
  float cfo{};
  float time_offset{};
};

/* phy.hpp:170-185 (same name and caller-visible fields; device state instead of kissfft) */
struct lora_demod_workspace {
  size_t N{};
  window_type window_kind{window_type::window_none};
  lora_metrics metrics{};
  std::complex<float>* scratch{};
  size_t scratch_len{};
  // device side, owned between lora_demod_init and lora_demod_free
  unsigned sf{};
  unsigned plan_osr{};
  int device{};
  ::lora_demod_plan* plan{};
  void* dev{};          // one device allocation: IQ | symbols | per-frame outputs | workspace
  size_t dev_samples{};  // IQ capacity of `dev` in complex samples
  void* stream{};        // hipStream_t
};

void lora_demod_init(lora_demod_workspace* ws, unsigned sf, window_type win = window_type::window_none,
                     std::complex<float>* scratch = nullptr, size_t max_samples = 0);
void lora_demod_free(lora_demod_workspace* ws);

size_t lora_modulate(const uint16_t* symbols, size_t symbol_count, std::complex<float>* out_samples, unsigned sf,
                     unsigned osr, bandwidth bw, float amplitude = 1.0f, uint8_t sync = 0x12);

size_t lora_demodulate(lora_demod_workspace* ws, const std::complex<float>* samples, size_t sample_count,
                       uint16_t* out_symbols, unsigned osr, uint8_t* out_sync = nullptr);

size_t lora_encode(const uint8_t* bytes, size_t byte_count, uint16_t* out_symbols, unsigned sf);
size_t lora_decode(const uint16_t* symbols, size_t symbol_count, uint8_t* out_bytes);

}  // namespace lora_phy

/* ChirpGenerator.hpp:24-50 for Type = float (the reference's template is only ever
 * instantiated with float): the same fp32 recurrence the plan tables use. */
int genChirp(std::complex<float>* samps, int N, int osr, int NN, float f0, bool down, const float ampl,
             float& phaseAccum, float bw_scale = 1.0f);

#endif /* LORA_MI355X_PHY_HPP */
