/*
 * lora_mi355x_phy.hpp — C++ drop-in for the reference's <lora_phy/phy.hpp> API, over the
 * C-ABI of lora_mi355x.h (the same liblora_mi355x.so exports both).
 *
 * A caller written against the reference's phy.hpp and <lora_phy/ChirpGenerator.hpp>
 * (e.g. tests/e2e_chain_test.cpp:54-117, runners/rx_runner.cpp:102-122) compiles
 * unchanged with -I<repo>/include/compat (whose lora_phy/phy.hpp and
 * lora_phy/ChirpGenerator.hpp only include this header) and links with -llora_phy
 * (liblora_phy.so, the drop-in over liblora_mi355x.so).  Loading liblora_phy.so sets up the
 * GPU side once, before main (the HIP runtime, a private AQL queue with every kernel object
 * resolved, LEGACY plans for SF 2-12 x both windows, buffers for frames of up to 1 M samples
 * and a modulator staging area), so lora_modulate, lora_demod_init and lora_demodulate
 * allocate nothing on the host (no_alloc_test.cpp:52-99).  LORA_MI355X_DROPIN_LAZY=1 in the
 * environment skips that set-up (each call then sets up what it needs, allocating).
 * The functions keep the reference's names, argument meaning and return values; the
 * demodulation runs on the GPU:
 *
 *   workspace API (phy.hpp:96-156, src/phy/phy.cpp:26-261)
 *   init / reset                          phy.hpp:102-106, phy.cpp:26-53
 *   encode / decode                       phy.hpp:111-121, phy.cpp:55-63, 241-256
 *   modulate                              phy.hpp:126-128, phy.cpp:65-76
 *   demodulate                            phy.hpp:134-136, phy.cpp:178-239
 *   estimate_offsets / compensate_offsets phy.hpp:142-152, phy.cpp:78-176
 *   get_last_metrics                      phy.hpp:156, phy.cpp:258-261
 *   legacy helpers (phy.hpp:158-215)
 *   lora_demod_init / lora_demod_free     phy.hpp:190-194, LoRaDemod.cpp:10-47
 *   lora_demodulate                       phy.hpp:204-207, LoRaDemod.cpp:49-195
 *   lora_modulate                         phy.hpp:198-201, LoRaMod.cpp:8-41
 *   lora_encode / lora_decode             phy.hpp:210-215, LoRaEncoder.cpp / LoRaDecoder.cpp
 *   genChirp (float)                      ChirpGenerator.hpp:24-50
 *
 * Source-compatible, not binary-compatible: lora_workspace and lora_demod_workspace have
 * the reference's names and every field callers touch, but hold a device plan, device
 * buffers and pinned host staging instead of kissfft state.  Ownership follows the
 * reference: the caller owns the workspace object and its buffers (symbol_buf, fft_in,
 * fft_out, window, scratch); the device resources are created by init / lora_demod_init
 * and released by lora_demod_free or, for lora_workspace (whose reference API has no free
 * call), by its destructor.  Neither workspace may be copied.  Each call is synchronous,
 * host pointers in and out, like the reference's; lora_demodulate performs no host
 * allocation when the frame fits the max_samples given to lora_demod_init (the
 * reference's no_alloc_test.cpp:90-99 guard); with the load-time runtime, lora_demod_init
 * (max_samples <= 1 M) and lora_modulate (<= 2 M output samples) do not either.  For batches of frames already in device
 * memory use lora_demod_batch (lora_mi355x.h) directly.
 */
#ifndef LORA_MI355X_PHY_HPP
#define LORA_MI355X_PHY_HPP

#include <sys/types.h>

#include <cmath>
#include <complex>
#include <cstddef>
#include <cstdint>

struct lora_demod_plan;  // lora_mi355x.h

/* 0 when liblora_phy.so's load-time runtime is up (the legacy calls then allocate nothing),
 * else the set-up step that failed (csrc/lora_phy_dropin.hip). */
extern "C" int lora_phy_dropin_status(void);
/* Diagnostics: where the last lora_demodulate / lora_modulate call on the private AQL queue
 * spent its time, in microseconds - out[0..3] the demodulation's copy into the pinned
 * staging, host logic (lora_demod_batch with the launch recorder), dispatch to completion
 * (aql_run), copy out; out[4..7] the same for the modulation.  Returns 8. */
extern "C" int lora_phy_dropin_last_timing(double* out);

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

/* phy.hpp:51-58 */
struct lora_params {
  unsigned sf{};
  bandwidth bw{bandwidth::bw_125};
  unsigned cr{};
  unsigned osr{1};
  window_type window{window_type::window_none};
  uint8_t sync_word{0x12};
};

/* phy.hpp:65-69 */
struct lora_metrics {
  bool crc_ok{};
  float cfo{};
  float time_offset{};
};

namespace detail {
/* Device side of a workspace: an API- or LEGACY-mode plan, one device allocation (IQ |
 * symbols | per-frame outputs | batch workspace), pinned host staging for the same
 * layout, a stream, and a private AQL queue on which each frame's kernels are dispatched
 * without a HIP runtime call (so without a host allocation). */
struct device_state {
  unsigned sf{};
  unsigned plan_osr{};
  int plan_window{-1};
  unsigned plan_bw{};
  int device{};
  ::lora_demod_plan* plan{};
  void* dev{};
  void* host{};
  size_t bytes{};    // capacity of dev and host
  size_t samples{};  // IQ capacity in complex samples
  void* stream{};    // hipStream_t
  void* aql{};       // lora::AqlQueue (csrc/lora_aql.hip); null: frames go through HIP
  int aql_status{};  // why there is no queue: 0, or the failing step's code (lora_internal.h)
  // Borrowed from the drop-in library's load-time runtime (no allocation at init): a slot
  // of preallocated buffers (dev / host / stream while they are the slot's), a shared plan,
  // the shared AQL queue.  release() returns them instead of freeing them.
  int slot{-1};
  bool shared_plan{};
  bool shared_aql{};
};
void release(device_state& d);
}  // namespace detail

/* phy.hpp:77-92 (same name and caller-visible fields; device state instead of kissfft
 * plans).  Released by its destructor: the reference's workspace API has no free call.
 * Lifetime: destroy it while the HIP runtime is alive (before exit's static destructors); a
 * workspace destroyed after the runtime's teardown skips the release (hipGetDevice fails). */
struct lora_workspace {
  uint16_t* symbol_buf{};
  std::complex<float>* fft_in{};
  std::complex<float>* fft_out{};
  float* window{};
  window_type window_kind{window_type::window_none};
  lora_metrics metrics{};
  unsigned osr{1};
  bandwidth bw{bandwidth::bw_125};
  uint8_t sync_word{0x12};
  // device side, owned between init and destruction
  detail::device_state gpu{};

  lora_workspace() = default;
  lora_workspace(const lora_workspace&) = delete;
  lora_workspace& operator=(const lora_workspace&) = delete;
  ~lora_workspace() { detail::release(gpu); }
};

int init(lora_workspace* ws, const lora_params* cfg);
void reset(lora_workspace* ws);
ssize_t encode(lora_workspace* ws, const uint8_t* payload, size_t payload_len, uint16_t* symbols,
               size_t symbol_cap);
ssize_t decode(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count, uint8_t* payload,
               size_t payload_cap);
ssize_t modulate(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count, std::complex<float>* iq,
                 size_t iq_cap);
ssize_t demodulate(lora_workspace* ws, const std::complex<float>* iq, size_t sample_count, uint16_t* symbols,
                   size_t symbol_cap);
void estimate_offsets(lora_workspace* ws, const std::complex<float>* samples, size_t sample_count);
void compensate_offsets(const lora_workspace* ws, std::complex<float>* samples, size_t sample_count);
const lora_metrics* get_last_metrics(const lora_workspace* ws);

/* phy.hpp:170-185 (same name and caller-visible fields; device state instead of kissfft) */
struct lora_demod_workspace {
  size_t N{};
  window_type window_kind{window_type::window_none};
  lora_metrics metrics{};
  std::complex<float>* scratch{};
  size_t scratch_len{};
  // device side, owned between lora_demod_init and lora_demod_free
  detail::device_state gpu{};
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
