/*
 * lora_mi355x.h — C-ABI of the MI355X LoRa PHY demodulator/modulator.
 *
 * This is the drop-in boundary for the reference's hot path.  Every entry point
 * names the reference interface it replaces (paths relative to the reference
 * checkout yakir1991/LoRa-SDR-Lightweight-Standalone-Library-):
 *
 *   lora_demod_plan_create / _destroy
 *       replaces lora_phy::lora_demod_init / lora_demod_free
 *       (include/lora_phy/phy.hpp:190-194, src/phy/LoRaDemod.cpp:10-47) and, in
 *       LORA_MODE_API, lora_phy::init (phy.hpp:102, phy.cpp:26-49).
 *   lora_demod_batch
 *       replaces lora_phy::lora_demodulate (phy.hpp:204-207, LoRaDemod.cpp:49-195),
 *       one call per frame in the reference, F frames per call here; with
 *       params.dechirp = 1 it also absorbs the caller-side dechirp loop every
 *       reference caller runs first (tests/e2e_chain_test.cpp:85-93).
 *       In LORA_MODE_API it replaces lora_phy::demodulate (phy.hpp:134-136,
 *       phy.cpp:178-239) including estimate_offsets (phy.cpp:78-145) and
 *       get_last_metrics (phy.cpp:258-261).
 *   lora_mod_batch
 *       replaces lora_phy::lora_modulate (phy.hpp:198-201, LoRaMod.cpp:8-43) and
 *       lora_phy::modulate (phy.hpp:126-128, phy.cpp:65-76).
 *
 * Conventions: plain pointers and sizes only.  IQ buffers are interleaved fp32
 * (I,Q) pairs — the layout of std::complex<float> and torch.complex64 — and live in
 * device memory (HBM) of the plan's device.  The caller owns every buffer
 * (API_SPEC.md ownership rule); the plan owns only its constant tables.  No call
 * allocates or synchronises: `stream` is a hipStream_t (NULL = default stream); the
 * work is enqueued on it and nothing else, so the calls are hipGraph-capturable.
 * A plan may be used by one host thread at a time.
 *
 * Errors are negative errno values (the reference returns -1, phy.cpp:27,58,181-190);
 * lora_last_error() gives a thread-local message.
 */
#ifndef LORA_MI355X_H
#define LORA_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LORA_OK 0
#define LORA_EIO (-5)     /* HIP runtime error */
#define LORA_ENOMEM (-12) /* device allocation failed at plan creation */
#define LORA_EINVAL (-22) /* bad parameter / size (reference: -1) */
#define LORA_ERANGE (-34) /* output capacity too small (reference: -1) */

/* phy.hpp:29-32 */
#define LORA_WINDOW_NONE 0
#define LORA_WINDOW_HANN 1

/* LEGACY: lora_demodulate semantics (LoRaDemod.cpp:49-195): max-amplitude
 *   normalisation, 2-symbol CFO/timing estimate on the (dechirped) input, per-symbol
 *   CFO rotation + FFT + argmax; frames of any length, sync nibbles from symbols 0/1.
 * API: lora_phy::demodulate semantics (phy.cpp:178-239): no normalisation, estimate
 *   on the raw input, per-symbol fused down-chirp; frame length must be a whole
 *   number (>= 2) of symbols. */
#define LORA_MODE_LEGACY 0
#define LORA_MODE_API 1
/* RAW: the detector primitive alone - per whole symbol: (dechirp) -> (window) ->
 *   2^SF FFT -> lowest-index argmax |X|^2 (LoRaDetector.hpp:39-58), no normalisation,
 *   no offset estimate, no rotation, every symbol output (no sync word: sync, cfo,
 *   time_offset, max_amp are written as 0).  This is the demodulator of the
 *   reference's Python AWGN sweep (tests/awgn_sweep.py:262-265). */
#define LORA_MODE_RAW 2

/* Rotation arithmetic of the symbol demod (lora_demod_batch, LEGACY / API modes).
 * EXACT: bit-identical to the reference (glibc sincosf per sample, LoRaDemod.cpp:151-157;
 *   every output equals lora_demodulate's).  The default.
 * FAST: the per-sample CFO rotation uses the hardware sine/cosine (v_sin/v_cos_f32 on
 *   the phase in revolutions, absolute phase error ~1e-5 rad) instead of glibc's
 *   double-precision polynomial.  The normalisation, the offset estimate (cfo,
 *   time_offset) and the sync word stay exact; data symbol indices equal the reference
 *   except where two FFT bins are within rounding of each other (near-ties under
 *   noise).  Stated tolerance, checked by tests/test_gpu_fast_rotation.py: identical
 *   symbols on noiseless and >= 0 dB frames; >= 99 % per-symbol agreement at -10 dB
 *   SF7, and SER within 0.01 absolute of the exact path at any SNR. */
#define LORA_PRECISION_EXACT 0
#define LORA_PRECISION_FAST 1

typedef struct lora_demod_plan lora_demod_plan;

typedef struct {
  unsigned sf;    /* spreading factor, 2..12 (N = 2^sf <= 4096, kissfft.hh:34) */
  unsigned osr;   /* oversampling ratio >= 1 (0 is treated as 1, phy.cpp:32) */
  unsigned bw_hz; /* 125000, 250000 or 500000 (phy.hpp:37-41) */
  int window;     /* LORA_WINDOW_* */
  int dechirp;    /* LEGACY / RAW: 1 = input is raw IQ, multiply sample j of each frame
                     by genChirp(N, osr, N*osr, down)[j mod N*osr] first
                     (e2e_chain_test.cpp:85-93); 0 = input already dechirped */
  int mode;       /* LORA_MODE_* */
  int device;     /* HIP device ordinal */
  int precision;  /* LORA_PRECISION_* (0 = EXACT) */
} lora_demod_params;

/* Per-frame outputs; any pointer may be NULL.  Device pointers. */
typedef struct {
  uint16_t* symbols;     /* [frames][sym_stride]; symbol indices (LoRaDemod.cpp:165-174) */
  int64_t sym_stride;    /* elements between frames in `symbols` (>= symbols per frame) */
  uint8_t* sync;         /* [frames] sync word from symbols 0/1 (LoRaDemod.cpp:177-192) */
  float* cfo;            /* [frames] lora_metrics.cfo (LoRaDemod.cpp:131) */
  float* time_offset;    /* [frames] lora_metrics.time_offset (LoRaDemod.cpp:134-135) */
  float* max_amp;        /* [frames] LEGACY: max(|I|,|Q|) of the (dechirped) frame
                            (LoRaDemod.cpp:59-67); callers emulating the scratch-size
                            rule (LoRaDemod.cpp:69-71) need it */
} lora_demod_outputs;

int lora_demod_plan_create(const lora_demod_params* params, lora_demod_plan** plan);
int lora_demod_plan_destroy(lora_demod_plan* plan);

/* Symbols each frame of `frame_len` samples yields (>= 0), or a negative error
 * (LORA_MODE_API: frame_len must be a multiple of N*osr with >= 2 symbols). */
int64_t lora_demod_symbols_per_frame(const lora_demod_plan* plan, int64_t frame_len);

/* Device workspace bytes lora_demod_batch needs for `frames` frames of `frame_len`
 * samples (0 when frames is 0).  The reference's workspace is caller-owned too
 * (lora_demod_workspace, phy.hpp:170-185, plus its scratch buffer sized to the frame). */
size_t lora_demod_workspace_bytes(const lora_demod_plan* plan, int64_t frames, int64_t frame_len);

/* Demodulate `frames` frames of `frame_len` complex samples each, frame f starting
 * at iq + 2*f*frame_stride floats.  `workspace` must hold
 * lora_demod_workspace_bytes(plan, frames, frame_len) bytes of device memory (may be NULL
 * if 0).
 * Returns symbols per frame (>= 0) or a negative error. */
int64_t lora_demod_batch(lora_demod_plan* plan, const float* iq, int64_t frames,
                         int64_t frame_len, int64_t frame_stride, const lora_demod_outputs* out,
                         void* workspace, size_t workspace_bytes, void* stream);

/* lora_phy::estimate_offsets (phy.hpp:142-144, phy.cpp:78-145) for F frames: every
 * whole symbol of each frame, osr phases, raw (not dechirped, not normalised)
 * windowed samples, plain '>' phase selection.  Writes cfo[f] / time_offset[f]
 * (device arrays) unless the frame holds no whole symbol, in which case the
 * outputs are left untouched (phy.cpp:81,87).  Uses the plan's sf/osr/window only.
 * Returns the number of symbols each frame's estimate used. */
int64_t lora_estimate_offsets_batch(lora_demod_plan* plan, const float* iq, int64_t frames,
                                    int64_t frame_len, int64_t frame_stride, float* cfo,
                                    float* time_offset, void* stream);

/* lora_phy::compensate_offsets (phy.hpp:150-152, phy.cpp:147-176) for F frames,
 * out of place: out[f] = shift(in[f] * exp(j*rate*n)), rate = -2*pi*cfo[f]/(N*osr),
 * shift by round(time_offset[f]) samples with zero fill.  `in` and `out` must not
 * overlap (the caller copies back for the reference's in-place semantics).
 * cfo / time_offset are device arrays of `frames` floats.  Returns frame_len. */
int64_t lora_compensate_offsets_batch(unsigned sf, unsigned osr, const float* in, int64_t frames,
                                      int64_t frame_len, int64_t frame_stride, const float* cfo,
                                      const float* time_offset, int device, void* stream,
                                      float* out);

/* lora_modulate for `frames` independent frames: symbols [frames][sym_count] ->
 * iq [frames][(sym_count+2)*N*osr] (2 sync up-chirps then one chirp per symbol,
 * phase-continuous within a frame, LoRaMod.cpp:8-41).  Returns samples per frame. */
int64_t lora_mod_batch(unsigned sf, unsigned osr, unsigned bw_hz, float amplitude, uint8_t sync,
                       const uint16_t* symbols, int64_t frames, int64_t sym_count, float* iq,
                       int device, void* stream);

/* Measurement hooks (bench.py): while enabled, every kernel lora_demod_batch launches
 * on this plan is bracketed by a pair of HIP events on the stream it runs on, for up
 * to `max_calls` calls.  Stages: 0 = frame max, 1 = estimate + sync symbols (with the
 * speculative pipeline: its pre-pass and certification kernels), 2 = symbol demod.
 * lora_demod_profile_read waits for the recorded events and returns, per stage, the
 * summed kernel ms over the recorded calls (stage_ms[3]) and the number of calls
 * recorded.  No effect on results. */
int lora_demod_profile_enable(lora_demod_plan* plan, int max_calls);
int lora_demod_profile_read(lora_demod_plan* plan, float* stage_ms, int* calls);

/* Which kernels the plan's last lora_demod_batch call launched (bit mask, for tests and
 * measurement): the speculative single-read pipeline is SPEC + ESTIMATE + DEMOD; the
 * three-launch path is FRAME_MAX (LEGACY) + ESTIMATE + DEMOD; GENERIC marks the LDS
 * estimate kernel (frames with fewer than two whole symbols).  0 before the first call.
 * Host-side bookkeeping only.  (Bit 8 belonged to a frame-resident kernel that measured
 * slower and was removed; it is never set.) */
#define LORA_KERNEL_FRAME_MAX 1
#define LORA_KERNEL_ESTIMATE 2
#define LORA_KERNEL_DEMOD 4
#define LORA_KERNEL_GENERIC 16
#define LORA_KERNEL_FRAME_MAX_WAVE 32 /* with FRAME_MAX: the one-wave-per-frame variant (short frames) */
#define LORA_KERNEL_SPEC 64 /* the speculative single-read pipeline (with ESTIMATE + DEMOD) */
int lora_demod_last_kernels(const lora_demod_plan* plan);

/* LEGACY frames at osr 1-4 with either window (none or Hann), SF 6-12, of 3 .. 2 + 4 * 2^SF symbols (SF7: 514),
 * run as a speculative single-read pipeline (LORA_KERNEL_SPEC) - and LORA_MODE_API frames at osr 1 (the exact
 * estimate first, then every data symbol rotated with the hardware sine/cosine and certified or recomputed
 * exactly; phy.cpp:178-239) and LORA_MODE_RAW frames at osr 1, SF 6-9 (every symbol through the same symbol
 * pass with no rotation, certified against the transforms' rounding or recomputed): the offset estimate on
 * unscaled samples, every
 * data symbol demodulated once while the frame maximum is reduced from the same read, then
 * the exact estimate, with each data symbol either certified by a rounding bound on its
 * argmax margin or recomputed exactly - the outputs equal the reference's (LoRaDemod.cpp:
 * 49-195) either way.  This returns how many data symbols this plan has recomputed so far
 * (synchronises the device; for tests and diagnostics).  LORA_MI355X_SPEC=0 disables the
 * pipeline (three launches: frame max, estimate, demod). */
int64_t lora_demod_spec_recomputed(lora_demod_plan* plan);

/* Choose the plan's path explicitly (instead of the process-wide LORA_MI355X_SPEC read at
 * plan creation): speculative = 1 runs the speculative single-read pipeline wherever it
 * covers the configuration (the default), 0 always the three-launch exact path.  Both give
 * the reference's outputs; the second is the pipeline's checker in the tests.  Returns 0. */
int lora_demod_plan_set_pipeline(lora_demod_plan* plan, int speculative);

/* Diagnostics of the C++ drop-in's private AQL queue (liblora_phy.so): with
 * LORA_MI355X_AQL_PROFILE=1 set before the queue is created, every dispatch is timestamped
 * and this returns the last call's timeline in microseconds relative to its doorbell:
 * out[0] = packets n, out[1 + 2i], out[2 + 2i] = packet i's start and end on the GPU,
 * out[1 + 2n] = when the host saw the completion.  Returns the doubles written (0 when
 * nothing was profiled or cap < 2n + 2). */
int lora_aql_last_profile(double* out, int cap);

/* Thread-local text of the last error ("" if none). */
const char* lora_last_error(void);

/* Library version string. */
const char* lora_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LORA_MI355X_H */
