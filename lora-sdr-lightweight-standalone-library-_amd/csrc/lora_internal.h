// lora_internal.h — kernel argument block shared by the demod translation units.
#pragma once
#include <complex>

#include "lora_device.h"

namespace lora {

// Partial maxima per frame kept in the workspace by k_frame_max (no zeroing pass, no
// atomics); frames longer than kMaxBpf * 4096 samples use proportionally longer blocks.
constexpr int kMaxBpf = 80;  // SF12 frames of 66 symbols: 66 blocks of 4096 samples
// Speculative pipeline: a frame of up to kSpecChunks * T data symbols (T = N/16 lanes per
// symbol; SF6 256, SF7 512, ..., SF12 16384), one certification bit per data symbol in the
// certify kernel's LDS.
constexpr int kSpecChunks = 64;
// The certification's reject list in kFixStripes stripes (stage-2 workgroup b appends to
// stripe b % kFixStripes): one counter per stripe, 64 bytes apart - a single counter took
// one returning atomic per wave and round from every workgroup, serialised on one address
// (about 35 us of the SF7 certify kernel at -10 dB).
constexpr int kFixStripes = 16;
// frames per workgroup of the stage-2 kernel (k_est_fast: a T-lane group per frame in
// blocks of max(T, 64) lanes, T = N/16): the stripes' capacity follows from it
inline int est_frames_per_block(int N) {
  const int T = N >= 16 ? N / 16 : 1;
  return (T >= 64 ? 256 : 64) / T;
}

struct KArgs {
  const cf* iq;
  int64_t frame_len, frame_stride;
  int sf, N, osr, step, total, have_sync, mode, dechirp, hann;
  float power_scale;
  const cf* tw;
  const uint16_t* rev;
  const float* win;
  const cf* down;   // legacy dechirp table, `step` entries stored twice (2*step, no wrap)
  const cf* down1;  // API per-symbol down-chirp, N entries
  const uint32_t* maxbits;  // LEGACY: per-frame partial maxima [frame][mx_bpf] (float bits)
  int mx_bpf;               // partials per frame; 0 = none (empty frames -> max 0)
  lora::FrameParams* fp;
  uint16_t* syms;
  int64_t sym_stride;
  uint8_t* sync;
  float* cfo;
  float* toff;
  float* max_amp;
  int est_only;  // lora_estimate_offsets_batch: all symbols, raw samples, outputs only
  int fast_rot;  // LORA_PRECISION_FAST: hardware sin/cos rotation in the symbol demod
  const cf* twTA;  // fast kernels: slot-major twiddles of LDS pass A / B (or null)
  const cf* twTB;
  // twTB in slot pairs: float4 {slot 2p, slot 2p+1} at [p*MA + k], an odd last slot after
  // them as cf at [(NT/2)*MA*2 + k] - one 16-byte load per two twiddles (or null)
  const cf* twTB2;
  // LEGACY osr-1 dechirp table in pairs (speculative demod): float4 {down[c + T*2p],
  // down[c + T*(2p+1)]} at [p*(N + T) + c], T = N/16, c < N + T (or null)
  const cf* downP;
  // Speculative single-read pipeline (lora_demod_batch, LEGACY osr-1 unwindowed frames):
  // the estimate on unscaled samples, the data symbols' window maxima and certification
  // margins written by the symbol demod, and a device counter of exact recomputations.
  FrameParams* fp_spec = nullptr;  // [frame] estimate on unscaled samples
  // [frame][symbol s < total][2]: |X1| - |X2| and, for a data symbol (s >= 2), its window's
  // max(|I|,|Q|); for a sync symbol (s < 2) the speculative index's bits
  float* spec_marg = nullptr;
  uint32_t* spec_max = nullptr;    // writable alias of maxbits: [frame] max outside the windows
  unsigned int* spec_fix = nullptr;
  // the symbols certification rejected, compacted per stripe: kFixStripes counts (zeroed
  // by the pre-pass, fix_count[16 s]) and (frame, data symbol) pairs at fix_list[2 (s
  // fix_cap + i)], recomputed exactly by the pipeline's fourth launch
  unsigned int* fix_count = nullptr;
  uint32_t* fix_list = nullptr;
  int64_t fix_cap = 0;
};

// Shape of the fast kernels' LDS passes for SF >= 6 (lora_demod_fast.hip Geo<SF>): pass-1
// span R1 (8 for odd SF, radix-2 innermost; 16 for even), then pass A of span RA over
// groups k < MA_A = R1 and pass B of span RB over k < MA_B = R1*RA (span 1 = no pass).
struct PassShape {
  int RA, MA_A, RB, MA_B;
};
__host__ __device__ constexpr PassShape pass_shape(int sf) {
  const int R1 = (sf & 1) ? 8 : 16;
  const int X = (1 << sf) / R1;
  const int RA = X >= 16 ? 16 : X;
  const int RB = X > 16 ? X / 16 : 1;
  return PassShape{RA, R1, RB, R1 * RA};
}

// Twiddle index of slot j of a radix-16 (15 slots) or radix-4 (3 slots) LDS pass with
// butterfly group k < MA, in pass_regs' order: slots 0-2 the first radix-4 stage
// (tw[q*k*fs1], q = 1..3, fs1 = N/(4*MA)), slots 3+3*uu+(q-1) the second (kk = k + MA*uu,
// tw[q*kk*fs2], fs2 = fs1/4).
__host__ __device__ constexpr int twT_index(int N, int MA, int j, int k) {
  return j < 3 ? (j + 1) * k * (N / (4 * MA))
               : ((j - 3) % 3 + 1) * (k + MA * ((j - 3) / 3)) * (N / (16 * MA));
}

// LoRaDemod.cpp:59-67 max_amp of frame f from k_frame_max's partials.
__device__ __forceinline__ float frame_maxv(const KArgs& a, int64_t f) {
  float m = 0.0f;
  for (int c = 0; c < a.mx_bpf; ++c) m = fmaxf(m, __uint_as_float(a.maxbits[f * a.mx_bpf + c]));
  return m;
}

// ChirpGenerator.hpp:105-132 genChirp on the host (the fp32 recurrence, glibc sincosf):
// the plan's down-chirp tables and the C++ drop-in's genChirp (lora_phy_dropin.cpp).
void host_gen_chirp(std::complex<float>* out, int N, int osr, int NN, float f0, bool down, float ampl,
                    float& phase, float bw_scale);

// Fast symbol demodulator (lora_demod_fast.hip): register-blocked kissfft-exact FFT.
// Returns false if the configuration is not covered (caller uses the generic kernel).
bool launch_demod_fast(const KArgs& a, int s0, int64_t work, hipStream_t st);

// Speculative single-read pipeline, SF 6-12, LEGACY osr-1 unwindowed frames with >= 3
// symbols (lora_capi.hip): stage 0 = the pre-pass (estimate on unscaled samples + the
// maximum outside the data windows), 1 = k_spec_demod (every data symbol, window maxima
// and certification margins), 2 = k_est_fast<SPEC=2> (exact estimate, outputs, sync word,
// certification; rejected symbols listed), 3 = k_spec_fix (the listed symbols recomputed
// exactly).  a.mx_bpf = 1.
bool launch_spec(const KArgs& a, int64_t frames, int stage, hipStream_t st);

// Offset estimate + sync symbols with the same FFT machinery, one lane group per frame
// (frames with >= 2 whole symbols; false = not covered, use k_estimate).
bool launch_est_fast(const KArgs& a, int64_t frames, hipStream_t st);

// ---- launch recording: the C++ drop-in's allocation-free dispatch (lora_aql.hip) -------
// Every kernel launch of lora_demod_batch goes through lora::launch.  Normally that is
// hipLaunchKernelGGL; while a thread has a LaunchRecord installed (t_launch_record) the
// launch is recorded instead - kernel host stub, 1-D grid and block, dynamic LDS, and the
// explicit kernel arguments packed at their C++ ABI offsets (what the code object's
// kernarg metadata lists, tests/test_aql_kernargs.py) - and lora_aql.hip later writes it
// as an AQL dispatch packet into a queue of its own, with no HIP call and so no host
// allocation per call (the reference's no_alloc_test.cpp:90-99 guard).
struct RecordedLaunch {
  static constexpr unsigned kArgBytes = 384;  // explicit arguments (the kernels use <= 264)
  const void* fn;
  unsigned grid, block, lds, arg_bytes;
  alignas(16) unsigned char args[kArgBytes];
};
struct LaunchRecord {
  static constexpr int kMax = 6;
  RecordedLaunch l[kMax];
  int n = 0;
  bool bad = false;  // an unsupported launch (more than kMax, a 2-D/3-D shape, a memset)
};
extern thread_local LaunchRecord* t_launch_record;

template <class... P>
void record_launch(LaunchRecord& r, const void* fn, dim3 grid, dim3 block, size_t lds, P... v) {
  if (r.n >= LaunchRecord::kMax || grid.y != 1 || grid.z != 1 || block.y != 1 || block.z != 1) {
    r.bad = true;
    return;
  }
  RecordedLaunch& L = r.l[r.n++];
  L.fn = fn;
  L.grid = grid.x;
  L.block = block.x;
  L.lds = (unsigned)lds;
  size_t off = 0;
  auto put = [&](const void* p, size_t size, size_t align) {
    off = (off + align - 1) / align * align;
    if (off + size > RecordedLaunch::kArgBytes) {
      r.bad = true;
      return;
    }
    __builtin_memcpy(L.args + off, p, size);
    off += size;
  };
  (put(&v, sizeof(P), alignof(P)), ...);
  L.arg_bytes = (unsigned)off;
}

template <class... P, class... A>
inline void launch(void (*k)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t st, A&&... args) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  if (LaunchRecord* r = t_launch_record) {
    record_launch<P...>(*r, reinterpret_cast<const void*>(k), grid, block, lds, static_cast<P>(args)...);
    return;
  }
  hipLaunchKernelGGL(k, grid, block, lds, st, static_cast<P>(args)...);
}

// A private AQL queue on the device's HSA agent (lora_aql.hip).  aql_run writes the
// record's launches as dispatch packets (barrier bit: in order; system-scope acquire on
// the first and release on the last, so host-resident inputs and outputs are coherent),
// rings the doorbell once and waits for the last packet's completion signal.  Kernel
// objects are found once per kernel in the code object the HIP runtime loaded
// (hipKernelNameRefByPtr + the HSA loader extension) and cached.  Return 0 or a negative
// code naming the step that failed (aql_create: -101 .. -110, -111 the library's code objects are compressed bundles; aql_run, before any packet is
// written: -22 an unusable record, -120 a kernel object not found, -121 an unexpected kernarg
// layout, -63 the queue is not idle or broken; after dispatch: -62 timeout, after which the
// queue is broken - its packets may still run - and aql_destroy leaves it alone).
struct AqlQueue;
int aql_create(int device, AqlQueue** out);
int aql_run(AqlQueue* q, const LaunchRecord& r);
void aql_destroy(AqlQueue* q);

}  // namespace lora
