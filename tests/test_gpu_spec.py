"""GPU: the speculative single-read pipeline (LORA_MI355X_SPEC, default on) is exact.

The pipeline (lora_capi.hip) demodulates every data symbol with offsets
estimated on the UNSCALED frame, then certifies each symbol against the exact
(LoRaDemod.cpp:59-67 rescaled) estimate through a rounding-error bound on its
top-bin / runner-up margin and recomputes the symbols it cannot certify.  These tests
drive the three outcomes against the CPU oracle, bit for bit:

  * verbatim frames (max(|I|,|Q|) <= 1: no rescaling, nothing to certify),
  * certified frames (max > 1, margins far above the bound),
  * recomputed symbols (exact ties between two bins, a tie in the sync pair that moves
    the time offset, low SNR), which lora_demod_spec_recomputed() counts,

over SF 6-12, plus the eligibility boundary (3 .. 2 + kSpecChunks * N/16 symbols) and the three-launch
path the pipeline replaces.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

SPEC = {"spec", "estimate", "demod"}


@pytest.fixture(scope="module")
def O():
    from oracle.pyoracle import Oracle

    return Oracle()


@pytest.fixture(scope="module")
def amd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lora_phy_amd

    return lora_phy_amd


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def check(O, amd, iq, sf, spec=True):
    """Run `iq` ([F, L] dechirped frames) through a fresh plan and compare every output
    with the oracle; returns (plan, recomputed symbols).  spec=False: three-launch path."""
    with amd.spec_pipeline(spec):
        plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=False)
    res = plan.run(torch.from_numpy(np.ascontiguousarray(iq)).cuda())
    torch.cuda.synchronize()
    syms = res.symbols.cpu().numpy()
    sync = res.sync.cpu().numpy()
    cfo = res.cfo.cpu().numpy()
    toff = res.time_offset.cpu().numpy()
    for f in range(iq.shape[0]):
        osym, osync, ocfo, otoff = O.lora_demodulate(iq[f], sf, 1, False)
        assert syms.shape[1] == len(osym)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f} symbols")
        assert sync[f] == osync, f"frame {f} sync"
        assert bits(cfo[f]) == bits(ocfo), f"frame {f} cfo {cfo[f]} vs {ocfo}"
        assert bits(toff[f]) == bits(otoff), f"frame {f} toff {toff[f]} vs {otoff}"
    return plan, plan.spec_recomputed()


def tone(N, k, amp=1.0, ph=0.0):
    n = np.arange(N)
    return (amp * np.exp(1j * (2 * np.pi * k * n / N + ph))).astype(np.complex64)


def modulated(O, rng, sf, S, F, amp=1.0, noise=0.0):
    """F dechirped frames of S symbols (2 sync + S-2 data) at amplitude `amp` plus complex
    Gaussian noise of standard deviation `noise` per component."""
    N = 1 << sf
    out = np.zeros((F, S * N), np.complex64)
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.dechirp(O.lora_modulate(syms, sf, 1, 125000, amp, int(rng.integers(0, 256))), sf, 1)[: S * N]
        if noise > 0:
            x = x + noise * (rng.standard_normal(S * N) + 1j * rng.standard_normal(S * N))
        out[f] = x.astype(np.complex64)
    return out


@pytest.mark.parametrize("sf", [6, 7, 8, 9, 10, 11, 12])
def test_unscaled_frames(O, amd, sf):
    """max(|I|,|Q|) <= 1: the scale is 1 and the pre-pass estimate IS the exact one; the
    symbols (hardware rotation) are certified, and a frame whose estimated CFO sits near
    half a bin (two bins of almost equal power in every data symbol, e.g. frame 5 at SF7
    here) has a few recomputed."""
    rng = np.random.default_rng(100 + sf)
    iq = modulated(O, rng, sf, 8 if sf < 11 else 5, 6, amp=0.5, noise=0.05)
    assert np.abs(iq.view(np.float32)).max() <= 1.0
    plan, fixed = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC
    assert fixed <= iq.shape[0] * (iq.shape[1] // (1 << sf) - 2) // 4


@pytest.mark.parametrize("sf", [6, 7, 8, 9, 10, 11, 12])
@pytest.mark.parametrize("snr_db", [20, 0, -10, -15])
def test_rescaled_frames_match_oracle(O, amd, sf, snr_db):
    """max > 1 (rescaled) at high and low SNR: certified or recomputed, always exact."""
    rng = np.random.default_rng(1000 * sf + snr_db + 50)
    amp = 2.5
    noise = amp * 10 ** (-snr_db / 20) / np.sqrt(2)
    iq = modulated(O, rng, sf, 10 if sf < 11 else 5, 8 if sf < 10 else 3, amp=amp, noise=noise)
    assert np.abs(iq.view(np.float32)).max() > 1.0
    plan, fixed = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC
    assert fixed >= 0


@pytest.mark.parametrize("sf", [6, 7, 9, 12])
def test_equal_power_tie_is_recomputed(O, amd, sf):
    """Two data-symbol bins of exactly equal power (equal_power_bin_test.cpp's case in the
    dechirped domain): the margin is ~0, no bound certifies it, the symbol is recomputed
    exactly and the lowest index wins as in the reference.  The sync pair is bin 0 in
    phase, so the estimate is (close to) no rotation and the two bins stay equal."""
    N = 1 << sf
    S, F = 6, 4
    iq = np.zeros((F, S * N), np.complex64)
    for f in range(F):
        iq[f, :N] = tone(N, 0, 1.7)
        iq[f, N:2 * N] = tone(N, 0, 1.7)
        for s in range(2, S):
            a, b = (5 * s + f) % N, (N // 2 + 7 * s + f) % N
            iq[f, s * N:(s + 1) * N] = tone(N, a, 1.3) + tone(N, b, 1.3, 0.7)
    plan, fixed = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC
    assert fixed > 0


def test_sync_pair_tie_moves_time_offset(O, amd):
    """Equal-power bins in symbol 0 (the time-offset estimate's input) at max > 1: the
    scaled and unscaled estimates may pick different t_off, which sends the whole frame to
    exact recomputation; every frame still matches the oracle."""
    sf, N, S, F = 7, 128, 8, 16
    rng = np.random.default_rng(9)
    iq = np.zeros((F, S * N), np.complex64)
    for f in range(F):
        iq[f, :N] = tone(N, 10 + f, 1.1) + tone(N, 40 + 3 * f, 1.1, 0.3 * f)
        iq[f, N:2 * N] = tone(N, 20 + f, 1.4)
        for s in range(2, S):
            iq[f, s * N:(s + 1) * N] = tone(N, int(rng.integers(0, N)), 1.2)
        iq[f] += (0.01 * (rng.standard_normal(S * N) + 1j * rng.standard_normal(S * N))).astype(np.complex64)
    check(O, amd, iq, sf)


@pytest.mark.parametrize("amp", [0.0, 1.0, 1.0000001, 3e4, 1e-30])
def test_amplitude_extremes(O, amd, amp):
    """Zero frames (max 0), max exactly 1 and one ulp above, huge and tiny amplitudes."""
    rng = np.random.default_rng(int(amp * 7) % 1000 + 3)
    sf = 7
    iq = modulated(O, rng, sf, 6, 4, amp=1.0)
    m = np.abs(iq.view(np.float32)).max()
    iq = (iq * np.float32(amp / m)).astype(np.complex64) if amp > 0 else np.zeros_like(iq)
    plan, _ = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC


@pytest.mark.parametrize("sf,nsym,spec", [(7, 2, False), (7, 3, True), (9, 82, True), (6, 258, True),
                                          (6, 259, False), (12, 3, True), (6, 40, True)])
def test_eligibility_boundary(O, amd, sf, nsym, spec):
    """The pipeline covers frames of 3 .. 2 + kSpecChunks * N/16 symbols (SF6: 258); others
    take the three-launch path; both are exact."""
    rng = np.random.default_rng(sf * 100 + nsym)
    iq = modulated(O, rng, sf, nsym, 2, amp=1.8, noise=0.3)
    plan, _ = check(O, amd, iq, sf)
    assert ("spec" in plan.last_kernels()) == spec
    if not spec:
        assert "frame_max" in plan.last_kernels() or "frame_max_wave" in plan.last_kernels()


@pytest.mark.parametrize("sf", [7, 12])
def test_three_launch_path_agrees(O, amd, sf):
    """LORA_MI355X_SPEC=0 (frame max, estimate, demod) on the same rescaled low-SNR frames."""
    rng = np.random.default_rng(sf + 31)
    iq = modulated(O, rng, sf, 8 if sf < 12 else 5, 4, amp=2.0, noise=2.0)
    plan, fixed = check(O, amd, iq, sf, spec=False)
    assert "spec" not in plan.last_kernels()
    assert fixed == 0


@pytest.mark.parametrize("sf", [6, 8, 10, 11, 12])
def test_mixed_frames_in_one_block(O, amd, sf):
    """Rescaled and unscaled frames side by side (one block holds 256 / T frames; SF11 two
    frames of two waves each): the unscaled frames leave the estimate kernels early, the
    others continue through the block's barriers."""
    rng = np.random.default_rng(300 + sf)
    F = 8 if sf < 11 else 4
    iq = modulated(O, rng, sf, 5, F, amp=0.6, noise=0.02)
    iq[1::2] *= np.float32(4.0)
    if F > 2:
        iq[2, 7] = np.complex64(1.5 + 0.0j)  # rescaled by a single sample in symbol 0
    plan, _ = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC


@pytest.mark.parametrize("sf", [6, 7, 8, 9])
def test_scale_guess_holds_and_fails(O, amd, sf):
    """The SF 6-9 pre-pass normalises symbols 0/1 by their own maximum (k_est_split's scale
    guess) and stage 2 takes that estimate as the exact one only when the frame's maximum
    gives the same scale.  Frames of every case side by side, so a stage-2 wave (64 / 2T
    frames) holds several: the guess holds with max > 1 (noiseless frames that dechirp to
    1 + 2^-23, and a 1.7 sync peak that is the frame's), it fails because a data window
    exceeds the sync windows' maximum (both > 1, or sync <= 1 < data), it holds with the
    whole frame <= 1, and two maxima with the same reciprocal in float (1/m equal, m not)."""
    rng = np.random.default_rng(500 + sf)
    N = 1 << sf
    S = 8
    base = modulated(O, rng, sf, S, 12, amp=1.0)  # noiseless: max 1 or 1 + ulp everywhere
    iq = base.copy()
    iq[1] *= np.float32(1.7)                       # guess holds, scaled
    iq[2, 5 * N + 3] = np.complex64(3.0 + 0.5j)    # data window above the sync windows' 1 + ulp
    iq[3] *= np.float32(0.6)                       # whole frame <= 1
    iq[4] *= np.float32(0.6)
    iq[4, 6 * N + 11] = np.complex64(0.2 - 1.25j)  # sync <= 1 < data: guess unscaled, frame scaled
    iq[5] *= np.float32(2.0)
    ms = np.abs(iq[5, :2 * N].view(np.float32)).max()
    iq[5, 4 * N + 7] = np.complex64(complex(np.nextafter(ms, np.float32(4.0), dtype=np.float32), 0.0))  # one ulp above
    # two different maxima whose reciprocals round to the same float: sync max m0, a data
    # sample m1 > m0 with fl(1/m1) == fl(1/m0) (the reference's inputs are then identical)
    m0 = np.float32(1.5)
    for _ in range(10000):
        m1 = np.nextafter(m0, np.float32(2.0), dtype=np.float32)
        if np.float32(1.0) / m1 == np.float32(1.0) / m0:
            break
        m0 = m1
    assert np.float32(1.0) / m1 == np.float32(1.0) / m0 and m1 > m0
    iq[6] = (base[6] / np.float32(np.abs(base[6].view(np.float32)).max()) * np.float32(0.9)).astype(np.complex64)
    iq[6, 5] = np.complex64(complex(m0, 0.0))          # symbol 0: the sync windows' maximum
    iq[6, 3 * N + 1] = np.complex64(complex(0.0, m1))  # a data window: the frame's
    iq[7] = (iq[7] + 0.3 * (rng.standard_normal(S * N) + 1j * rng.standard_normal(S * N))).astype(np.complex64)
    plan, _ = check(O, amd, iq, sf)
    assert plan.last_kernels() == SPEC


def test_ragged_tail_and_many_frames(O, amd):
    """Frame length not a symbol multiple (the tail is ignored) over 700 frames (many lane
    groups per launch), mixed amplitudes."""
    sf, N = 8, 256
    rng = np.random.default_rng(17)
    F = 700
    base = modulated(O, rng, sf, 5, 8, amp=1.0, noise=0.2)
    iq = np.concatenate([base[rng.integers(0, 8, F)], np.zeros((F, 37), np.complex64)], axis=1)
    iq *= rng.choice([0.3, 1.0, 2.0, 50.0], F).astype(np.float32)[:, None]
    iq[:, -37:] = (5 * rng.standard_normal((F, 37))).astype(np.complex64)
    iq = iq.astype(np.complex64)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=False)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert plan.last_kernels() == SPEC
    syms = res.symbols.cpu().numpy()
    cfo = res.cfo.cpu().numpy()
    for f in range(0, F, 7):
        osym, osync, ocfo, otoff = O.lora_demodulate(iq[f], sf, 1, False)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert bits(cfo[f]) == bits(ocfo)
        assert int(res.sync[f]) == osync
        assert bits(res.time_offset[f].item()) == bits(otoff)


@pytest.mark.parametrize("sf,snr_db", [(7, 20), (7, -10), (9, 0), (12, 10)])
def test_fast_precision_rescaled_frames_are_exact(O, amd, sf, snr_db):
    """LORA_PRECISION_FAST in the pipeline: the hardware-sin/cos symbols of rescaled frames
    are certified against the EXACT reference (bound widened by the rotation's phase
    error) or recomputed exactly, so every output equals the oracle's."""
    rng = np.random.default_rng(700 + sf + snr_db)
    amp = 2.0
    noise = amp * 10 ** (-snr_db / 20) / np.sqrt(2)
    iq = modulated(O, rng, sf, 10 if sf < 12 else 5, 8 if sf < 12 else 3, amp=amp, noise=noise)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=False, precision="fast")
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert plan.last_kernels() == SPEC
    syms = res.symbols.cpu().numpy()
    for f in range(iq.shape[0]):
        osym, osync, ocfo, otoff = O.lora_demodulate(iq[f], sf, 1, False)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync
        assert bits(res.cfo[f].item()) == bits(ocfo)
        assert bits(res.time_offset[f].item()) == bits(otoff)


@pytest.mark.parametrize("path", ["spec", "split"])
@pytest.mark.parametrize("sf,dechirp", [(7, True), (7, False), (9, True), (12, True)])
def test_max_amp_is_the_reference_frame_maximum(O, amd, sf, dechirp, path):
    """max_amp (LoRaDemod.cpp:59-67: max of |I|, |Q| over the whole frame as handed to
    lora_demodulate, i.e. after the caller's dechirp) bit for bit, with the rescaling it
    drives: the pipeline assembles it from window maxima of exactly-dechirped samples (the
    demod's fused multiply-adds must not reach them).  Frames of random symbols at random
    amplitude around 1, some with a ragged tail."""
    N = 1 << sf
    S = 6 if sf < 12 else 4
    F = 48 if sf < 12 else 8
    rng = np.random.default_rng(4242 + sf + dechirp)
    L = S * N + 29
    iq = np.zeros((F, L), np.complex64)
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, int(rng.integers(0, 256)))[: S * N]
        x = x * np.float32(rng.uniform(0.6, 1.6))
        x = x + np.float32(0.2) * (rng.standard_normal(S * N) + 1j * rng.standard_normal(S * N))
        if not dechirp:
            x = O.dechirp(x.astype(np.complex64), sf, 1)
        iq[f, : S * N] = x.astype(np.complex64)
        iq[f, S * N:] = (0.3 * rng.standard_normal(L - S * N)).astype(np.complex64)
    with amd.spec_pipeline(path != "split"):
        plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=dechirp)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert ("spec" in plan.last_kernels()) == (path != "split")
    got = res.max_amp.cpu().numpy()
    syms = res.symbols.cpu().numpy()
    for f in range(F):
        xd = O.dechirp(iq[f], sf, 1) if dechirp else iq[f]
        ref = np.abs(xd.view(np.float32)).max()
        assert bits(got[f]) == bits(ref), f"frame {f}: max_amp {got[f]!r} vs {ref!r}"
        osym, osync, ocfo, otoff = O.lora_demodulate(xd, sf, 1, False)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert bits(res.cfo[f].item()) == bits(ocfo)
        assert bits(res.time_offset[f].item()) == bits(otoff)


@pytest.mark.parametrize("sf,S,F", [(7, 81, 24), (9, 81, 8), (12, 24, 4)])
@pytest.mark.parametrize("snr_db", [10, -5])
def test_fused_dechirp_large_cfo_and_delay(O, amd, sf, S, F, snr_db):
    """The benchmark's path (LEGACY, fused caller dechirp): frames with a carrier offset of
    up to +-0.45 bin, a random sample delay (so t_off != 0 and every window starts at a
    table phase cg != 0 of the paired dechirp table) and long frames (81 symbols here;
    tests/test_gpu_scale.py goes to 514: the largest rotation phases the certification bound must cover, which for the
    recurrence-built rotation factors grows with rate * L), against the oracle on the
    caller-dechirped frames, bit for bit."""
    N = 1 << sf
    rng = np.random.default_rng(7000 + 10 * sf + snr_db)
    L = S * N
    iq = np.zeros((F, L), np.complex64)
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, int(rng.integers(0, 256))).astype(np.complex128)
        cfo = rng.uniform(-0.45, 0.45)
        x = x * np.exp(2j * np.pi * cfo * np.arange(len(x)) / N)
        d = int(rng.integers(1, N // 3))
        x = np.concatenate([np.zeros(d), x])[:L]
        amp = rng.uniform(0.7, 1.5)
        sigma = amp * 10 ** (-snr_db / 20) / np.sqrt(2)
        x = amp * x + sigma * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        iq[f] = x.astype(np.complex64)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert "spec" in plan.last_kernels()
    syms = res.symbols.cpu().numpy()
    nz = 0
    for f in range(F):
        xd = O.dechirp(iq[f], sf, 1)
        osym, osync, ocfo, otoff = O.lora_demodulate(xd, sf, 1, False)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync
        assert bits(res.cfo[f].item()) == bits(ocfo)
        assert bits(res.time_offset[f].item()) == bits(otoff)
        nz += otoff != 0
    assert nz > 0, "no frame exercised a non-zero time offset"


@pytest.mark.parametrize("sf,S,F,dechirp", [(6, 40, 16, True), (7, 66, 24, True), (7, 20, 12, False),
                                            (9, 30, 6, True), (10, 12, 4, False), (12, 8, 3, True)])
@pytest.mark.parametrize("snr_db", [20, -5])
def test_hann_window_through_the_pipeline(O, amd, sf, S, F, dechirp, snr_db):
    """Hann-windowed frames (LoRaDemod.cpp:88-92, 158-160: the window multiplies every
    sample after the rotation, in the estimate and in the symbol loop) take the speculative
    pipeline (the window's product is one more rounding in the certification bound, |w| <= 1
    keeps the bound's n1): carrier offsets up to +-0.45 bin and random delays (t_off != 0),
    against the oracle bit for bit, fused caller dechirp and dechirped input."""
    N = 1 << sf
    rng = np.random.default_rng(9100 + 10 * sf + snr_db + S)
    L = S * N
    iq = np.zeros((F, L), np.complex64)
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, int(rng.integers(0, 256))).astype(np.complex128)
        x = x * np.exp(2j * np.pi * rng.uniform(-0.45, 0.45) * np.arange(len(x)) / N)
        d = int(rng.integers(0, N // 3))
        x = np.concatenate([np.zeros(d), x])[:L]
        amp = rng.uniform(0.7, 1.5)
        sigma = amp * 10 ** (-snr_db / 20) / np.sqrt(2)
        x = amp * x + sigma * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        iq[f] = x.astype(np.complex64)
    plan = amd.DemodPlan(sf, 1, 125000, "hann", dechirp=dechirp)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert "spec" in plan.last_kernels()
    syms = res.symbols.cpu().numpy()
    for f in range(F):
        xd = O.dechirp(iq[f], sf, 1) if dechirp else iq[f]
        osym, osync, ocfo, otoff = O.lora_demodulate(xd, sf, 1, True)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync, f"frame {f} sync"
        assert bits(res.cfo[f].item()) == bits(ocfo), f"frame {f} cfo"
        assert bits(res.time_offset[f].item()) == bits(otoff), f"frame {f} toff"


@pytest.mark.parametrize("sf", [6, 7, 8, 9, 10, 12])
@pytest.mark.parametrize("hann", [False, True])
@pytest.mark.parametrize("snr_db", [20, -10])
def test_api_mode_through_the_pipeline(O, amd, sf, hann, snr_db):
    """LORA_MODE_API (lora_phy::demodulate, phy.cpp:178-239) at osr 1 takes the pipeline: the
    exact estimate with the sync word first, then the symbol pass with those offsets (the
    down-chirp from table phase 0, hardware rotation), each symbol certified with no rate
    difference or recomputed exactly.  Raw modulated frames with a carrier offset, a sample
    delay (t_off != 0: misaligned windows), noise; every output bit-equal to the reference's
    API demodulate, and the three-launch path (LORA_MI355X_SPEC=0) agrees."""
    rng = np.random.default_rng(700 + 10 * sf + hann + (snr_db < 0))
    N = 1 << sf
    F, S = (6, 10) if sf < 11 else (3, 6)
    frames = []
    noise = 10 ** (-snr_db / 20) / np.sqrt(2)
    for f in range(F):
        syms = rng.integers(0, N, S).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, 0x34)
        n = np.arange(len(x))
        x = x * np.exp(2j * np.pi * (0.3 + 0.05 * f) * n / N)  # carrier offset, in bins
        x = np.roll(x, f)  # a delay of f samples
        x = x + noise * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x)))
        frames.append(x.astype(np.complex64))
    iq = np.stack(frames)
    window = "hann" if hann else "none"
    for spec in (True, False):
        with amd.spec_pipeline(spec):
            plan = amd.DemodPlan(sf, 1, 125000, window, mode="api")
        res = plan.run(torch.from_numpy(iq).cuda())
        torch.cuda.synchronize()
        assert ("spec" in plan.last_kernels()) == spec
        syms = res.symbols.cpu().numpy()
        for f in range(F):
            r, osym, osync, ocfo, otoff = O.api_demodulate(iq[f], sf, 1, hann)
            assert r == S
            np.testing.assert_array_equal(syms[f], osym, err_msg=f"spec={spec} frame {f}")
            assert int(res.sync[f]) == osync
            assert bits(res.cfo[f].item()) == bits(ocfo)
            assert bits(res.time_offset[f].item()) == bits(otoff)


@pytest.mark.parametrize("sf", [6, 7, 8, 9])
@pytest.mark.parametrize("hann", [False, True])
@pytest.mark.parametrize("dechirp", [True, False])
def test_raw_mode_through_the_pipeline(O, amd, sf, hann, dechirp):
    """LORA_MODE_RAW (the detector alone, awgn_sweep.py:262-273) at osr 1, SF 6-9 takes the
    pipeline: every symbol of the frame through the symbol pass (no offsets, no rotation),
    certified against the transforms' rounding alone (k_cert_raw) or recomputed exactly.
    Frames from noiseless to -15 dB (many near-ties), two exact equal-power ties and a
    ragged tail; every symbol equal to the reference's detector, and to the three-launch
    path."""
    rng = np.random.default_rng(900 + 10 * sf + 2 * hann + dechirp)
    N = 1 << sf
    F, S = 8, 9
    L = S * N + 5
    rows = []
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, 0x12)
        if not dechirp:
            x = O.dechirp(x, sf, 1)
        x = np.concatenate([x, np.zeros(5, np.complex64)])
        sig = [0.0, 0.3, 1.0, 3.0, 4.0, 0.0, 0.5, 2.0][f]
        x = (x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L))).astype(np.complex64)
        rows.append(x)
    iq = np.stack(rows)
    # two symbols of frame 5 with two bins of exactly equal power (dechirped domain)
    if not dechirp:
        for s in (3, 6):
            iq[5, s * N:(s + 1) * N] = tone(N, 5 + s, 1.3) + tone(N, N // 2 + s, 1.3, 0.7)
    for spec in (True, False):
        with amd.spec_pipeline(spec):
            plan = amd.DemodPlan(sf, 1, 125000, "hann" if hann else "none", dechirp=dechirp, mode="raw")
        res = plan.run(torch.from_numpy(iq).cuda())
        torch.cuda.synchronize()
        assert ("spec" in plan.last_kernels()) == spec
        got = res.symbols.cpu().numpy()
        assert got.shape == (F, S)
        for f in range(F):
            np.testing.assert_array_equal(got[f], O.raw_demod(iq[f], sf, 1, hann, dechirp=dechirp),
                                          err_msg=f"spec={spec} frame {f}")
        assert int(res.sync.to(torch.int32).sum()) == 0 and float(res.cfo.abs().sum()) == 0.0
        if spec and not dechirp:
            assert plan.spec_recomputed() > 0  # the ties at least


@pytest.mark.parametrize("dechirp", [True, False])
@pytest.mark.parametrize("snr_db", [None, 5.0, -10.0])
def test_sf7_whole_line_pass_every_line_offset(O, amd, dechirp, snr_db):
    """The SF7 whole-line symbol pass (k_spec_demod PL: lane l holds residues (2l + h - d) mod
    16 of a window at offset d in its 128-byte line, late elements from the 9th line) at every
    offset d = 0..15 - a fractional carrier offset per frame from -0.5 to +0.5 bin (estimated
    time offsets from -64 to +63 samples), sample delays and advances, the windows' last line
    taken from the next lane group or from the late elements' own loads (a wave's last group,
    frame ends) - every symbol, sync word and cfo / time_offset bit against the oracle."""
    sf, N, F, S = 7, 128, 48, 21  # 21 data symbols: blocks of 8 with a partial last one
    rng = np.random.default_rng(7000 + (0 if snr_db is None else int(snr_db) + 100) + int(dechirp))
    L = (S + 2) * N
    iq = np.zeros((F, L), np.complex64)
    n = np.arange(L)
    for f in range(F):
        syms = rng.integers(0, N, S).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, int(rng.integers(0, 256)))
        d = f % 16 + 16 * (f // 16 % 2)  # offsets 0..31: every d, both halves of a symbol's lead
        x = np.concatenate([np.zeros(d, np.complex64), x])[:L] if f % 3 else np.concatenate([x[d:], np.zeros(d, np.complex64)])
        # a fractional carrier offset per frame: the estimate's time offset is -frac N
        # (LoRaDemod.cpp:127-131), so the frames' windows start at every offset in a line
        x = (x * np.exp(2j * np.pi * ((f + 0.37) / F - 0.5) * n / N)).astype(np.complex64)
        if snr_db is not None:
            sigma = 10.0 ** (-snr_db / 20.0) / np.sqrt(2.0)
            x = x + sigma * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        iq[f] = x.astype(np.complex64)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=dechirp)
    host = iq if dechirp else np.stack([O.dechirp(iq[f], sf) for f in range(F)]).astype(np.complex64)
    res = plan.run(torch.from_numpy(host).cuda())
    torch.cuda.synchronize()
    assert plan.last_kernels() == SPEC
    syms = res.symbols.cpu().numpy()
    toffs = set()
    for f in range(F):
        osym, osync, ocfo, otoff = O.lora_demodulate(O.dechirp(iq[f], sf), sf, 1, False)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync, f"frame {f} sync"
        assert bits(res.cfo[f].item()) == bits(ocfo) and bits(res.time_offset[f].item()) == bits(otoff), f"frame {f}"
        toffs.add(int(round(float(otoff))) % 16)
    if snr_db is None:
        assert len(toffs) >= 12, toffs  # the line offsets the frames exercised


@pytest.mark.parametrize("osr,window", [(1, "none"), (2, "none"), (4, "none"), (1, "hann")])
def test_frames_at_unaligned_addresses(O, amd, osr, window):
    """Frames that start 8 bytes off a 16-byte boundary - an odd row stride and an odd first
    sample (a view into a larger tensor) - through the pipeline's 16-byte sample loads (SF7's
    whole-line pass, osr 2's point pairs, osr 4's line pairs; Hann takes the 8-byte loop):
    every output equal to the oracle's."""
    sf, N, F, S = 7, 128, 12, 20
    L = (S + 2) * N * osr
    rng = np.random.default_rng(4040 + osr)
    big = np.zeros((F, L + 3), np.complex64)  # row stride L + 3: odd
    for f in range(F):
        syms = rng.integers(0, N, S).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, 0x34)
        x = x * np.exp(2j * np.pi * ((f + 0.5) / F - 0.5) * np.arange(L) / (N * osr))
        x = x + 0.2 * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        big[f, 1:1 + L] = x.astype(np.complex64)
    t = torch.from_numpy(big).cuda()[:, 1:1 + L]  # first sample 8 bytes past the row start
    assert t.stride(0) % 2 == 1 and (t.data_ptr() % 16) == 8
    plan = amd.DemodPlan(sf, osr, 125000, window, dechirp=True)
    res = plan.run(t)
    torch.cuda.synchronize()
    assert "spec" in plan.last_kernels()
    syms = res.symbols.cpu().numpy()
    for f in range(F):
        osym, osync, ocfo, otoff = O.lora_demodulate(O.dechirp(big[f, 1:1 + L], sf, osr), sf, osr, window == "hann")
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync
        assert bits(res.cfo[f].item()) == bits(ocfo) and bits(res.time_offset[f].item()) == bits(otoff)
