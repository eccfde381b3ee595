"""Oversampled LEGACY frames (osr 2-4) through the speculative single-read pipeline.

The reference's decimating demod reads sym_samps[i * osr] after a maximum over EVERY sample
of the frame and an offset estimate over the osr phases of symbols 0/1
(/root/reference/src/phy/LoRaDemod.cpp:59-77, 86-111, 141-162); its only real-capture
fixture is osr 2 (tests/gr_lora_sdr_interop.cpp:34).  Here each frame is read once: the
symbol pass transforms every osr-th sample of a window and takes the window's maximum over
all of them (k_spec_demod<..., OSRV>: osr 2 / 4 in 16-byte loads, 3 and Hann at run-time osr), the pre-pass / stage 2 estimate over the osr phases
(k_est_fast<SF, 2, 1|2>), rejected symbols recomputed exactly (k_spec_fix<SF, 2>).  Every
output is compared with the oracle bit for bit, and the plan must report the pipeline."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


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


def frames(O, rng, sf, osr, F, S, dechirp, snr_db, amp):
    """F frames of 2 sync + S data symbols at `osr`, a random delay of 0..step-1 samples
    (t_off != 0) and a random carrier offset, AWGN at snr_db (None: none), scaled by amp."""
    N = 1 << sf
    step = N * osr
    L = (S + 2) * step
    out = np.zeros((F, L), np.complex64)
    for f in range(F):
        syms = rng.integers(0, N, S).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, int(rng.integers(0, 256)))
        d = int(rng.integers(0, step)) if f % 2 else 0
        x = np.concatenate([np.zeros(d, np.complex64), x])[:L]
        n = np.arange(L)
        cfo = rng.uniform(-0.4, 0.4) / step
        x = (x * np.exp(2j * np.pi * cfo * n)).astype(np.complex64)
        if not dechirp:
            x = O.dechirp(x, sf, osr)
        if snr_db is not None:
            s = np.sqrt(0.5 * 10 ** (-snr_db / 10))
            x = x + s * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        out[f] = (x * amp).astype(np.complex64)
    return out


CASES = [  # (sf, osr, dechirp, hann, F, S, snr, amp)
    (7, 2, True, False, 24, 20, None, 1.0),   # gr_lora_sdr_interop's shape
    (7, 2, False, False, 16, 12, 0.0, 1.0),
    (7, 4, True, False, 8, 10, 10.0, 0.7),
    (7, 3, False, True, 8, 9, 5.0, 2.0),
    (6, 2, True, False, 12, 6, -5.0, 1.0),
    (8, 4, False, False, 6, 7, -10.0, 1.0),
    (9, 3, True, True, 4, 6, 3.0, 0.5),
    (10, 2, True, False, 3, 6, None, 3e4),
    (11, 4, False, False, 2, 4, 0.0, 1.0),
    (12, 2, True, False, 2, 4, -5.0, 1.0),
    (12, 4, False, True, 1, 3, 10.0, 1.5),
]


@pytest.mark.parametrize("case", CASES, ids=[f"sf{c[0]}-osr{c[1]}-d{int(c[2])}-h{int(c[3])}-snr{c[6]}-a{c[7]}"
                                             for c in CASES])
def test_oversampled_frames_through_the_pipeline(O, amd, case):
    sf, osr, dechirp, hann, F, S, snr, amp = case
    rng = np.random.default_rng(1000 * sf + 10 * osr + S)
    iq = frames(O, rng, sf, osr, F, S, dechirp, snr, amp)
    plan = amd.DemodPlan(sf, osr, 125000, "hann" if hann else "none", dechirp=dechirp)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    assert "spec" in plan.last_kernels(), plan.last_kernels()
    syms, sync = res.symbols.cpu().numpy(), res.sync.cpu().numpy()
    cfo, toff = res.cfo.cpu().numpy(), res.time_offset.cpu().numpy()
    for f in range(F):
        x = O.dechirp(iq[f], sf, osr) if dechirp else iq[f]
        osym, osync, ocfo, otoff = O.lora_demodulate(x, sf, osr, hann)
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f} symbols")
        assert sync[f] == osync, f"frame {f} sync"
        assert bits(cfo[f]) == bits(ocfo), f"frame {f} cfo {cfo[f]} vs {ocfo}"
        assert bits(toff[f]) == bits(otoff), f"frame {f} toff {toff[f]} vs {otoff}"
    print(f"\nsf{sf} osr{osr}: {F} frames bit-exact, {plan.spec_recomputed()} recomputed")


def test_interop_capture_osr2_takes_the_pipeline(O, amd):
    """The reference's real capture (tests/golden/test_output.iq, osr 2, sync 0x29) through
    the pipeline: the decoded payload and sync equal gr_lora_sdr_interop.cpp's expectations."""
    import os

    from lora_phy_amd import iq_io

    path = os.path.join(os.path.dirname(__file__), "golden", "test_output.iq")
    x = iq_io.read_iq(path).numpy()
    sf, osr = 7, 2
    plan = amd.DemodPlan(sf, osr, 125000, "none", dechirp=False)
    res = plan.run(torch.from_numpy(x[None, :]).cuda())
    torch.cuda.synchronize()
    assert "spec" in plan.last_kernels(), plan.last_kernels()
    osym, osync, ocfo, otoff = O.lora_demodulate(x, sf, osr, False)
    np.testing.assert_array_equal(res.symbols.cpu().numpy()[0], osym)
    assert int(res.sync[0]) == osync == 0x29
    assert bits(res.cfo.cpu().numpy()[0]) == bits(ocfo)
