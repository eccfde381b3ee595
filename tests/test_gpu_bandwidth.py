"""GPU parity at BW 250 / 500 kHz (phy.hpp:37-49 bw_scale), through the C-ABI, bit for bit.

Bandwidth enters the demodulator in two places, both covered here against the oracle (itself
pinned to the reference at these bandwidths by tests/test_oracle_vs_reference.py
::test_bandwidth_*):

* the caller-side dechirp every reference caller runs before lora_demodulate, with
  genChirp(..., bw_scale(p.bw)) (e2e_chain_test.cpp:84-93, performance_test.cpp:94-116,
  awgn_sweep_gtest.cpp:85-92) - fused into the kernels' loads here (params.dechirp = 1);
* lora_phy::demodulate's per-symbol down-chirp (phy.cpp:202-204) - LORA_MODE_API.

Each on the speculative single-read pipeline ("spec") and on the three-launch exact path
("split"), SF 7 / 9 / 12, osr 1 and 2, both windows, noiseless to noisy frames with sample
delays and a carrier offset.  And end to end on the GPU: lora_mod_batch at bw -> the fused
dechirp at bw -> (symbol * bw_scale) mod N, the reference's own behaviour.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

BWS = {125000: 1, 250000: 2, 500000: 4}


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


def frames_at(O, rng, sf, osr, bw, F, nsym, cfo_bins=0.0):
    """F frames of nsym data symbols modulated at `bw` by the oracle (bit-equal to the
    reference's lora_modulate), each delayed by a few samples, with a carrier offset and
    AWGN of a per-frame level (0 = noiseless)."""
    N = 1 << sf
    L = (nsym + 2) * N * osr
    out = np.zeros((F, L), np.complex64)
    n = np.arange(L)
    for f in range(F):
        syms = rng.integers(0, N, nsym).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, bw, 1.0, int(rng.integers(0, 256)))
        d = int(rng.integers(0, N * osr // 4)) if f % 3 else 0
        x = np.concatenate([np.zeros(d, np.complex64), x])[:L]
        if cfo_bins:
            x = (x * np.exp(2j * np.pi * cfo_bins * (n % (N * osr)) / (N * osr))).astype(np.complex64)
        sig = [0.0, 0.05, 0.4, 1.2][f % 4]
        if sig:
            x = x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L))
        out[f] = x.astype(np.complex64)
    return out


CASES = [  # (sf, osr, hann, frames, data symbols)
    (7, 1, False, 24, 30),
    (7, 1, True, 12, 20),
    (7, 2, False, 8, 12),
    (9, 1, False, 12, 16),
    (9, 2, True, 6, 8),
    (12, 1, False, 4, 8),
    (12, 2, True, 2, 4),
]


@pytest.mark.parametrize("path", ["spec", "split"])
@pytest.mark.parametrize("bw", [250000, 500000])
@pytest.mark.parametrize("case", CASES, ids=[f"sf{c[0]}-osr{c[1]}-h{int(c[2])}" for c in CASES])
def test_legacy_fused_dechirp_at_bandwidth(O, amd, case, bw, path):
    """LEGACY with the fused caller dechirp at bw: every symbol, sync word and cfo /
    time_offset bit equal to the oracle's lora_demodulate on the oracle's dechirp(bw)."""
    sf, osr, hann, F, nsym = case
    rng = np.random.default_rng(sf * 1000 + osr * 10 + bw // 1000 + int(hann))
    iq = frames_at(O, rng, sf, osr, bw, F, nsym, cfo_bins=0.2)
    plan = amd.DemodPlan(sf, osr, bw, "hann" if hann else "none", dechirp=True, pipeline=path)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    if path == "spec":
        assert "spec" in plan.last_kernels()
    else:
        assert "spec" not in plan.last_kernels()
    syms, sync = res.symbols.cpu().numpy(), res.sync.cpu().numpy()
    cfo, toff = res.cfo.cpu().numpy(), res.time_offset.cpu().numpy()
    for f in range(F):
        os_, osync, ocfo, otoff = O.lora_demodulate(O.dechirp(iq[f], sf, osr, bw), sf, osr, hann)
        np.testing.assert_array_equal(syms[f], os_, err_msg=f"frame {f} symbols")
        assert sync[f] == osync, f"frame {f} sync"
        assert bits(cfo[f]) == bits(ocfo), f"frame {f} cfo"
        assert bits(toff[f]) == bits(otoff), f"frame {f} time_offset"


@pytest.mark.parametrize("path", ["spec", "split"])
@pytest.mark.parametrize("bw", [250000, 500000])
@pytest.mark.parametrize("sf,osr,hann", [(7, 1, False), (7, 1, True), (9, 1, False), (9, 2, True), (12, 1, False),
                                         (12, 2, False)])
def test_api_mode_at_bandwidth(O, amd, sf, osr, hann, bw, path):
    """LORA_MODE_API (lora_phy::demodulate, its down-chirp generated with bw_scale,
    phy.cpp:202-204) at bw: return count, symbols, sync, cfo / time_offset bits equal to the
    oracle's api_demodulate(bw)."""
    rng = np.random.default_rng(sf * 77 + osr + bw // 1000 + int(hann))
    F, nsym = (6, 8) if sf < 12 else (3, 4)
    iq = frames_at(O, rng, sf, osr, bw, F, nsym)
    plan = amd.DemodPlan(sf, osr, bw, "hann" if hann else "none", mode="api", pipeline=path)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    if path == "spec" and osr == 1:
        assert "spec" in plan.last_kernels()
    syms = res.symbols.cpu().numpy()
    for f in range(F):
        r, osym, osync, ocfo, otoff = O.api_demodulate(iq[f], sf, osr, hann, bw=bw)
        assert r == nsym
        np.testing.assert_array_equal(syms[f], osym, err_msg=f"frame {f}")
        assert int(res.sync[f]) == osync
        assert bits(res.cfo[f].item()) == bits(ocfo)
        assert bits(res.time_offset[f].item()) == bits(otoff)


@pytest.mark.parametrize("bw", [250000, 500000])
@pytest.mark.parametrize("sf,osr,hann", [(7, 1, False), (9, 1, True), (8, 2, False)])
def test_raw_mode_at_bandwidth(O, amd, sf, osr, hann, bw):
    """LORA_MODE_RAW (the detector alone, awgn_sweep.py:262-265) with the fused dechirp at bw."""
    rng = np.random.default_rng(sf * 5 + osr + bw // 1000)
    iq = frames_at(O, rng, sf, osr, bw, 6, 7)
    plan = amd.DemodPlan(sf, osr, bw, "hann" if hann else "none", dechirp=True, mode="raw")
    got = plan.run(torch.from_numpy(iq).cuda()).symbols.cpu().numpy()
    for f in range(iq.shape[0]):
        np.testing.assert_array_equal(got[f], O.raw_demod(iq[f], sf, osr, hann, dechirp=True, bw=bw))


@pytest.mark.parametrize("path", ["spec", "split"])
@pytest.mark.parametrize("bw", [125000, 250000, 500000])
@pytest.mark.parametrize("sf", [7, 9, 12])
def test_bandwidth_quirk_end_to_end_on_the_gpu(O, amd, sf, bw, path):
    """SURVEY.md 8(a11), reproduced on the GPU: lora_mod_batch(bw) -> the fused dechirp at bw
    -> lora_demod_batch gives (symbol * bw_scale) mod N for every noiseless symbol and the
    sync word of the shifted sync symbols - as the reference's own chain does
    (test_oracle_vs_reference::test_bandwidth_quirk_symbol_times_bw_scale) - and equals the
    oracle frame for frame."""
    rng = np.random.default_rng(sf + bw // 1000)
    N, F, S = 1 << sf, (64 if sf < 12 else 8), 12
    syms = rng.integers(0, N, (F, S)).astype(np.int32)
    iq = amd.modulate(torch.from_numpy(syms).cuda(), sf, 1, bw, 1.0, 0x12)
    plan = amd.DemodPlan(sf, 1, bw, dechirp=True, pipeline=path)
    res = plan.run(iq)
    got = res.symbols.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(got, (syms.astype(np.int64) * BWS[bw]) % N)
    sh = sf - 4
    sw0, sw1 = ((0x12 >> 4) << sh) * BWS[bw] % N, ((0x12 & 0xF) << sh) * BWS[bw] % N
    assert (res.sync.cpu().numpy() == ((((sw0 >> sh) & 0xF) << 4) | ((sw1 >> sh) & 0xF))).all()
    x = iq.cpu().numpy()
    for f in (0, F // 2, F - 1):
        os_, osync, ocfo, otoff = O.lora_demodulate(O.dechirp(x[f], sf, 1, bw), sf)
        np.testing.assert_array_equal(got[f], os_)
        assert bits(res.cfo[f].item()) == bits(ocfo) and bits(res.time_offset[f].item()) == bits(otoff)
