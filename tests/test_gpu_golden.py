"""GPU: the HIP path against the reference's own golden fixtures (tests/golden/).

Every expected value here was produced by the reference (make_golden.py over the
reference build); inputs are the reference's fixtures or seeded frames regenerated
with the pinned oracle modulator and checked by sha256 before use.
"""
import base64
import json
import os

import numpy as np
import pytest

from tests.golden_inputs import STRESS, f32bits, sha, stress_input

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def G():
    with open(os.path.join(GOLD, "golden.json")) as fh:
        return json.load(fh)


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


def check_frame(res, f, rec):
    n = len(rec["symbols"])
    assert res.symbols.shape[1] == n
    np.testing.assert_array_equal(res.symbols[f].cpu().numpy(), rec["symbols"])
    assert int(res.sync[f]) == rec["sync"]
    assert f32bits(res.cfo[f].item()) == rec["cfo_bits"]
    assert f32bits(res.time_offset[f].item()) == rec["toff_bits"]


def test_interop_fixture_gpu(G, amd):
    """gr_lora_sdr_interop.cpp: raw IQ, SF7 osr 2 -> sync 0x29, payload BE E7 82 75 E0."""
    rec = G["interop"]
    x = np.fromfile(os.path.join(GOLD, rec["file"]), dtype=np.complex64)
    assert sha(x) == rec["sha256"]
    demod = amd.LoRaDemod(7, sync=0x29, osr=2, dechirp=False)
    syms = demod.work(torch.from_numpy(x).cuda())
    check_frame(demod.last, 0, rec)
    assert bool(demod.sync_ok()[0])
    assert amd.codes.lora_decode(syms.cpu().numpy()).tobytes().hex() == rec["expected_payload"]


def test_e2e_chain_gpu(G, amd):
    """e2e_chain_test.cpp: encode -> GPU modulate -> fused dechirp + demod -> decode."""
    for rec in G["e2e"]:
        syms = amd.codes.lora_encode(bytes.fromhex(rec["payload"]))
        iq = amd.modulate(torch.from_numpy(syms.astype(np.int32)).cuda(), rec["sf"])
        assert sha(iq.cpu().numpy()) == rec["iq_sha256"]
        demod = amd.LoRaDemod(rec["sf"])
        out = demod.work(iq)
        check_frame(demod.last, 0, rec)
        assert amd.codes.lora_decode(out.cpu().numpy()).tobytes().hex() == rec["payload"]


def test_no_alloc_and_equal_power_gpu(G, amd):
    rec = G["no_alloc"]
    iq = amd.LoRaMod(7).work(rec["tx_symbols"])
    assert sha(iq.cpu().numpy()) == rec["iq_sha256"]
    demod = amd.LoRaDemod(7)
    demod.work(iq)
    check_frame(demod.last, 0, rec)
    rec = G["equal_power"]
    x = np.frombuffer(base64.b64decode(rec["iq_b64"]), np.complex64).copy()
    demod = amd.LoRaDemod(2, dechirp=False)
    assert demod.work(torch.from_numpy(x).cuda()).cpu().tolist() == [0]
    check_frame(demod.last, 0, rec)


def test_awgn_gtest_frames_gpu(G, O, amd):
    """awgn_sweep_gtest.cpp at 12 dB: 15 noisy packets, every one decodes, and the
    GPU matches the reference's symbols/metrics exactly."""
    frames = G["awgn_gtest"]["frames"]
    iq, _ = O.awgn_gtest_frames([(7, 125000), (7, 125000), (8, 125000)])
    for sf in (7, 8):
        recs = [r for r in frames if r["sf"] == sf]
        L = (2 * 16 + 2) << sf
        start = sum(((2 * 16 + 2) << r["sf"]) for r in frames[: frames.index(recs[0])])
        x = iq[start:start + L * len(recs)].reshape(len(recs), L)
        for k, r in enumerate(recs):
            assert sha(x[k]) == r["iq_sha256"]
        res = amd.DemodPlan(sf, dechirp=True).run(torch.from_numpy(x).cuda())
        for k, r in enumerate(recs):
            check_frame(res, k, r)
            dec = amd.codes.lora_decode(res.symbols[k].cpu().numpy()).tobytes().hex()
            assert dec == r["decoded"] == r["payload"]


@pytest.mark.parametrize("ci", range(len(STRESS)))
def test_stress_cases_gpu(G, O, amd, ci):
    case = STRESS[ci]
    rec = G["stress"][ci]
    sf, osr, hann, dech, F = case[:5]
    x = stress_input(O, case, rec["seed"])
    assert sha(x) == rec["iq_sha256"], "input generator drifted; regenerate the goldens"
    plan = amd.DemodPlan(sf, osr, 125000, "hann" if hann else "none", dechirp=dech)
    res = plan.run(torch.from_numpy(x).cuda())
    for f, fr in enumerate(rec["frames"]):
        check_frame(res, f, fr)


def test_api_cases_gpu(G, O, amd):
    for rec in G["api"]:
        sf, osr, hann = rec["sf"], rec["osr"], rec["hann"]
        rng = np.random.default_rng(rec["seed"])
        syms = rng.integers(0, 1 << sf, rec["nsym"]).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, 0x34)
        x = (x + 0.25 * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x)))).astype(np.complex64)
        assert sha(x) == rec["iq_sha256"]
        plan = amd.DemodPlan(sf, osr, 125000, "hann" if hann else "none", mode="api")
        res = plan.run(torch.from_numpy(x).cuda())
        assert res.symbols.shape[1] == rec["ret"]
        check_frame(res, 0, rec)
        cfo = torch.zeros(1, device="cuda")
        toff = torch.zeros(1, device="cuda")
        plan.estimate_offsets(torch.from_numpy(x).cuda(), cfo, toff)
        assert f32bits(cfo.item()) == rec["est_cfo_bits"]
        assert f32bits(toff.item()) == rec["est_toff_bits"]


def test_capture_excerpt_gpu(G, amd):
    """Real capture from the reference (vectors_binary, SF7): one long frame, GPU vs the
    reference's lora_demodulate for osr 1/2/4, raw and fused dechirp, both windows."""
    cap = G["capture"]
    x = np.fromfile(os.path.join(GOLD, cap["file"]), dtype=np.complex64)
    assert sha(x) == cap["sha256"]
    xt = torch.from_numpy(x).cuda()
    for rec in cap["cases"]:
        plan = amd.DemodPlan(7, rec["osr"], 125000, "hann" if rec["hann"] else "none",
                             dechirp=rec["dechirp"])
        check_frame(plan.run(xt), 0, rec)


def test_capture_file_streamed_to_gpu(G, amd):
    """iq_io streams the reference's capture excerpt into HBM; GPU demod equals the
    reference's output for the raw osr-1 case."""
    from lora_phy_amd import iq_io

    cap = G["capture"]
    x = iq_io.read_iq(os.path.join(GOLD, cap["file"]), device="cuda", slice_samples=4096)
    rec = [r for r in cap["cases"] if r["osr"] == 1 and not r["dechirp"] and not r["hann"]][0]
    check_frame(amd.DemodPlan(7).run(x), 0, rec)
