"""GPU: the phy.hpp functional mirror (lora_phy_amd.phy) against the oracle / goldens."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def O():
    from oracle.pyoracle import Oracle

    return Oracle()


@pytest.fixture(scope="module")
def phy():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from lora_phy_amd import phy

    return phy


def bits(v):
    return np.float32(v).view(np.uint32)


def test_workspace_api_flow(O, phy):
    ws = phy.init(phy.lora_params(sf=8, osr=2, window="hann", sync_word=0x34))
    rng = np.random.default_rng(8)
    syms = rng.integers(0, 256, 9).astype(np.int32)
    iq = phy.modulate(ws, syms)
    ref_iq = O.lora_modulate(syms.astype(np.uint16), 8, 2, 125000, 1.0, 0x34)
    np.testing.assert_array_equal(iq.cpu().numpy().view(np.uint32), ref_iq.view(np.uint32))
    noisy = iq + torch.from_numpy((0.3 * (rng.standard_normal(iq.shape[0]) +
                                         1j * rng.standard_normal(iq.shape[0]))).astype(np.complex64)).cuda()
    out = phy.demodulate(ws, noisy)
    r, osym, osync, ocfo, otoff = O.api_demodulate(noisy.cpu().numpy(), 8, 2, True)
    assert r == len(out)
    np.testing.assert_array_equal(out.cpu().numpy(), osym)
    assert ws.sync_word == osync
    m = phy.get_last_metrics(ws)
    assert bits(m.cfo) == bits(ocfo) and bits(m.time_offset) == bits(otoff)
    with pytest.raises(phy.LoraError):
        phy.demodulate(ws, noisy[:-1])  # not a whole number of symbols (phy.cpp:183-186)
    phy.estimate_offsets(ws, noisy)
    ecfo, etoff = O.estimate_offsets(noisy.cpu().numpy(), 8, 2, True)
    assert bits(ws.metrics.cfo) == bits(ecfo) and bits(ws.metrics.time_offset) == bits(etoff)
    x = noisy.clone()
    phy.compensate_offsets(ws, x)
    ref = O.compensate_offsets(noisy.cpu().numpy(), 8, 2, ecfo, etoff)
    np.testing.assert_array_equal(x.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_legacy_api_interop_fixture(phy):
    rec = json.load(open(os.path.join(GOLD, "golden.json")))["interop"]
    x = torch.from_numpy(np.fromfile(os.path.join(GOLD, rec["file"]), dtype=np.complex64)).cuda()
    ws = phy.lora_demod_init(7)
    syms, sync = phy.lora_demodulate(ws, x, osr=2)
    assert syms.cpu().tolist() == rec["symbols"] and int(sync) == 0x29
    assert bits(ws.metrics.cfo) == rec["cfo_bits"] and bits(ws.metrics.time_offset) == rec["toff_bits"]
    assert phy.lora_decode(syms).hex() == rec["expected_payload"]
    phy.lora_demod_free(ws)


def test_legacy_api_batch_with_dechirp(O, phy):
    rng = np.random.default_rng(12)
    payloads = [rng.integers(0, 256, 16).astype(np.uint8).tobytes() for _ in range(6)]
    syms = np.stack([phy.lora_encode(p) for p in payloads]).astype(np.int32)
    iq = phy.lora_modulate(syms, 9)
    ws = phy.lora_demod_init(9, dechirp=True)
    out, sync = phy.lora_demodulate(ws, iq)
    for f, p in enumerate(payloads):
        assert phy.lora_decode(out[f]) == p
        o = O.lora_demodulate(O.dechirp(iq[f].cpu().numpy(), 9), 9)
        np.testing.assert_array_equal(out[f].cpu().numpy(), o[0])
        assert int(sync[f]) == o[1] == 0x12
