"""CPU: BASELINE.json configs[0] - SF7 BW125 CR 4/5 single-frame loopback on the CPU path
(plumbing, no GPU): payload -> host encode (lora_phy_amd.codes; the library path applies
Hamming 8/4 per nibble whatever the CR, LoRaEncoder.cpp:8-19) -> lora_modulate -> caller
dechirp -> lora_demodulate -> host decode, through the restatement and, where it is built
here, through the reference itself (oracle/_ref), which must agree bit for bit.
Hamming 8/4 codewords reach 255 but an SF7 symbol holds 7 bits: the demodulator returns
the codeword mod 128 and the decoder corrects that top-bit error, as in the reference's
e2e_chain_test.cpp:62-113."""
import numpy as np
import pytest

from lora_phy_amd import phy
from oracle.pyoracle import Oracle, Reference


def loopback(impl, payload, sync=0x12):
    syms = phy.lora_encode(payload)
    iq = impl.lora_modulate(syms, 7, 1, 125000, 1.0, sync)
    x = Oracle().dechirp(iq, 7, 1)  # e2e_chain_test.cpp:85-93
    out, osync, cfo, toff = impl.lora_demodulate(x, 7, 1, False)
    return syms, iq, out, osync, cfo, toff


@pytest.mark.parametrize("n", [1, 5, 32, 64])
def test_sf7_cr45_single_frame_loopback(n):
    payload = bytes(np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8))
    syms, iq, out, osync, cfo, toff = loopback(Oracle(), payload)
    np.testing.assert_array_equal(out[:len(syms)], syms % 128)
    assert osync == 0x12
    assert phy.lora_decode(out[:len(syms)]) == payload
    if Reference.available():
        r_syms, r_iq, r_out, r_sync, r_cfo, r_toff = loopback(Reference(), payload)
        np.testing.assert_array_equal(r_iq.view(np.uint32), iq.view(np.uint32))
        np.testing.assert_array_equal(r_out, out)
        assert (r_sync, np.float32(r_cfo).view(np.uint32), np.float32(r_toff).view(np.uint32)) == \
            (osync, np.float32(cfo).view(np.uint32), np.float32(toff).view(np.uint32))
