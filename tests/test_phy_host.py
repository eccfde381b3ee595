"""CPU: host-side parts of the phy.hpp mirror (lora_phy_amd.phy) - argument checking
and the encode/decode/CRC chain (phy.cpp:55-63, 241-256).  No GPU needed."""
import numpy as np
import pytest

from lora_phy_amd import LoraError, codes, phy


def test_init_rejects_invalid_params():
    for bad in (phy.lora_params(sf=1), phy.lora_params(sf=13), phy.lora_params(bw=100000),
                phy.lora_params(window="kaiser")):
        with pytest.raises(LoraError):
            phy.init(bad)
    with pytest.raises(LoraError):
        phy.init(None)
    with pytest.raises(LoraError):
        phy.lora_demod_init(13)


def test_encode_decode_crc():
    ws = phy.lora_workspace(sf=7)
    payload = bytes(range(10))
    crc = codes.sx1272_data_checksum(payload[2:])
    frame = payload + bytes([crc & 0xFF, crc >> 8])
    syms = phy.encode(ws, frame)
    assert len(syms) == 2 * len(frame)
    with pytest.raises(LoraError):
        phy.encode(ws, frame, symbol_cap=3)
    assert phy.decode(ws, syms) == frame
    assert phy.get_last_metrics(ws).crc_ok is True
    bad = syms.copy()
    bad[5] ^= 0x0F  # two-nibble error: Hamming 8/4 cannot fix it -> CRC fails
    phy.decode(ws, bad)
    assert phy.get_last_metrics(ws).crc_ok is False
    phy.reset(ws)
    assert phy.get_last_metrics(ws).crc_ok is False and phy.get_last_metrics(ws).cfo == 0.0


def test_legacy_encode_decode():
    p = bytes([0xDE, 0xAD, 0xBE, 0xEF])
    np.testing.assert_array_equal(phy.lora_encode(p), [141, 46, 154, 141, 75, 46, 46, 255])
    assert phy.lora_decode(phy.lora_encode(p)) == p
    assert phy.bw_scale(250000) == 2.0
