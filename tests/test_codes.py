"""CPU: host-side coding chain (lora_phy_amd.codes) bit-exact against the reference.

Goldens in tests/golden/golden.json["codes"] come from the reference's LoRaCodes.hpp
compiled in oracle/_ref (make_golden.py); plus the reference's own known-answer tests
roundtrip_test.cpp:30-31 and whitening_test.cpp:30-31.  When the reference build is
present the tables are also re-derived live.
"""
import base64
import json
import os

import numpy as np
import pytest

from lora_phy_amd import codes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")


@pytest.fixture(scope="module")
def C():
    with open(GOLD) as fh:
        return json.load(fh)["codes"]


def test_hamming_and_parity_tables(C):
    np.testing.assert_array_equal(codes.encode_hamming84(np.arange(16)), C["enc_h84"])
    n, e, b = codes.decode_hamming84(np.arange(256))
    np.testing.assert_array_equal(np.stack([n, e, b], 1).astype(int), C["dec_h84"])
    np.testing.assert_array_equal(codes.encode_hamming74(np.arange(16)), C["enc_h74"])
    n, e = codes.decode_hamming74(np.arange(128))
    np.testing.assert_array_equal(np.stack([n, e], 1).astype(int), C["dec_h74"])
    np.testing.assert_array_equal(codes.encode_parity54(np.arange(16)), C["enc_p54"])
    n, e = codes.check_parity54(np.arange(32))
    np.testing.assert_array_equal(np.stack([n, e], 1).astype(int), C["chk_p54"])
    np.testing.assert_array_equal(codes.encode_parity64(np.arange(16)), C["enc_p64"])
    n, e = codes.check_parity64(np.arange(64))
    np.testing.assert_array_equal(np.stack([n, e], 1).astype(int), C["chk_p64"])


def test_gray(C):
    g = np.array(C["gray_in"], np.uint16)
    np.testing.assert_array_equal(codes.gray_to_binary16(g), C["gray2bin"])
    np.testing.assert_array_equal(codes.binary_to_gray16(g), C["bin2gray"])
    np.testing.assert_array_equal(codes.gray_to_binary16(codes.binary_to_gray16(g)), g)


def test_checksums(C):
    blob = bytes.fromhex(C["blob"])
    assert [codes.checksum8(blob[:n]) for n in range(0, 40, 3)] == C["checksum8"]
    assert [codes.sx1272_data_checksum(blob[:n]) for n in range(0, 40, 3)] == C["sx1272_crc"]
    for h, want in C["header_checksum"]:
        assert codes.header_checksum(bytes.fromhex(h)) == want


def test_whitening(C):
    blob = bytes.fromhex(C["blob"])
    w = C["whiten"]
    assert codes.sx1232_whitening(blob).hex() == w["sx1232"]
    assert codes.sx1272_whitening(blob, 0, 4).hex() == w["sx1272_0_4"]
    assert codes.sx1272_whitening(blob, 1, 1).hex() == w["sx1272_1_1"]
    assert codes.sx1272_whitening_lfsr(blob, 0, 4).hex() == w["lfsr_0_4"]
    assert codes.sx1272_whitening_lfsr(blob, 2, 3).hex() == w["lfsr_2_3"]


def test_interleave(C):
    for key, rec in C["interleave"].items():
        ppm, rdd = map(int, key.split("_"))
        cw = np.frombuffer(bytes.fromhex(rec["codewords"]), np.uint8)
        syms = codes.diagonal_interleave(cw, ppm, rdd)
        np.testing.assert_array_equal(syms, rec["symbols"])
        assert codes.diagonal_deinterleave(syms, ppm, rdd).tobytes().hex() == rec["deinterleave"]
        if rec["deinterleave2"] is not None:  # None: the reference reads out of bounds
            assert codes.diagonal_deinterleave2(syms, ppm, rdd).tobytes().hex() == rec["deinterleave2"]


def test_reference_known_answers(C):
    """roundtrip_test.cpp:30-31 and whitening_test.cpp:30-31, verbatim vectors."""
    rt = C["roundtrip"]
    want = np.frombuffer(base64.b64decode(rt["expected_b64"]), "<u2")
    got = codes.lora_encode(bytes.fromhex(rt["payload"]))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, rt["symbols"])
    assert codes.lora_decode(got).tobytes().hex() == rt["payload"]
    wt = C["whitening"]
    plain = bytes.fromhex(wt["plain"])
    white = codes.sx1272_whitening_lfsr(plain, 0, 4)
    assert white.hex() == wt["whitened"]
    back = codes.sx1272_whitening_lfsr(white, 0, 4)
    assert back == plain
    crc = codes.sx1272_data_checksum(back[:-2])
    assert crc == back[-2] | (back[-1] << 8)


def test_decode_with_crc_and_batches():
    rng = np.random.default_rng(1)
    payload = rng.integers(0, 256, 10).astype(np.uint8).tobytes()
    crc = codes.sx1272_data_checksum(payload[2:])
    frame = payload + bytes([crc & 0xFF, crc >> 8])
    out, ok = codes.decode_with_crc(codes.lora_encode(frame))
    assert ok and out.tobytes() == frame
    batch = np.stack([codes.lora_encode(frame)] * 3)
    np.testing.assert_array_equal(codes.lora_decode(batch), np.stack([np.frombuffer(frame, np.uint8)] * 3))


def test_live_reference_if_present():
    from oracle.pyoracle import Reference

    if not Reference.available():
        pytest.skip("reference build absent")
    R = Reference()
    rng = np.random.default_rng(11)
    for _ in range(20):
        p = rng.integers(0, 256, int(rng.integers(0, 40))).astype(np.uint8).tobytes()
        np.testing.assert_array_equal(codes.lora_encode(p), R.lora_encode(p))
        s = rng.integers(0, 1 << 12, 2 * len(p)).astype(np.uint16)
        assert codes.lora_decode(s).tobytes() == R.lora_decode(s)
