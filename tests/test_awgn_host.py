"""CPU: host pieces of the AWGN sweep (lora_phy_amd.awgn) equal the reference script's.

tests/golden/awgn_sweep.json["pieces"] was recorded from the reference's own
tests/awgn_sweep.py (make_golden.py): payload -> bits for CR 4/5 and 4/8, bit <->
symbol packing at SF7/9/12, the Hamming 8/4 decoder over all 256 codewords, and the
float64 chirp of the Python model.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from lora_phy_amd import awgn, codes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "awgn_sweep.json")


@pytest.fixture(scope="module")
def P():
    return json.load(open(GOLD))["pieces"]


@pytest.mark.parametrize("cr", ["4/5", "4/8"])
def test_payload_bits_and_packing(P, cr):
    pay = bytes.fromhex(P["payload"])
    bits = awgn.encode_payload(pay, cr)
    np.testing.assert_array_equal(bits, P["bits_" + cr])
    for sf in (7, 9, 12):
        syms = awgn.bits_to_symbols(bits, sf)
        np.testing.assert_array_equal(syms, P[f"syms_{cr}_sf{sf}"])
        np.testing.assert_array_equal(awgn.symbols_to_bits(syms, sf, len(bits)), bits)
    np.testing.assert_array_equal(awgn.decode_payload(bits, cr, len(pay)), P["decoded_" + cr])


def test_hamming_decoder_matches_script(P):
    n, e, b = codes.decode_hamming84(np.arange(256))
    got = [[int(x), bool(y), bool(z)] for x, y, z in zip(n, e, b)]
    want = [[x, bool(y), bool(z)] for x, y, z in P["dec_h84"]]
    assert got == want


def test_python_model_chirp(P):
    up, down = awgn.make_chirps(7)
    assert hashlib.sha256(np.ascontiguousarray(up).tobytes()).hexdigest() == P["up7_sha"]
    np.testing.assert_array_equal(down, np.conj(up))


def test_decode_corrects_single_bit_errors():
    rng = np.random.default_rng(3)
    pay = rng.integers(0, 256, 8).astype(np.uint8).tobytes()
    bits = awgn.encode_payload(pay, "4/8")
    for k in range(0, len(bits), 8):  # one flipped bit per codeword
        bits[k + int(rng.integers(0, 8))] ^= 1
    assert awgn.decode_payload(bits, "4/8", len(pay)).tobytes() == pay
