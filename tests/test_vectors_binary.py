"""CPU: the host coding chain (lora_phy_amd.codes) on the reference's vectors_binary/*.bin.

north_star: Gray demap, diagonal deinterleave, Hamming and whitening "checked bit-exact
against vectors_binary/ and the C++/Python reference".  The .bin files carry inputs only
(scripts/create_binary_vectors.py:33-69); tests/golden/make_vectors_binary.py parsed every
record and ran it through the reference's own LoRaCodes.hpp / lora_encode / lora_decode
(compiled in oracle/_ref), storing inputs and reference outputs in
tests/golden/vectors_binary.json.  Here codes.py must reproduce every stage bit for bit.
When /root/reference is present the fixture's inputs are re-parsed from the .bin files.
"""
import json
import os

import numpy as np
import pytest

from lora_phy_amd import codes

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "vectors_binary.json")
VEC_DIR = "/root/reference/vectors_binary"


@pytest.fixture(scope="module")
def V():
    with open(GOLD) as fh:
        return json.load(fh)["files"]


def payload_records(V):
    return [(fn, r) for fn, f in V.items() for r in f["checked"] if "chain" in r]


def test_every_file_accounted_for(V):
    """Each .bin is listed with its record count; records without data are named."""
    assert len(V) == 10
    total = sum(f["records"] for f in V.values())
    checked = sum(len(f["checked"]) for f in V.values())
    no_data = sum(sum(f["no_data"].values()) for f in V.values())
    assert total == checked + no_data == 939
    assert checked == 314  # 284 payload records + 30 interleaver codeword records
    for fn in ("encoder_decoder_tests.bin", "loopback_tests.bin", "modulation_tests.bin",
               "validation_tests.bin", "interleaver_test_vectors.bin"):
        assert len(V[fn]["checked"]) == V[fn]["records"], fn


def test_library_encode_decode(V):
    """lora_encode / lora_decode (LoRaEncoder.cpp:8-19, LoRaDecoder.cpp:8-19)."""
    for fn, r in payload_records(V):
        p = bytes.fromhex(r["payload"])
        sym = codes.lora_encode(p)
        np.testing.assert_array_equal(sym, r["lib_symbols"], err_msg=f"{fn}[{r['index']}]")
        assert codes.lora_decode(sym).tobytes().hex() == r["lib_decoded"] == r["payload"]


def test_tx_chain_stages(V):
    """nibble code -> whitening -> diagonal interleave (PPM = SF) -> Gray, per record SF / CR."""
    seen = set()
    for fn, r in payload_records(V):
        rdd = codes.rdd_of(r["cr"])
        assert rdd == r["rdd"]
        seen.add((r["sf"], rdd))
        e = codes.encode_chain(bytes.fromhex(r["payload"]), r["sf"], rdd)
        c = r["chain"]
        where = f"{fn}[{r['index']}] sf{r['sf']} rdd{rdd}"
        assert e["codewords"].tobytes().hex() == c["codewords"], where
        assert e["whitened"].tobytes().hex() == c["whitened"], where
        np.testing.assert_array_equal(e["interleaved"], c["interleaved"], err_msg=where)
        np.testing.assert_array_equal(e["symbols"], c["symbols"], err_msg=where)
    assert {rdd for _, rdd in seen} == {0, 1, 2, 3, 4}
    assert {sf for sf, _ in seen} >= {7, 8, 9, 10, 11, 12}


def test_rx_chain_stages(V):
    """Gray demap -> diagonal deinterleave -> de-whitening -> nibble decode -> payload."""
    for fn, r in payload_records(V):
        rdd = r["rdd"]
        c = r["chain"]
        n = len(bytes.fromhex(r["payload"]))
        d = codes.decode_chain(np.array(c["symbols"], np.uint16), r["sf"], rdd, n)
        where = f"{fn}[{r['index']}]"
        np.testing.assert_array_equal(d["binary"], c["binary"], err_msg=where)
        assert d["deinterleaved"].tobytes().hex() == c["deinterleaved"], where
        assert d["dewhitened"].tobytes().hex() == c["dewhitened"], where
        nib, err = codes.nibble_decode(d["dewhitened"], rdd)
        np.testing.assert_array_equal(nib, c["nibbles"], err_msg=where)
        np.testing.assert_array_equal(err.astype(int), c["errors"], err_msg=where)
        assert d["payload"].tobytes().hex() == c["decoded"] == r["payload"], where


def test_decoders_on_flipped_bits(V):
    """One flipped bit per codeword: corrected / flagged exactly as the reference decoders."""
    for fn, r in payload_records(V):
        c = r["chain"]
        nib, err = codes.nibble_decode(np.frombuffer(bytes.fromhex(c["flipped"]), np.uint8), r["rdd"])
        np.testing.assert_array_equal(nib, c["flipped_nibbles"], err_msg=f"{fn}[{r['index']}]")
        np.testing.assert_array_equal(err.astype(int), c["flipped_errors"], err_msg=f"{fn}[{r['index']}]")


def test_interleaver_records(V):
    """interleaver_test_vectors.bin: the stored codewords, PPM = their count."""
    recs = V["interleaver_test_vectors.bin"]["checked"]
    assert len(recs) == 30
    for r in recs:
        cw = np.frombuffer(bytes.fromhex(r["input_codewords"]), np.uint8)
        rdd = codes.rdd_of(r["cr"])
        il = codes.diagonal_interleave(cw, len(cw), rdd)
        np.testing.assert_array_equal(il, r["interleaved"])
        np.testing.assert_array_equal(codes.binary_to_gray16(il), r["symbols"])
        assert codes.diagonal_deinterleave(il, len(cw), rdd).tobytes().hex() == r["deinterleaved"]


@pytest.mark.skipif(not os.path.isdir(VEC_DIR), reason="reference checkout not present")
def test_fixture_inputs_match_the_bin_files(V):
    import importlib.util

    spec = importlib.util.spec_from_file_location("mkvb", os.path.join(HERE, "golden", "make_vectors_binary.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    for fn, f in V.items():
        recs = mk.parse_bin(os.path.join(VEC_DIR, fn))
        assert len(recs) == f["records"]
        for r in f["checked"]:
            src = recs[r["index"]]
            assert src["payload"].hex() == r["payload"] and src["codewords"].hex() == r["input_codewords"]
            assert src["sf"] == r["sf"] and src["cr"] == r["cr"] and src["test_type"] == r["test_type"]
