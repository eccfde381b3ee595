"""CPU: the oracle (oracle/lora_oracle.cpp) against the reference's golden fixtures.

tests/golden/golden.json was produced by the reference itself (tests/golden/
make_golden.py over oracle/_ref, the reference's src/phy compiled from
/root/reference).  These tests pin the restatement to it without needing the
reference at run time, so the oracle that checks the GPU path is itself checked.
"""
import base64
import json
import os

import numpy as np
import pytest

from tests.golden_inputs import STRESS, dechirp, f32bits, sha, stress_input

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def G():
    with open(os.path.join(GOLD, "golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def O():
    from oracle.pyoracle import Oracle

    return Oracle()


def check(rec, out):
    syms, sync, cfo, toff = out
    assert [int(s) for s in syms] == rec["symbols"]
    assert int(sync) == rec["sync"]
    assert f32bits(cfo) == rec["cfo_bits"]
    assert f32bits(toff) == rec["toff_bits"]


def test_interop_fixture(G, O):
    """gr_lora_sdr_interop.cpp:21-53 - sync 0x29 and payload BE E7 82 75 E0."""
    rec = G["interop"]
    x = np.fromfile(os.path.join(GOLD, rec["file"]), dtype=np.complex64)
    assert sha(x) == rec["sha256"]
    out = O.lora_demodulate(x, rec["sf"], rec["osr"], False)
    check(rec, out)
    assert out[1] == rec["expected_sync"] == 0x29
    assert O.lora_decode(out[0]).hex() == rec["expected_payload"]


def test_e2e_chain(G, O):
    """e2e_chain_test.cpp:62-113 - modulate, dechirp, demodulate, decode."""
    for rec in G["e2e"]:
        syms = O.lora_encode(bytes.fromhex(rec["payload"]))
        assert [int(s) for s in syms] == rec["tx_symbols"]
        iq = O.lora_modulate(syms, rec["sf"], 1, rec["bw"], 1.0, 0x12)
        assert sha(iq) == rec["iq_sha256"]
        d = O.dechirp(iq, rec["sf"])
        assert sha(d) == rec["dechirped_sha256"]
        out = O.lora_demodulate(d, rec["sf"])
        check(rec, out)
        assert O.lora_decode(out[0]).hex() == rec["decoded"] == rec["payload"]


def test_no_alloc_symbols(G, O):
    rec = G["no_alloc"]
    iq = O.lora_modulate(np.array(rec["tx_symbols"], np.uint16), 7)
    assert sha(iq) == rec["iq_sha256"]
    out = O.lora_demodulate(O.dechirp(iq, 7), 7)
    check(rec, out)
    assert rec["symbols"] == [0, 1, 12, 34, 56]


def test_equal_power_lowest_index(G, O):
    rec = G["equal_power"]
    x = np.frombuffer(base64.b64decode(rec["iq_b64"]), np.complex64).copy()
    out = O.lora_demodulate(x, 2)
    check(rec, out)
    assert rec["symbols"] == [0]


def test_awgn_gtest_frames(G, O):
    """awgn_sweep_gtest.cpp:52-108 at 12 dB: every packet decodes."""
    frames = G["awgn_gtest"]["frames"]
    iq, pay = O.awgn_gtest_frames([(7, 125000), (7, 125000), (8, 125000)])
    off = 0
    for k, rec in enumerate(frames):
        L = (2 * 16 + 2) << rec["sf"]
        x = iq[off:off + L]
        off += L
        assert sha(x) == rec["iq_sha256"]
        assert pay[k * 16:(k + 1) * 16].tobytes().hex() == rec["payload"]
        out = O.lora_demodulate(O.dechirp(x, rec["sf"]), rec["sf"])
        check(rec, out)
        assert O.lora_decode(out[0]).hex() == rec["decoded"] == rec["payload"]


@pytest.mark.parametrize("ci", range(len(STRESS)))
def test_stress_cases(G, O, ci):
    case = STRESS[ci]
    rec = G["stress"][ci]
    assert list(case) == rec["case"]
    sf, osr, hann, dech = case[:4]
    x = stress_input(O, case, rec["seed"])
    assert sha(x) == rec["iq_sha256"], "input generator drifted; regenerate the goldens"
    for f, fr in enumerate(rec["frames"]):
        xf = dechirp(O, x[f], sf, osr) if dech else x[f]
        # the oracle's own dechirp must agree with the fixture's fp32 product
        if dech:
            np.testing.assert_array_equal(O.dechirp(x[f], sf, osr).view(np.uint32), xf.view(np.uint32))
        check(fr, O.lora_demodulate(xf, sf, osr, hann))


def test_api_cases(G, O):
    for rec in G["api"]:
        sf, osr, hann = rec["sf"], rec["osr"], rec["hann"]
        rng = np.random.default_rng(rec["seed"])
        nsym = rec["nsym"]
        syms = rng.integers(0, 1 << sf, nsym).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, 0x34)
        x = (x + 0.25 * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x)))).astype(np.complex64)
        assert sha(x) == rec["iq_sha256"]
        r, osym, osync, ocfo, otoff = O.api_demodulate(x, sf, osr, hann)
        assert r == rec["ret"]
        assert [int(s) for s in osym] == rec["symbols"]
        assert osync == rec["sync"]
        assert f32bits(ocfo) == rec["cfo_bits"] and f32bits(otoff) == rec["toff_bits"]
        ecfo, etoff = O.estimate_offsets(x, sf, osr, hann)
        assert f32bits(ecfo) == rec["est_cfo_bits"] and f32bits(etoff) == rec["est_toff_bits"]


def test_capture_excerpt(G, O):
    """The reference's real SF7 capture (excerpt), every osr / dechirp / window case."""
    cap = G["capture"]
    x = np.fromfile(os.path.join(GOLD, cap["file"]), dtype=np.complex64)
    assert sha(x) == cap["sha256"]
    for rec in cap["cases"]:
        xi = dechirp(O, x, 7, rec["osr"]) if rec["dechirp"] else x
        check(rec, O.lora_demodulate(xi, 7, rec["osr"], rec["hann"]))
