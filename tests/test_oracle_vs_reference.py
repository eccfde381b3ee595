"""CPU: the restatement (oracle/lora_oracle.cpp) against the reference build itself.

oracle/_ref/liblora_ref.so is the reference's src/phy/*.cpp compiled by oracle/Makefile
from /root/reference; it exists only in the build container, so this module skips
elsewhere (tests/test_golden_oracle.py pins the oracle to committed fixtures there).
Randomised: every SF, osr 1..4, both windows, any amplitude (normalisation on/off),
odd lengths - bit-exact on every output.
"""
import numpy as np
import pytest

from oracle.pyoracle import Oracle, Reference

pytestmark = pytest.mark.skipif(not Reference.available(), reason="reference build absent")


@pytest.fixture(scope="module")
def O():
    return Oracle()


@pytest.fixture(scope="module")
def R():
    return Reference()


def u32(x):
    return np.asarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("sf", range(2, 13))
def test_fft_and_chirps(O, R, sf):
    N = 1 << sf
    rng = np.random.default_rng(sf)
    x = (rng.standard_normal(N) + 1j * rng.standard_normal(N)).astype(np.complex64)
    np.testing.assert_array_equal(O.fft(x).view(np.uint32), R.fft(x).view(np.uint32))
    for osr in (1, 2, 3):
        for down in (False, True):
            for bws in (1.0, 2.0, 4.0):
                a, pa = O.gen_chirp(N, osr, N * osr, 0.3, down, 0.7, 1.25, bws)
                b, pb = R.gen_chirp(N, osr, N * osr, 0.3, down, 0.7, 1.25, bws)
                np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
                assert u32(pa) == u32(pb)


@pytest.mark.parametrize("sf", range(2, 13))
def test_modulate(O, R, sf):
    rng = np.random.default_rng(100 + sf)
    for osr, bw in ((1, 125000), (2, 250000), (3, 500000)):
        syms = rng.integers(0, 1 << sf, 7).astype(np.uint16)
        a = O.lora_modulate(syms, sf, osr, bw, 0.8, 0x5A)
        b = R.lora_modulate(syms, sf, osr, bw, 0.8, 0x5A)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def _frames(rng, sf, osr, n):
    N = 1 << sf
    for _ in range(n):
        L = int(rng.integers(0, 12)) * N * osr + int(rng.integers(0, 3 * N))
        amp = float(rng.choice([0.01, 0.5, 1.0, 2.5, 40.0]))
        x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)) * amp
        if rng.random() < 0.6 and L >= N * osr:  # a real chirp train underneath
            k = L // (N * osr)
            syms = rng.integers(0, N, max(k - 2, 0)).astype(np.uint16)
            s = R_mod_cache(sf, osr, syms)
            x = x * 0.2 + np.concatenate([s, np.zeros(max(L - len(s), 0))])[:L]
        yield x.astype(np.complex64)


_REF = {}


def R_mod_cache(sf, osr, syms):
    r = _REF.setdefault("R", Reference())
    return r.lora_modulate(syms, sf, osr, 125000, 1.0, 0x12)


@pytest.mark.parametrize("sf", range(2, 13))
@pytest.mark.parametrize("osr", [1, 2, 4])
def test_lora_demodulate(O, R, sf, osr):
    rng = np.random.default_rng(sf * 31 + osr)
    for x in _frames(rng, sf, osr, 6 if sf < 11 else 3):
        for hann in (False, True):
            for dech in (False, True):
                xi = O.dechirp(x, sf, osr) if dech else x
                a = O.lora_demodulate(xi, sf, osr, hann)
                b = R.lora_demodulate(xi, sf, osr, hann)
                np.testing.assert_array_equal(a[0], b[0])
                assert a[1] == b[1]
                assert u32(a[2]) == u32(b[2]) and u32(a[3]) == u32(b[3])


@pytest.mark.parametrize("sf", [2, 5, 7, 8, 10, 12])
@pytest.mark.parametrize("osr", [1, 3])
def test_api_demodulate_estimate_compensate(O, R, sf, osr):
    rng = np.random.default_rng(sf * 7 + osr)
    N = 1 << sf
    for k in (1, 2, 3, 6):
        x = (rng.standard_normal(k * N * osr) + 1j * rng.standard_normal(k * N * osr)).astype(np.complex64)
        for hann in (False, True):
            ra = O.api_demodulate(x, sf, osr, hann)
            rb = R.api_demodulate(x, sf, osr, hann)
            assert ra[0] == rb[0]
            np.testing.assert_array_equal(ra[1], rb[1])
            if ra[0] >= 0:  # outputs other than the return code are only defined on success
                assert ra[2] == rb[2] and u32(ra[3]) == u32(rb[3]) and u32(ra[4]) == u32(rb[4])
            ea = O.estimate_offsets(x, sf, osr, hann)
            eb = R.estimate_offsets(x, sf, osr, hann)
            assert u32(ea[0]) == u32(eb[0]) and u32(ea[1]) == u32(eb[1])
        for cfo, to in ((0.3, 2.4), (-1.7, -5.5), (0.0, 0.0), (12.5, 1e6)):
            a = O.compensate_offsets(x, sf, osr, cfo, to)
            b = R.compensate_offsets(x, sf, osr, cfo, to)
            np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_encode_decode(O, R):
    rng = np.random.default_rng(3)
    for n in (0, 1, 5, 16, 33):
        p = rng.integers(0, 256, n).astype(np.uint8).tobytes()
        a = O.lora_encode(p)
        b = R.lora_encode(p)
        np.testing.assert_array_equal(a, b)
        assert O.lora_decode(a) == R.lora_decode(b) == p


@pytest.mark.parametrize("sf,osr,hann", [(7, 1, False), (9, 2, True), (12, 1, False)])
def test_batched_frames_bench_leg(O, R, sf, osr, hann):
    """ref_demod_frames (the reference itself, multi-threaded: bench.py cpu_baseline)
    equals the restatement's orc_demod_frames on the same batch."""
    rng = np.random.default_rng(sf)
    L = 6 * (1 << sf) * osr + 3
    x = (rng.standard_normal((9, L)) + 1j * rng.standard_normal((9, L))).astype(np.complex64)
    for dech in (False, True):
        a = O.demod_frames(x, sf, osr, hann, dechirp=dech, threads=3)
        b = R.demod_frames(x, sf, osr, hann, dechirp=dech, threads=2)
        for u, v in zip(a, b):
            np.testing.assert_array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
