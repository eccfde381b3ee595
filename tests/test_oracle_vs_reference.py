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


# ---- bandwidth (phy.hpp:37-49 bw_scale): BW 250 / 500 kHz on every demod entry ----------------

def _ref_dechirp(R, x, sf, osr, bw):
    """The reference callers' dechirp (e2e_chain_test.cpp:84-93, performance_test.cpp:94-116,
    awgn_sweep_gtest.cpp:85-92): genChirp(down, N, 1, N, 0, true, 1, phase, bw_scale(bw)) from
    the reference build itself, then x[s*N + i] * down[i] as std::complex<float>'s product
    (ac - bd, ad + bc: each product rounded to fp32, then the sum - no FMA on x86-64).  The
    reference callers dechirp at osr 1; at osr > 1 the N*osr-sample down-chirp of the same
    genChirp call with osr (the generalisation lora_demod_params.dechirp defines)."""
    N = 1 << sf
    down, _ = R.gen_chirp(N, osr, N * osr, 0.0, True, 1.0, 0.0, {125000: 1.0, 250000: 2.0, 500000: 4.0}[bw])
    d = np.resize(down, len(x))  # down[j mod N*osr]
    a, b = x.real.astype(np.float32), x.imag.astype(np.float32)
    c, e = d.real.astype(np.float32), d.imag.astype(np.float32)
    re = (a * c).astype(np.float32) - (b * e).astype(np.float32)
    im = (a * e).astype(np.float32) + (b * c).astype(np.float32)
    y = np.empty(len(x), np.complex64)
    y.real, y.imag = re, im  # (re + 1j * im would turn a -0.0 real part into +0.0)
    return y


@pytest.mark.parametrize("bw", [250000, 500000])
@pytest.mark.parametrize("sf,osr", [(7, 1), (9, 1), (9, 2), (12, 1), (5, 3)])
def test_bandwidth_dechirp_and_lora_demodulate(O, R, sf, osr, bw):
    """The oracle's dechirp at bw 250 / 500 kHz equals the reference callers' (bit for bit),
    and lora_demodulate on it equals the reference's: symbols, sync, cfo / time_offset bits -
    on frames modulated at the same bandwidth (the reference's own lora_modulate), with noise
    and sample delays."""
    rng = np.random.default_rng(sf * 11 + osr + bw // 1000)
    N = 1 << sf
    for k in range(4 if sf < 11 else 2):
        syms = rng.integers(0, N, 8).astype(np.uint16)
        x = R.lora_modulate(syms, sf, osr, bw, 1.0, int(rng.integers(0, 256)))
        delay = int(rng.integers(0, N * osr // 3))
        x = np.concatenate([np.zeros(delay, np.complex64), x])[:len(x)]
        x = (x + [0.0, 0.1, 0.5, 1.5][k] * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x))))
        x = x.astype(np.complex64)
        yo = O.dechirp(x, sf, osr, bw)
        yr = _ref_dechirp(R, x, sf, osr, bw)
        np.testing.assert_array_equal(yo.view(np.uint32), yr.view(np.uint32))
        for hann in (False, True):
            a = O.lora_demodulate(yo, sf, osr, hann)
            b = R.lora_demodulate(yr, sf, osr, hann)
            np.testing.assert_array_equal(a[0], b[0])
            assert a[1] == b[1]
            assert u32(a[2]) == u32(b[2]) and u32(a[3]) == u32(b[3])
        rb = O.raw_demod(x, sf, osr, False, dechirp=True, bw=bw)
        assert len(rb) == len(x) // (N * osr)


@pytest.mark.parametrize("bw", [250000, 500000])
@pytest.mark.parametrize("sf,osr", [(7, 1), (9, 1), (9, 2), (12, 1), (6, 3)])
def test_bandwidth_api_demodulate(O, R, sf, osr, bw):
    """lora_phy::demodulate at bw 250 / 500 kHz: its per-symbol down-chirp is generated with
    bw_scale (phy.cpp:202-204, reached by rx_runner --bw, runners/rx_runner.cpp:37-44) - the
    oracle's api_demodulate equals the reference's on every output, noiseless and noisy,
    both windows."""
    rng = np.random.default_rng(sf * 13 + osr + bw // 1000)
    N = 1 << sf
    for k in range(3):
        syms = rng.integers(0, N, 6).astype(np.uint16)
        x = R.lora_modulate(syms, sf, osr, bw, 1.0, 0x34)
        x = (x + [0.0, 0.3, 1.0][k] * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x))))
        x = x.astype(np.complex64)
        for hann in (False, True):
            ra = O.api_demodulate(x, sf, osr, hann, bw=bw)
            rb = R.api_demodulate(x, sf, osr, hann, bw=bw)
            assert ra[0] == rb[0] == 6
            np.testing.assert_array_equal(ra[1], rb[1])
            assert ra[2] == rb[2] and u32(ra[3]) == u32(rb[3]) and u32(ra[4]) == u32(rb[4])


@pytest.mark.parametrize("bw,bws", [(250000, 2), (500000, 4)])
@pytest.mark.parametrize("sf", [7, 8, 9, 10, 12])
def test_bandwidth_quirk_symbol_times_bw_scale(R, sf, bw, bws):
    """the reference's own chain at bw != 125 kHz, osr 1 -
    lora_modulate(bw) -> the caller's dechirp with bw_scale(bw) -> lora_demodulate - yields
    (symbol * bw_scale) mod N for every noiseless symbol (the modulator's frequency step is
    2*pi*sym*bw_scale/N while the demod's bins are 2*pi*k/N); and the sync word likewise."""
    rng = np.random.default_rng(sf + bw)
    N = 1 << sf
    syms = rng.integers(0, N, 16).astype(np.uint16)
    x = R.lora_modulate(syms, sf, 1, bw, 1.0, 0x12)
    got, sync, _, _ = R.lora_demodulate(_ref_dechirp(R, x, sf, 1, bw), sf, 1, False)
    np.testing.assert_array_equal(got, (syms.astype(np.int64) * bws) % N)
    sh = sf - 4
    sw0, sw1 = ((0x12 >> 4) << sh) * bws % N, ((0x12 & 0xF) << sh) * bws % N
    assert sync == (((sw0 >> sh) & 0xF) << 4) | ((sw1 >> sh) & 0xF)
