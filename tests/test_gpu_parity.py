"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle, bit for bit.

The oracle (oracle/lora_oracle.cpp) is pinned to the reference itself by
tests/test_oracle_vs_reference.py and tests/golden/.  Here every output of
lora_demod_batch / lora_mod_batch / lora_estimate_offsets_batch /
lora_compensate_offsets_batch must equal the oracle's exactly: symbol indices and
sync words (integers) and cfo / time_offset (compared as fp32 bit patterns), at every
SNR, SF 2..12, osr 1..4, both windows, odd frame lengths and empty frames.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


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


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def make_frames(O, rng, sf, osr, F, L, kind, dechirp):
    N = 1 << sf
    out = np.zeros((F, L), np.complex64)
    for f in range(F):
        if kind == "noise":
            amp = np.float32(rng.uniform(0.05, 3.0))
            x = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(np.complex64) * amp
        else:
            nsym = L // (N * osr) + 1
            syms = rng.integers(0, N, max(nsym - 2, 0)).astype(np.uint16)
            x = O.lora_modulate(syms, sf, osr, 125000, 1.0, int(rng.integers(0, 256)))
            if not dechirp:
                x = O.dechirp(x, sf, osr)
            x = np.concatenate([x, np.zeros(max(L - len(x), 0), np.complex64)])[:L]
            sig = float(rng.choice([0.0, 0.05, 0.3, 1.0, 3.0]))
            if sig > 0:
                x = (x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L))).astype(np.complex64)
        out[f] = x
    return out


def oracle_frames(O, iq, sf, osr, hann, dechirp):
    rows = []
    for f in range(iq.shape[0]):
        x = O.dechirp(iq[f], sf, osr) if dechirp else iq[f]
        rows.append(O.lora_demodulate(x, sf, osr, hann))
    return rows


CASES = [  # (sf, osr, hann, dechirp, F, symbols-per-frame, extra samples, kind)
    (7, 1, False, True, 24, 66, 0, "mod"),
    (7, 1, False, False, 16, 20, 37, "mod"),
    (7, 2, False, True, 8, 11, 0, "mod"),
    (7, 1, True, False, 8, 18, 0, "noise"),
    (8, 1, False, True, 12, 34, 0, "mod"),
    (9, 3, True, True, 4, 9, 5, "mod"),
    (10, 1, False, False, 6, 12, 0, "noise"),
    (11, 2, False, True, 3, 7, 100, "mod"),
    (12, 1, False, True, 4, 10, 0, "mod"),
    (12, 1, True, False, 2, 6, 17, "noise"),
    (2, 1, False, False, 40, 9, 1, "noise"),
    (3, 4, True, False, 10, 5, 3, "mod"),
    (5, 1, False, True, 10, 30, 0, "mod"),
    (6, 2, False, False, 6, 3, 0, "noise"),
    (7, 1, False, False, 5, 1, 20, "noise"),  # one symbol: no sync pair
    (7, 1, False, False, 3, 0, 50, "noise"),  # no whole symbol
]


def make_plan(amd, path, *args, **kw):
    """path "fast": the default - register-blocked kernels, as the speculative single-read
    pipeline wherever it covers the configuration (LEGACY, osr 1, SF >= 6,
    >= 3 symbols, either window); "split": the same kernels as three launches (frame max, estimate,
    demod: LORA_MI355X_SPEC=0, the one diagnostic knob)."""
    with amd.spec_pipeline(path != "split"):
        return amd.DemodPlan(*args, **kw)


@pytest.mark.parametrize("path", ["fast", "split"])
@pytest.mark.parametrize("case", CASES, ids=[f"sf{c[0]}-osr{c[1]}-h{int(c[2])}-d{int(c[3])}-{c[7]}-S{c[5]}"
                                             for c in CASES])
def test_legacy_demod_matches_oracle(O, amd, case, path):
    sf, osr, hann, dechirp, F, nsym, extra, kind = case
    rng = np.random.default_rng(sf * 1000 + osr * 10 + nsym)
    L = nsym * (1 << sf) * osr + extra
    iq = make_frames(O, rng, sf, osr, F, L, kind, dechirp)
    plan = make_plan(amd, path, sf, osr, 125000, "hann" if hann else "none", dechirp=dechirp)
    res = plan.run(torch.from_numpy(iq).cuda())
    torch.cuda.synchronize()
    syms = res.symbols.cpu().numpy()
    sync = res.sync.cpu().numpy()
    cfo = res.cfo.cpu().numpy()
    toff = res.time_offset.cpu().numpy()
    for f, (os_, osync, ocfo, otoff) in enumerate(oracle_frames(O, iq, sf, osr, hann, dechirp)):
        assert syms.shape[1] == len(os_)
        np.testing.assert_array_equal(syms[f], os_, err_msg=f"frame {f} symbols")
        assert sync[f] == osync, f"frame {f} sync"
        assert bits(cfo[f]) == bits(ocfo), f"frame {f} cfo {cfo[f]} vs {ocfo}"
        assert bits(toff[f]) == bits(otoff), f"frame {f} toff {toff[f]} vs {otoff}"


@pytest.mark.parametrize("sf,osr,hann", [(7, 1, False), (8, 2, True), (12, 1, False), (9, 1, False)])
def test_api_demod_matches_oracle(O, amd, sf, osr, hann):
    rng = np.random.default_rng(77 + sf)
    N = 1 << sf
    F, S = 6, 10
    frames = []
    for f in range(F):
        syms = rng.integers(0, N, S).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, 0x12)
        x = (x + 0.2 * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x)))).astype(np.complex64)
        frames.append(x)
    iq = np.stack(frames)
    plan = amd.DemodPlan(sf, osr, 125000, "hann" if hann else "none", mode="api")
    res = plan.run(torch.from_numpy(iq).cuda())
    syms = res.symbols.cpu().numpy()
    for f in range(F):
        r, osym, osync, ocfo, otoff = O.api_demodulate(iq[f], sf, osr, hann)
        assert r == S
        np.testing.assert_array_equal(syms[f], osym)
        assert int(res.sync[f]) == osync
        assert bits(res.cfo[f].item()) == bits(ocfo)
        assert bits(res.time_offset[f].item()) == bits(otoff)


def test_api_mode_rejects_partial_symbols(amd):
    plan = amd.DemodPlan(7, 1, mode="api")
    with pytest.raises(amd.LoraError):
        plan.run(torch.zeros((1, 128 * 5 + 3), dtype=torch.complex64, device="cuda"))
    with pytest.raises(amd.LoraError):
        plan.run(torch.zeros((1, 128), dtype=torch.complex64, device="cuda"))


@pytest.mark.parametrize("sf,osr,bw", [(7, 1, 125000), (8, 2, 250000), (12, 1, 500000), (2, 3, 125000),
                                       (10, 1, 125000), (11, 2, 125000), (10, 4, 250000), (12, 2, 125000)])
def test_modulator_matches_oracle(O, amd, sf, osr, bw):
    rng = np.random.default_rng(sf + osr)
    F, S = 5, 12
    syms = rng.integers(0, 1 << sf, (F, S)).astype(np.uint16)
    iq = amd.modulate(torch.from_numpy(syms.astype(np.int32)).cuda(), sf, osr, bw, 0.9, 0x34)
    got = iq.cpu().numpy()
    for f in range(F):
        ref = O.lora_modulate(syms[f], sf, osr, bw, 0.9, 0x34)
        np.testing.assert_array_equal(got[f].view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("sf,frames", [(10, 2100), (12, 1030)])
def test_modulator_many_frames_matches_oracle(O, amd, sf, frames):
    """More than 1024 frames: k_mod_phase packs several frames per wave (ModArgs::fpw) and
    runs the recurrence in speculative 16-step blocks; frames from the first, middle and
    last waves against the oracle, bit for bit."""
    rng = np.random.default_rng(sf)
    S = 3
    syms = rng.integers(0, 1 << sf, (frames, S)).astype(np.uint16)
    iq = amd.modulate(torch.from_numpy(syms.astype(np.int32)).cuda(), sf, 1, 125000, 1.0, 0x12)
    for f in (0, 1, 63, 64, frames // 2, frames - 2, frames - 1):
        ref = O.lora_modulate(syms[f], sf, 1, 125000, 1.0, 0x12)
        np.testing.assert_array_equal(iq[f].cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("sf,osr,S,frames,big", [(7, 1, 64, 1, False), (7, 1, 64, 1, True), (8, 3, 40, 3, True),
                                                  (10, 1, 30, 2, True), (11, 3, 6, 2, False), (12, 1, 10, 1, True),
                                                  (12, 4, 3, 2, False), (2, 1, 50, 4, True), (9, 2, 20, 512, False),
                                                  (9, 2, 20, 513, False), (10, 5, 6, 3, False), (10, 9, 4, 2, True),
                                                  (9, 5, 8, 2, False), (12, 3, 3, 1, False)])
def test_modulator_frame_kernel_matches_oracle(O, amd, sf, osr, S, frames, big):
    """Up to 512 frames take k_mod_frame (a workgroup per frame: frequencies from the runs of
    csrc/lora_chirp.h or the per-chirp recurrence, one lane's phase chain, parallel sincosf)
    - 513 the bulk kernels.  Windows of whole chirps and of chirp fractions (osr 3/4 at
    SF 11/12), partial last windows, and symbols >= N (lora_encode's codewords reach 255;
    `big`: uint16 values up to 65535, whose chirps may overflow the run table and fall back
    to the recurrence) - every sample bit for bit against the oracle.  osr 5 at SF10 (5,120-sample
    chirps) and osr 9 have no window length that is an exact fraction of a chirp: they take the
    bulk kernels - checked the same way."""
    rng = np.random.default_rng(sf * 131 + osr + frames)
    hi = 65536 if big else (1 << sf)
    syms = rng.integers(0, hi, (frames, S)).astype(np.uint16)
    bw = 250000 if sf == 10 else 125000
    iq = amd.modulate(torch.from_numpy(syms.astype(np.int32)).cuda(), sf, osr, bw, 1.0, 0x12).cpu().numpy()
    for f in sorted({0, frames // 2, frames - 1}):
        ref = O.lora_modulate(syms[f], sf, osr, bw, 1.0, 0x12)
        np.testing.assert_array_equal(iq[f].view(np.uint32), ref.view(np.uint32))


def test_modulator_into_a_preallocated_buffer(amd):
    """modulate(..., out=): the same samples written into the caller's buffer (what
    bench.py times), and a wrong-shaped buffer is refused."""
    syms = torch.randint(0, 128, (3, 9), dtype=torch.int32).cuda()
    ref = amd.modulate(syms, 7)
    out = torch.full_like(ref, complex(7.0, 7.0))
    got = amd.modulate(syms, 7, out=out)
    assert got.data_ptr() == out.data_ptr()
    assert torch.equal(out.view(torch.int64), ref.view(torch.int64))
    with pytest.raises(ValueError):
        amd.modulate(syms, 7, out=torch.empty((3, 10), dtype=torch.complex64, device="cuda"))


def test_estimate_and_compensate_match_oracle(O, amd):
    rng = np.random.default_rng(5)
    sf, osr = 8, 2
    L = 5 * (1 << sf) * osr + 11
    iq = (rng.standard_normal((4, L)) + 1j * rng.standard_normal((4, L))).astype(np.complex64)
    plan = amd.DemodPlan(sf, osr, window="hann", mode="api")
    cfo = torch.zeros(4, device="cuda")
    toff = torch.zeros(4, device="cuda")
    plan.estimate_offsets(torch.from_numpy(iq).cuda(), cfo, toff)
    for f in range(4):
        oc, ot = O.estimate_offsets(iq[f], sf, osr, True)
        assert bits(cfo[f].item()) == bits(oc)
        assert bits(toff[f].item()) == bits(ot)
    cfo_in = torch.tensor([0.3, -0.7, 1.9, 0.0], device="cuda")
    to_in = torch.tensor([3.4, -5.6, 0.2, 2000.0], device="cuda")
    out = amd.compensate_offsets(torch.from_numpy(iq).cuda(), sf, osr, cfo_in, to_in).cpu().numpy()
    for f in range(4):
        ref = O.compensate_offsets(iq[f], sf, osr, float(cfo_in[f]), float(to_in[f]))
        np.testing.assert_array_equal(out[f].view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("sf,F,nsym,hann,dechirp,mode", [
    (7, 5000, 6, False, True, "legacy"),
    (9, 2100, 4, True, False, "legacy"),
    (8, 3000, 5, False, False, "api"),
])
def test_large_batch_matches_oracle(O, amd, sf, F, nsym, hann, dechirp, mode):
    """Thousands of frames per call (many workgroups per frame kind, mixed amplitudes);
    results must be identical to the one-frame-at-a-time oracle."""
    rng = np.random.default_rng(sf * 7 + F)
    N = 1 << sf
    L = nsym * N
    syms = rng.integers(0, N, (F, nsym - 2)).astype(np.int32)
    iq = amd.modulate(torch.from_numpy(syms).cuda(), sf, 1, 125000, 1.0, 0x12)
    noise = (rng.standard_normal((F, L)) + 1j * rng.standard_normal((F, L))).astype(np.complex64)
    scale = rng.choice([0.0, 0.2, 1.0, 4.0], F).astype(np.float32)[:, None]
    iq = iq + torch.from_numpy(noise * scale).cuda()
    if mode == "legacy" and not dechirp:
        iq = torch.from_numpy(np.stack([O.dechirp(r, sf) for r in iq.cpu().numpy()])).cuda()
    plan = amd.DemodPlan(sf, 1, 125000, "hann" if hann else "none", dechirp=dechirp, mode=mode)
    res = plan.run(iq)
    torch.cuda.synchronize()
    x = iq.cpu().numpy()
    if mode == "legacy":
        osyms, osync, ocfo, otoff, cnt = O.demod_frames(x, sf, 1, hann, dechirp=dechirp, threads=8)
        assert (cnt == nsym - 2).all()
        osyms = osyms[:, :nsym - 2]
    else:
        rows = [O.api_demodulate(x[f], sf, 1, hann) for f in range(F)]
        osyms = np.stack([r[1] for r in rows])
        osync = np.array([r[2] for r in rows])
        ocfo = np.array([r[3] for r in rows], np.float32)
        otoff = np.array([r[4] for r in rows], np.float32)
    np.testing.assert_array_equal(res.symbols.cpu().numpy(), osyms)
    np.testing.assert_array_equal(res.sync.cpu().numpy(), osync)
    np.testing.assert_array_equal(bits(res.cfo.cpu().numpy()), bits(ocfo))
    np.testing.assert_array_equal(bits(res.time_offset.cpu().numpy()), bits(otoff))


@pytest.mark.parametrize("sf,osr,hann,dechirp", [(7, 1, False, True), (7, 1, False, False), (9, 2, True, True),
                                                 (12, 1, False, True), (5, 3, True, False), (2, 1, False, False),
                                                 (11, 1, True, True)])
def test_raw_mode_matches_oracle(O, amd, sf, osr, hann, dechirp):
    """LORA_MODE_RAW (detector only) vs the oracle's orc_raw_demod, any SNR."""
    rng = np.random.default_rng(sf * 100 + osr)
    N = 1 << sf
    F, S = 6, 9
    L = S * N * osr + 5
    rows = []
    for f in range(F):
        syms = rng.integers(0, N, S - 2).astype(np.uint16)
        x = O.lora_modulate(syms, sf, osr, 125000, 1.0, 0x12)
        if not dechirp:
            x = O.dechirp(x, sf, osr)
        x = np.concatenate([x, np.zeros(5, np.complex64)])
        sig = [0.0, 0.5, 2.0][f % 3]
        x = (x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L))).astype(np.complex64)
        rows.append(x)
    iq = np.stack(rows)
    plan = amd.DemodPlan(sf, osr, 125000, "hann" if hann else "none", dechirp=dechirp, mode="raw")
    res = plan.run(torch.from_numpy(iq).cuda())
    got = res.symbols.cpu().numpy()
    assert got.shape == (F, L // (N * osr))  # every whole symbol, sync symbols included
    for f in range(F):
        np.testing.assert_array_equal(got[f], O.raw_demod(iq[f], sf, osr, hann, dechirp=dechirp))
    assert int(res.sync.to(torch.int32).sum()) == 0 and float(res.cfo.abs().sum()) == 0.0
