"""GPU parity of the frame-resident single-read kernel (k_frame_fused) vs the CPU oracle.

The kernel reads each frame from HBM once into LDS and runs the normalisation
(LoRaDemod.cpp:59-77), the 2-symbol offset estimate (:79-135) and every symbol
(:137-192) from there, transposing each symbol in place in its own LDS row.  The
cases here aim at what that design adds: rounds going up (t_off >= 0) and down
(t_off < 0), two or more rounds per frame, odd frame lengths (a partial last row), frames
with and without rescaling, the FAST rotation, and the LDS limit (LORA_MI355X_FUSED).
Every output must equal the oracle bit for bit, and the plan must report that the
fused kernel (and nothing else) ran.
"""
import os

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


ROW = {6: 68, 7: 136, 8: 272}  # lds_row<SF>() complex values per LDS row
TWT = {6: 48, 7: 120, 8: 240}   # pass-A slot-major twiddles


def fused_lds_bytes(sf, L):
    """k_frame_fused's dynamic LDS: frame rows + 2 scratch rows + FFT tables."""
    N = 1 << sf
    rows = -(-L // N)
    tables = (8 * (N + TWT[sf]) + 2 * N + 15) // 16 * 16
    return 8 * (rows + 2) * ROW[sf] + tables


LIMIT = {80: 80 * 1024 - 256, 160: 160 * 1024 - 128}


def plan_with(amd, sf, dechirp, fused_kib=80, precision="exact"):
    """fused_kib: LORA_MI355X_FUSED (the kernel is opt-in; 80 = two frames per CU)."""
    if fused_kib is not None:
        os.environ["LORA_MI355X_FUSED"] = str(fused_kib)
    try:
        return amd.DemodPlan(sf, 1, 125000, "none", dechirp=dechirp, precision=precision)
    finally:
        os.environ.pop("LORA_MI355X_FUSED", None)


def frames(O, rng, sf, F, nsym, extra, dechirp, cfo_bins=0.0):
    """Modulated frames (random sync), a per-frame noise level (none .. 0 dB .. -10 dB)
    and amplitude (rescaled or not), optionally a CFO ramp (phase cfo_bins*2*pi*n/N)."""
    N = 1 << sf
    L = nsym * N + extra
    out = np.zeros((F, L), np.complex64)
    n = np.arange(L)
    for f in range(F):
        syms = rng.integers(0, N, nsym - 2 + 1).astype(np.uint16)
        x = O.lora_modulate(syms, sf, 1, 125000, 1.0, int(rng.integers(0, 256)))[:L]
        x = np.concatenate([x, np.zeros(max(L - len(x), 0), np.complex64)])
        if cfo_bins:
            x = (x * np.exp(1j * 2 * np.pi * cfo_bins * n / N)).astype(np.complex64)
        sig = float(rng.choice([0.0, 0.1, 0.7, 1.0, 3.0]))
        amp = float(rng.choice([0.5, 1.0, 2.5]))
        x = amp * (x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L)))
        out[f] = x.astype(np.complex64)
    if not dechirp:
        out = np.stack([O.dechirp(r, sf) for r in out])
    return out


def device_frames(iq):
    """[F, L] on the GPU with an even row stride (16-byte aligned frames, as the fused
    kernel's loads need): odd lengths sit in an [F, L+1] buffer."""
    F, L = iq.shape
    if L % 2 == 0:
        return torch.from_numpy(iq).cuda()
    buf = torch.zeros((F, L + 1), dtype=torch.complex64, device="cuda")
    buf[:, :L] = torch.from_numpy(iq).cuda()
    return buf[:, :L]


def check(O, amd, plan, iq, sf, dechirp, expect_fused=True, limit_kib=80):
    if expect_fused:
        assert fused_lds_bytes(sf, iq.shape[1]) <= LIMIT[limit_kib], "case does not fit the fused kernel"
    res = plan.run(device_frames(iq))
    torch.cuda.synchronize()
    ran = plan.last_kernels()
    if expect_fused:
        assert ran == {"fused"}, ran
    else:
        assert "fused" not in ran, ran
    nsym = plan.symbols_per_frame(iq.shape[1])
    osyms, osync, ocfo, otoff, cnt = O.demod_frames(iq, sf, 1, False, dechirp=dechirp, threads=8)
    assert (cnt == nsym).all()
    np.testing.assert_array_equal(res.symbols.cpu().numpy(), osyms[:, :nsym])
    np.testing.assert_array_equal(res.sync.cpu().numpy(), osync)
    np.testing.assert_array_equal(bits(res.cfo.cpu().numpy()), bits(ocfo))
    np.testing.assert_array_equal(bits(res.time_offset.cpu().numpy()), bits(otoff))
    return np.rint(otoff).astype(np.int64)


# (sf, total symbols, extra samples, dechirp, frames): one and two rounds of data symbols
# per frame within the default limit (two frames per CU: rows + 2 scratch rows <= 80 KiB;
# SF7 rounds of 64, SF8 of 32, SF6 of 128)
CASES = [
    (7, 66, 0, True, 96),     # the benchmark shape: one round of 64
    (7, 66, 0, False, 64),
    (7, 69, 33, True, 64),    # two rounds (64 + 3), odd length: partial last row
    (7, 18, 0, True, 128),    # configs[4] shape (S = 16)
    (7, 5, 1, False, 32),     # three data symbols, odd length
    (8, 32, 255, True, 48),   # SF8, partial last row of 255 samples
    (8, 31, 77, False, 48),   # SF8, odd length
    (6, 36, 0, True, 64),     # SF6
    (6, 140, 0, True, 32),    # two rounds (128 + 10) at SF6
    (6, 12, 3, False, 64),
    (7, 2, 0, True, 16),      # sync symbols only, no data symbol
]


@pytest.mark.parametrize("sf,nsym,extra,dechirp,F", CASES,
                         ids=[f"sf{c[0]}-S{c[1]}-x{c[2]}-d{int(c[3])}" for c in CASES])
def test_fused_matches_oracle(O, amd, sf, nsym, extra, dechirp, F):
    rng = np.random.default_rng(sf * 101 + nsym * 7 + extra)
    plan = plan_with(amd, sf, dechirp)
    iq = frames(O, rng, sf, F, nsym, extra, dechirp)
    check(O, amd, plan, iq, sf, dechirp)


@pytest.mark.parametrize("cfo_bins", [0.3, -0.3, 0.45, -0.45])
def test_fused_both_round_orders(O, amd, cfo_bins):
    """A fractional CFO makes the estimate shift symbol windows (t_off != 0, sign of
    -frac): rounds go up for t_off > 0 and down for t_off < 0, over two rounds per frame."""
    sf, nsym, F = 7, 69, 64
    rng = np.random.default_rng(int(abs(cfo_bins) * 1000) + (5 if cfo_bins > 0 else 6))
    plan = plan_with(amd, sf, True)
    iq = frames(O, rng, sf, F, nsym, 17, True, cfo_bins=cfo_bins)
    t_off = check(O, amd, plan, iq, sf, True)
    assert (t_off != 0).any(), "no frame exercised a shifted window"


def test_fused_orders_seen(O, amd):
    """Across CFOs of both signs the batch holds frames with t_off > 0 and t_off < 0."""
    sf, nsym, F = 8, 33, 96
    rng = np.random.default_rng(77)
    plan = plan_with(amd, sf, True)
    parts = [frames(O, rng, sf, F // 2, nsym, 0, True, cfo_bins=c) for c in (0.4, -0.4)]
    t_off = check(O, amd, plan, np.concatenate(parts), sf, True)
    assert (t_off > 0).any() and (t_off < 0).any(), np.unique(t_off)


@pytest.mark.parametrize("sf,nsym", [(7, 140), (8, 69), (6, 288)])
def test_fused_large_lds_limit(O, amd, sf, nsym):
    """LORA_MI355X_FUSED=160: frames up to 160 KiB of LDS (one per CU), three or more rounds."""
    rng = np.random.default_rng(sf + nsym)
    plan = plan_with(amd, sf, True, fused_kib=160)
    iq = frames(O, rng, sf, 16, nsym, 9, True, cfo_bins=float(rng.choice([0.3, -0.3])))
    check(O, amd, plan, iq, sf, True, limit_kib=160)


def test_fused_two_rounds_sf8(O, amd):
    """SF8: rounds of 32 symbols; 35 symbols per frame need the 160 KiB limit."""
    rng = np.random.default_rng(88)
    plan = plan_with(amd, 8, True, fused_kib=160)
    iq = frames(O, rng, 8, 32, 35, 0, True, cfo_bins=-0.35)
    check(O, amd, plan, iq, 8, True, limit_kib=160)


def test_fused_off_and_over_limit(O, amd):
    """LORA_MI355X_FUSED unset (the default) or 0, and frames over the limit, take the
    three-launch path."""
    rng = np.random.default_rng(3)
    iq = frames(O, rng, 7, 8, 66, 0, True)
    check(O, amd, plan_with(amd, 7, True, fused_kib=0), iq, 7, True, expect_fused=False)
    check(O, amd, plan_with(amd, 7, True, fused_kib=None), iq, 7, True, expect_fused=False)  # default: off
    iq = frames(O, rng, 7, 8, 90, 0, True)  # 92 rows x 1088 B > 80 KiB
    check(O, amd, plan_with(amd, 7, True), iq, 7, True, expect_fused=False)


def test_fused_fast_rotation_matches_split(amd, O):
    """precision="fast": the fused kernel's rotation is the hardware sin/cos of the split
    path's k_demod_fast<FAST>, so both give the same symbols; the estimate and sync stay
    exact (equal to the oracle)."""
    sf, nsym, F = 7, 66, 64
    rng = np.random.default_rng(11)
    iq = frames(O, rng, sf, F, nsym, 0, True)
    x = torch.from_numpy(iq).cuda()
    pf = plan_with(amd, sf, True, precision="fast")
    ps = plan_with(amd, sf, True, fused_kib=0, precision="fast")
    rf, rs = pf.run(x), ps.run(x)
    torch.cuda.synchronize()
    assert pf.last_kernels() == {"fused"} and "fused" not in ps.last_kernels()
    np.testing.assert_array_equal(rf.symbols.cpu().numpy(), rs.symbols.cpu().numpy())
    _, osync, ocfo, otoff, _ = O.demod_frames(iq, sf, 1, False, dechirp=True, threads=8)
    np.testing.assert_array_equal(rf.sync.cpu().numpy(), osync)
    np.testing.assert_array_equal(bits(rf.cfo.cpu().numpy()), bits(ocfo))


def test_fused_unaligned_stride_falls_back(O, amd):
    """An odd frame stride (frames not 16-byte aligned) takes the three-launch path."""
    sf, nsym, F = 7, 20, 8  # L even, stride L + 1 odd
    rng = np.random.default_rng(5)
    iq = frames(O, rng, sf, F, nsym, 0, True)
    L = iq.shape[1]
    buf = torch.zeros((F, L + 1), dtype=torch.complex64, device="cuda")
    buf[:, :L] = torch.from_numpy(iq).cuda()
    view = buf[:, :L]
    plan = plan_with(amd, sf, True)
    res = plan.run(view)
    torch.cuda.synchronize()
    assert "fused" not in plan.last_kernels()
    osyms, osync, _, _, _ = O.demod_frames(iq, sf, 1, False, dechirp=True, threads=8)
    np.testing.assert_array_equal(res.symbols.cpu().numpy(), osyms[:, :nsym - 2])
