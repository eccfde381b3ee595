"""GPU: the speculative certified pipeline is exact at scale, under near-ties and on long
frames.

* Every symbol, sync word and cfo / time_offset / max_amp bit of >= 1e5 SF7 frames and
  >= 2,000 SF12 frames at -10 and -15 dB with a 0.4-bin carrier offset and per-frame
  sample delays is compared between the default pipeline and the three-launch path
  (LORA_MI355X_SPEC=0: frame max, estimate, demod with glibc-faithful sincosf, itself
  oracle-pinned by test_gpu_parity / test_gpu_spec).  Millions of argmax margins sit
  near the certification bound here; the recomputed-symbol count is printed.
* The full configs[2] batch (15,625 SF12 frames x 66 symbols = 33.8 GB, 4.3e9 samples,
  past 2^32) through the default pipeline, its first, last and 46 random frames against
  the CPU oracle bit for bit (the large-offset addressing at the end of the batch).
* Long frames (82, 256 and 512 symbols at SF7; 100 at SF12) run in the single-read
  pipeline and match the oracle (reference: LoRaDemod.cpp:55-77 has no length limit).

Reference: /root/reference/src/phy/LoRaDemod.cpp:137-175 (the per-symbol loop the
certification must reproduce), tests/awgn_sweep.py:245-273 (the SNR model).
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SPEC = {"spec", "estimate", "demod"}


@pytest.fixture(scope="module")
def amd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lora_phy_amd

    return lora_phy_amd


@pytest.fixture(scope="module")
def O():
    from oracle.pyoracle import Oracle

    return Oracle()


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def noisy_batch(amd, sf, F, S, snr_db, cfo_bins, seed, chunk=8192):
    """[F, (S+2) N] raw IQ on the GPU: GPU-modulated random symbols (amplitude 1, sync
    0x12), a carrier offset of `cfo_bins` bins, a random delay of 0..N/3 samples per frame
    (zero fill), complex AWGN with sigma = 10^(-snr/20) / sqrt(2) per component
    (awgn_sweep_gtest.cpp:76-80).  Built in chunks of `chunk` frames."""
    dev = torch.device("cuda", 0)
    N = 1 << sf
    L = (S + 2) * N
    iq = torch.empty((F, L), dtype=torch.complex64, device=dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    gn = torch.Generator(device=dev).manual_seed(seed + 1)
    n_idx = torch.arange(L, device=dev)
    rot = torch.polar(torch.ones(L, device=dev, dtype=torch.float64),
                      2 * np.pi * cfo_bins * n_idx.to(torch.float64) / N).to(torch.complex64)
    sigma = 10.0 ** (-snr_db / 20.0) / np.sqrt(2.0)
    for r0 in range(0, F, chunk):
        n = min(chunk, F - r0)
        syms = torch.randint(0, N, (n, S), generator=g, dtype=torch.int32).to(dev)
        x = amd.modulate(syms, sf, 1, 125000, 1.0, 0x12) * rot
        d = torch.randint(0, N // 3, (n, 1), generator=gn, device=dev)
        src = n_idx[None, :] - d
        x = torch.where(src >= 0, torch.gather(x, 1, src.clamp(min=0)), torch.zeros((), dtype=x.dtype, device=dev))
        x += torch.view_as_complex(torch.randn((n, L, 2), generator=gn, device=dev)) * sigma
        iq[r0:r0 + n] = x
        del x, src
    return iq


def plan_for(amd, sf, spec):
    with amd.spec_pipeline(spec):
        return amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy")


@pytest.mark.parametrize("sf,F", [(7, 100_000), (12, 2_000)])
@pytest.mark.parametrize("snr_db", [-10, -15])
def test_certified_equals_exact_every_symbol(amd, sf, F, snr_db):
    S = 64
    iq = noisy_batch(amd, sf, F, S, snr_db, 0.4, 9000 + sf * 10 - snr_db)
    ps, px = plan_for(amd, sf, True), plan_for(amd, sf, False)
    fixed0 = ps.spec_recomputed()
    rs = ps.run(iq)
    rx = px.run(iq)
    torch.cuda.synchronize()
    assert ps.last_kernels() == SPEC and "spec" not in px.last_kernels()
    fixed = ps.spec_recomputed() - fixed0
    bad = int((rs.symbols != rx.symbols).sum())
    print(f"\nSF{sf} {snr_db} dB: {F} frames x {S} data symbols, {fixed} recomputed "
          f"({fixed / (F * S):.2e} of the symbols), mismatches {bad}")
    assert bad == 0
    assert torch.equal(rs.sync, rx.sync)
    for name in ("cfo", "time_offset", "max_amp"):
        a, b = getattr(rs, name), getattr(rx, name)
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), name
    # the batch exercised near-ties and shifted windows
    assert fixed > 0
    assert int((rs.time_offset.round() != 0).sum()) > F // 10
    del iq
    torch.cuda.empty_cache()


def test_configs2_full_batch_vs_oracle(amd, O):
    """BASELINE.json configs[2]: 1,000,000 SF12 data symbols = 15,625 frames x (2 + 64),
    33.8 GB resident, 0 dB AWGN with a 0.3-bin carrier offset, one call."""
    sf, S, F = 12, 64, 15625
    N = 1 << sf
    iq = noisy_batch(amd, sf, F, S, 0.0, 0.3, 4242, chunk=512)
    assert iq.numel() > 2 ** 31  # complex samples: 64-bit indexing
    plan = plan_for(amd, sf, True)
    res = plan.run(iq)
    torch.cuda.synchronize()
    assert plan.last_kernels() == SPEC
    rng = np.random.default_rng(12)
    pick = np.unique(np.concatenate([[0, F - 1], rng.integers(0, F, 46)]))
    idx = torch.from_numpy(pick).to(iq.device)
    x = iq.index_select(0, idx).cpu().numpy()
    osyms, osync, ocfo, otoff, cnt = O.demod_frames(x, sf, 1, False, dechirp=True, threads=8)
    assert (cnt == S).all()
    np.testing.assert_array_equal(res.symbols.index_select(0, idx).cpu().numpy(), osyms[:, :S])
    np.testing.assert_array_equal(res.sync.index_select(0, idx).cpu().numpy(), osync)
    np.testing.assert_array_equal(bits(res.cfo.index_select(0, idx).cpu().numpy()), bits(ocfo))
    np.testing.assert_array_equal(bits(res.time_offset.index_select(0, idx).cpu().numpy()), bits(otoff))
    print(f"\nconfigs[2]: {F} frames, {iq.numel() * 8 / 1e9:.1f} GB, {len(pick)} frames vs oracle, "
          f"{plan.spec_recomputed()} recomputed, last frame at sample offset {(F - 1) * (S + 2) * N}")
    del iq, res
    torch.cuda.empty_cache()


@pytest.mark.parametrize("sf,nsym,F,snr_db", [(7, 82, 16, 0.0), (7, 256, 12, -5.0), (7, 512, 12, 5.0),
                                              (7, 514, 4, -10.0), (12, 100, 3, 0.0), (9, 300, 4, 10.0)])
def test_long_frames_single_read_vs_oracle(amd, O, sf, nsym, F, snr_db):
    """Frames past the former 81-symbol limit run in the speculative pipeline (SPEC
    kernels only) and equal the oracle bit for bit; 514 symbols = 2 + 512 is the SF7
    maximum (kSpecChunks * T data symbols)."""
    iq = noisy_batch(amd, sf, F, nsym - 2, snr_db, 0.25, 300 + nsym + sf)
    plan = plan_for(amd, sf, True)
    res = plan.run(iq)
    torch.cuda.synchronize()
    assert plan.last_kernels() == SPEC, plan.last_kernels()
    x = iq.cpu().numpy()
    osyms, osync, ocfo, otoff, cnt = O.demod_frames(x, sf, 1, False, dechirp=True, threads=8)
    assert (cnt == nsym - 2).all()
    np.testing.assert_array_equal(res.symbols.cpu().numpy(), osyms[:, :nsym - 2])
    np.testing.assert_array_equal(res.sync.cpu().numpy(), osync)
    np.testing.assert_array_equal(bits(res.cfo.cpu().numpy()), bits(ocfo))
    np.testing.assert_array_equal(bits(res.time_offset.cpu().numpy()), bits(otoff))


def test_past_the_pipeline_limit_takes_three_launches(amd, O):
    """SF7 frames of 515 symbols (513 data symbols > kSpecChunks * T) take the three-launch
    path, also exact."""
    iq = noisy_batch(amd, 7, 3, 513, 0.0, 0.1, 77)
    plan = plan_for(amd, 7, True)
    res = plan.run(iq)
    torch.cuda.synchronize()
    assert "spec" not in plan.last_kernels() and "frame_max" in plan.last_kernels()
    x = iq.cpu().numpy()
    osyms, osync, ocfo, otoff, cnt = O.demod_frames(x, 7, 1, False, dechirp=True, threads=8)
    np.testing.assert_array_equal(res.symbols.cpu().numpy(), osyms[:, :513])
    np.testing.assert_array_equal(bits(res.cfo.cpu().numpy()), bits(ocfo))
