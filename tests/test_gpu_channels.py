"""GPU parity at the configs[4] shape (BASELINE.json: 8 channels x 1e6 frames, one channel
per GPU): 1,000,000 SF7 frames of 2 + 16 symbols resident in HBM (18.4 GB), demodulated in
<= 8 GB chunks like bench.py's channels line, with AWGN from noiseless to 0 dB so frames
rescale and shift their windows (t_off != 0).  From EVERY chunk, its first and last frames
and a seeded random sample are checked against the CPU oracle bit for bit (symbols, sync,
cfo / time_offset bits), through the default speculative single-read pipeline and through
the three-launch path, whose frame max runs as k_frame_max_wave (frames shorter than two
4096-sample batches).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("path", ["spec", "split"])
def test_configs4_shape_every_chunk_vs_oracle(path):
    """path "spec": the default speculative single-read pipeline; "split": three launches
    (LORA_MI355X_SPEC=0) with the one-wave-per-frame max pass."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lora_phy_amd as amd
    from oracle.pyoracle import Oracle

    O = Oracle()
    dev = torch.device("cuda", 0)
    sf, N, S, frames = 7, 128, 16, 1_000_000
    L = (S + 2) * N
    iq = torch.empty((frames, L), dtype=torch.complex64, device=dev)
    g = torch.Generator(device="cpu").manual_seed(2024)
    gn = torch.Generator(device=dev).manual_seed(2025)
    rows = 1 << 17
    for r0 in range(0, frames, rows):
        n = min(rows, frames - r0)
        syms = torch.randint(0, N, (n, S), generator=g, dtype=torch.int32).to(dev)
        x = amd.modulate(syms, sf, 1, 125000, 1.0, 0x12)
        # per-frame noise level: none, 10 dB, 0 dB (sigma/sqrt2 per component)
        lvl = torch.tensor([0.0, 10 ** (-10 / 20) / np.sqrt(2), 1 / np.sqrt(2)], device=dev)
        sig = lvl[torch.randint(0, 3, (n,), generator=gn, device=dev)][:, None]
        x += torch.view_as_complex(torch.randn((n, L, 2), generator=gn, device=dev)) * sig
        iq[r0:r0 + n] = x
        del x
    with amd.spec_pipeline(path != "split"):
        plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=dev)
    want = {"spec", "estimate", "demod"} if path == "spec" else {"frame_max", "frame_max_wave", "estimate", "demod"}
    per_chunk = int(8e9 // (L * 8))
    chunks = [(c0, min(per_chunk, frames - c0)) for c0 in range(0, frames, per_chunk)]
    assert len(chunks) == 3
    rng = np.random.default_rng(7)
    shifted = 0
    for c0, n in chunks:
        res = plan.run(iq[c0:c0 + n])
        torch.cuda.synchronize()
        assert plan.last_kernels() == want, plan.last_kernels()
        pick = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 46)]))
        idx = torch.from_numpy(pick).to(dev)
        x = iq[c0:c0 + n].index_select(0, idx).cpu().numpy()
        osyms, osync, ocfo, otoff, cnt = O.demod_frames(x, sf, 1, False, dechirp=True, threads=8)
        assert (cnt == S).all()
        got = res.symbols.index_select(0, idx).cpu().numpy()
        np.testing.assert_array_equal(got, osyms[:, :S], err_msg=f"chunk at {c0}")
        np.testing.assert_array_equal(res.sync.index_select(0, idx).cpu().numpy(), osync)
        np.testing.assert_array_equal(bits(res.cfo.index_select(0, idx).cpu().numpy()), bits(ocfo))
        np.testing.assert_array_equal(bits(res.time_offset.index_select(0, idx).cpu().numpy()), bits(otoff))
        shifted += int((np.rint(otoff) != 0).sum())
        del res
    assert shifted > 0, "no sampled frame had a shifted symbol window"
    del iq
    torch.cuda.empty_cache()
