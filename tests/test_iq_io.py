"""CPU: IQ file I/O in the reference runners' format (rx_runner.cpp:72-79)."""
import os

import numpy as np
import torch

from lora_phy_amd import iq_io

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_roundtrip_and_odd_tail(tmp_path):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(1000) + 1j * rng.standard_normal(1000)).astype(np.complex64)
    p = str(tmp_path / "a.iq")
    assert iq_io.write_iq(p, torch.from_numpy(x)) == 1000
    with open(p, "ab") as fh:  # a trailing unpaired float is ignored, as rx_runner does
        fh.write(np.float32(7.0).tobytes())
    y = iq_io.read_iq(p, slice_samples=333)
    np.testing.assert_array_equal(y.numpy().view(np.uint64), x.view(np.uint64))
    f = iq_io.read_iq(p, frame_len=128)
    assert f.shape == (7, 128)
    chunks = list(iq_io.iter_frames(p, 128, 3))
    assert [c.shape[0] for c in chunks] == [3, 3, 1]
    np.testing.assert_array_equal(torch.cat(chunks).numpy(), f.numpy())


def test_reference_fixtures_read_like_the_runner():
    for name in ("test_output.iq", "capture_sf7_excerpt.iq"):
        p = os.path.join(GOLD, name)
        raw = np.fromfile(p, dtype="<f4")
        want = (raw[0:len(raw) // 2 * 2:2] + 1j * raw[1:len(raw) // 2 * 2:2]).astype(np.complex64)
        np.testing.assert_array_equal(iq_io.read_iq(p).numpy(), want)
