"""IQ file I/O: the reference runners' raw format, streamed into HBM.

Format (runners/rx_runner.cpp:72-79, runners/tx_runner.cpp:133-138): interleaved
little-endian float32 (I, Q) pairs, no header; a trailing unpaired float is ignored.
Files are memory-mapped and copied to the device in slices, so captures larger than
host RAM stream through; frames are rows of `frame_len` samples.
"""
from __future__ import annotations

import os
from typing import Iterator, Optional

import numpy as np
import torch


def _mmap(path: str) -> np.ndarray:
    n = os.path.getsize(path) // 8
    if n == 0:
        return np.zeros(0, np.complex64)
    return np.memmap(path, dtype=np.complex64, mode="r", shape=(n,))


def read_iq(path: str, device=None, frame_len: Optional[int] = None, max_samples: Optional[int] = None,
            slice_samples: int = 1 << 24) -> torch.Tensor:
    """Whole file (or its first `max_samples`) as complex64 on `device` ([L], or [F, frame_len]
    with the tail that does not fill a frame dropped, like rx_runner's whole-symbol rule)."""
    x = _mmap(path)
    if max_samples is not None:
        x = x[:max_samples]
    if frame_len:
        x = x[: (len(x) // frame_len) * frame_len]
    dev = torch.device("cpu") if device is None else torch.device(device)
    out = torch.empty(len(x), dtype=torch.complex64, device=dev)
    for s0 in range(0, len(x), slice_samples):
        part = torch.from_numpy(np.array(x[s0:s0 + slice_samples]))  # writable host copy
        out[s0:s0 + len(part)].copy_(part, non_blocking=False)
    return out.view(-1, frame_len) if frame_len else out


def iter_frames(path: str, frame_len: int, frames_per_chunk: int, device=None) -> Iterator[torch.Tensor]:
    """Stream a capture as [<=frames_per_chunk, frame_len] device tensors."""
    x = _mmap(path)
    nf = len(x) // frame_len
    dev = torch.device("cpu") if device is None else torch.device(device)
    for f0 in range(0, nf, frames_per_chunk):
        n = min(frames_per_chunk, nf - f0)
        host = np.array(x[f0 * frame_len:(f0 + n) * frame_len]).reshape(n, frame_len)
        yield torch.from_numpy(host).to(dev)


def write_iq(path: str, iq: torch.Tensor) -> int:
    """tx_runner's output format; returns the number of samples written."""
    a = iq.detach().to("cpu").contiguous().view(-1).numpy().astype(np.complex64, copy=False)
    a.tofile(path)
    return len(a)
