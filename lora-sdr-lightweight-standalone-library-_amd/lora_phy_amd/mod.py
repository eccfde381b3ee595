"""GPU modulation: lora_mod_batch wrapper and the LoRaMod block."""
from __future__ import annotations

from typing import Optional

import torch

from . import _capi
from .demod import _require_cuda, _stream_handle


def modulate(symbols: torch.Tensor, sf: int, osr: int = 1, bw: int = 125000,
             amplitude: float = 1.0, sync: int = 0x12, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """lora_modulate (LoRaMod.cpp:8-43) for a [F, S] (or [S]) uint16/int CUDA tensor.

    Returns complex64 [F, (S+2)*N*osr] (or 1-D): two sync up-chirps, then one
    up-chirp per symbol, phase-continuous within each frame.  `out`: a contiguous
    complex64 tensor of that shape on the symbols' device to write into (no allocation).
    """
    _require_cuda(symbols, "symbols")
    squeeze = symbols.dim() == 1
    s = symbols.unsqueeze(0) if squeeze else symbols
    if s.dtype != torch.uint16:
        s = s.to(torch.int32).to(torch.uint16)
    s = s.contiguous()
    F, S = s.shape
    osr = int(osr) if osr else 1
    per = (S + 2) * (1 << int(sf)) * osr
    if out is None:
        out = torch.empty((F, per), dtype=torch.complex64, device=s.device)
    else:
        want = (per,) if squeeze else (F, per)
        if (tuple(out.shape) != want or out.dtype != torch.complex64 or out.device != s.device
                or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous complex64 {want} tensor on {s.device}")
        out = out.view(F, per)
    lib = _capi.lib()
    _capi.check(lib.lora_mod_batch(int(sf), osr, int(bw), float(amplitude), int(sync) & 0xFF,
                                   s.data_ptr() if S > 0 else None, F, S, out.data_ptr(),
                                   s.device.index, _stream_handle(s.device)))
    return out[0] if squeeze else out


class LoRaMod:
    """Block-style modulator mirroring the Pothos ``/lora/lora_mod`` surface
    (examples/lora_simulation.pth:312-326: sf, sync, padding, ampl, ovs) plus bw."""

    def __init__(self, sf: int, sync: int = 0x12, padding: int = 0, ampl: float = 1.0,
                 ovs: int = 1, bw: int = 125000, device=None):
        self.sf, self.sync, self.padding = int(sf), int(sync) & 0xFF, int(padding)
        self.ampl, self.ovs, self.bw = float(ampl), int(ovs) if ovs else 1, int(bw)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)

    def work(self, symbols) -> torch.Tensor:
        if not isinstance(symbols, torch.Tensor):
            symbols = torch.as_tensor(symbols, dtype=torch.int32)
        symbols = symbols.to(self.device)
        iq = modulate(symbols, self.sf, self.ovs, self.bw, self.ampl, self.sync)
        if self.padding > 0:  # trailing zero samples between packets (block "padding")
            pad = torch.zeros(iq.shape[:-1] + (self.padding,), dtype=iq.dtype, device=iq.device)
            iq = torch.cat([iq, pad], dim=-1)
        return iq
