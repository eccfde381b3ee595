"""Functional mirror of ``include/lora_phy/phy.hpp`` over GPU tensors.

Same names, argument meaning and error behaviour as the reference's C++ API, so code
and tests written against it read the same here; IQ is a torch.complex64 CUDA(HIP)
tensor (one frame ``[L]`` or a batch ``[F, L]``) and the arithmetic runs in the HIP
kernels behind include/lora_mi355x.h.  Where the reference returns ``-1`` this raises
:class:`LoraError` (code -EINVAL / -ERANGE).

Workspace API (phy.hpp:51-156, phy.cpp):  init, reset, encode, decode, modulate,
demodulate, estimate_offsets, compensate_offsets, get_last_metrics.
Legacy API (phy.hpp:170-215, LoRaDemod.cpp / LoRaMod.cpp / LoRaEncoder.cpp /
LoRaDecoder.cpp):  lora_demod_init, lora_demod_free, lora_demodulate, lora_modulate,
lora_encode, lora_decode, bw_scale.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np
import torch

from . import _capi, codes
from ._capi import LoraError
from .demod import DemodPlan, compensate_offsets as _compensate
from .mod import modulate as _modulate

BANDWIDTHS = (125000, 250000, 500000)  # phy.hpp:37-41


def bw_scale(bw: int) -> float:
    """phy.hpp:47-49."""
    return float(bw) / 125000.0


@dataclass
class lora_params:  # noqa: N801 - reference name (phy.hpp:51-58)
    sf: int = 7
    bw: int = 125000
    cr: int = 0
    osr: int = 1
    window: str = "none"
    sync_word: int = 0x12


@dataclass
class lora_metrics:  # noqa: N801 - phy.hpp:63-67 (per frame for batches)
    crc_ok: object = False
    cfo: object = 0.0
    time_offset: object = 0.0


@dataclass
class lora_workspace:  # noqa: N801 - phy.hpp:77-92; device plan instead of buffers
    sf: int = 0
    osr: int = 1
    bw: int = 125000
    window: str = "none"
    sync_word: object = 0x12
    metrics: lora_metrics = field(default_factory=lora_metrics)
    plan: Optional[DemodPlan] = None


def _err(code: int, msg: str):
    raise LoraError(code, msg)


def init(cfg: lora_params, device=None) -> lora_workspace:
    """phy.cpp:26-49.  Builds the device plan (API-mode demodulator)."""
    if cfg is None:
        _err(_capi.LORA_EINVAL, "null config")
    if not 2 <= int(cfg.sf) <= 12 or int(cfg.bw) not in BANDWIDTHS or cfg.window not in ("none", "hann"):
        _err(_capi.LORA_EINVAL, "invalid lora_params")
    ws = lora_workspace(sf=int(cfg.sf), osr=int(cfg.osr) or 1, bw=int(cfg.bw), window=cfg.window,
                        sync_word=int(cfg.sync_word) & 0xFF)
    ws.plan = DemodPlan(ws.sf, ws.osr, ws.bw, ws.window, mode="api", device=device)
    return ws


def reset(ws: lora_workspace) -> None:
    """phy.cpp:51-53."""
    if ws is not None:
        ws.metrics = lora_metrics()


def encode(ws: lora_workspace, payload: bytes, symbol_cap: Optional[int] = None) -> np.ndarray:
    """phy.cpp:55-63 (Hamming 8/4 per nibble, host-side)."""
    if ws is None or payload is None:
        _err(_capi.LORA_EINVAL, "null argument")
    syms = codes.lora_encode(payload)
    if symbol_cap is not None and len(syms) > symbol_cap:
        _err(_capi.LORA_ERANGE, "symbol buffer too small")
    return syms


def decode(ws: lora_workspace, symbols, payload_cap: Optional[int] = None) -> bytes:
    """phy.cpp:241-256: decode and set metrics.crc_ok (SX1272 CRC over [2, n-2))."""
    if ws is None or symbols is None:
        _err(_capi.LORA_EINVAL, "null argument")
    if isinstance(symbols, torch.Tensor):
        symbols = symbols.cpu().numpy()
    out, ok = codes.decode_with_crc(np.asarray(symbols).reshape(-1))
    if payload_cap is not None and len(out) > payload_cap:
        _err(_capi.LORA_ERANGE, "payload buffer too small")
    ws.metrics.crc_ok = bool(ok)
    return out.tobytes()


def modulate(ws: lora_workspace, symbols, iq_cap: Optional[int] = None) -> torch.Tensor:
    """phy.cpp:65-76: lora_modulate with the workspace's sf/osr/bw/sync, amplitude 1."""
    if ws is None or symbols is None:
        _err(_capi.LORA_EINVAL, "null argument")
    dev = ws.plan.device if ws.plan is not None else torch.device("cuda")
    s = symbols if isinstance(symbols, torch.Tensor) else torch.as_tensor(np.asarray(symbols, np.int32))
    iq = _modulate(s.to(dev), ws.sf, ws.osr, ws.bw, 1.0, int(ws.sync_word) & 0xFF)
    if iq_cap is not None and iq.shape[-1] > iq_cap:
        _err(_capi.LORA_ERANGE, "iq buffer too small")
    return iq


def demodulate(ws: lora_workspace, iq: torch.Tensor, symbol_cap: Optional[int] = None) -> torch.Tensor:
    """phy.cpp:178-239: estimate on raw samples, fused down-chirp, sync word from
    symbols 0/1 into ws.sync_word, returns the total-2 data symbols."""
    if ws is None or iq is None:
        _err(_capi.LORA_EINVAL, "null argument")
    res = ws.plan.run(iq)  # raises on size not a multiple of N*osr / < 2 symbols
    if symbol_cap is not None and res.symbols.shape[-1] > symbol_cap:
        _err(_capi.LORA_ERANGE, "symbol buffer too small")
    single = iq.dim() == 1
    ws.metrics.cfo = res.cfo[0].item() if single else res.cfo
    ws.metrics.time_offset = res.time_offset[0].item() if single else res.time_offset
    ws.sync_word = int(res.sync[0]) if single else res.sync
    return res.symbols[0] if single else res.symbols


def estimate_offsets(ws: lora_workspace, samples: torch.Tensor) -> None:
    """phy.cpp:78-145: results into ws.metrics (untouched if no whole symbol)."""
    x = samples if samples.dim() == 2 else samples.unsqueeze(0)
    F = x.shape[0]
    cfo = torch.full((F,), float(ws.metrics.cfo) if not torch.is_tensor(ws.metrics.cfo) else 0.0,
                     dtype=torch.float32, device=x.device)
    toff = torch.full((F,), float(ws.metrics.time_offset) if not torch.is_tensor(ws.metrics.time_offset)
                      else 0.0, dtype=torch.float32, device=x.device)
    ws.plan.estimate_offsets(x, cfo, toff)
    if samples.dim() == 1:
        ws.metrics.cfo, ws.metrics.time_offset = cfo[0].item(), toff[0].item()
    else:
        ws.metrics.cfo, ws.metrics.time_offset = cfo, toff


def compensate_offsets(ws: lora_workspace, samples: torch.Tensor) -> None:
    """phy.cpp:147-176, in place (like the reference) using ws.metrics."""
    x = samples if samples.dim() == 2 else samples.unsqueeze(0)
    F = x.shape[0]
    cfo = torch.as_tensor(ws.metrics.cfo, dtype=torch.float32, device=x.device).reshape(-1).expand(F)
    to = torch.as_tensor(ws.metrics.time_offset, dtype=torch.float32, device=x.device).reshape(-1).expand(F)
    out = _compensate(x, ws.sf, ws.osr, cfo.contiguous(), to.contiguous())
    x.copy_(out)


def get_last_metrics(ws: lora_workspace) -> Optional[lora_metrics]:
    """phy.cpp:258-261."""
    return None if ws is None else ws.metrics


# ---------------------------------------------------------------------------
# Legacy API (phy.hpp:170-215)
# ---------------------------------------------------------------------------


@dataclass
class lora_demod_workspace:  # noqa: N801
    sf: int
    window: str
    plan_cache: dict = field(default_factory=dict)
    metrics: lora_metrics = field(default_factory=lora_metrics)
    dechirp: bool = False
    device: object = None


def lora_demod_init(sf: int, window: str = "none", dechirp: bool = False, device=None) -> lora_demod_workspace:
    """LoRaDemod.cpp:10-47.  ``dechirp=True`` also fuses the caller-side dechirp loop
    of the reference's tests (e2e_chain_test.cpp:85-93)."""
    if not 2 <= int(sf) <= 12 or window not in ("none", "hann"):
        _err(_capi.LORA_EINVAL, "invalid sf/window")
    return lora_demod_workspace(int(sf), window, dechirp=bool(dechirp), device=device)


def lora_demod_free(ws: lora_demod_workspace) -> None:
    for p in ws.plan_cache.values():
        p.close()
    ws.plan_cache.clear()


def lora_demodulate(ws: lora_demod_workspace, samples: torch.Tensor, osr: int = 1,
                    bw: int = 125000) -> Tuple[torch.Tensor, torch.Tensor]:
    """LoRaDemod.cpp:49-195 for one frame ``[L]`` or a batch ``[F, L]``: returns
    (symbols, sync) and fills ws.metrics (cfo, time_offset)."""
    key = (int(osr) or 1, int(bw))
    plan = ws.plan_cache.get(key)
    if plan is None:
        plan = DemodPlan(ws.sf, key[0], key[1], ws.window, dechirp=ws.dechirp, mode="legacy",
                         device=ws.device)
        ws.plan_cache[key] = plan
    res = plan.run(samples)
    single = samples.dim() == 1
    ws.metrics.cfo = res.cfo[0].item() if single else res.cfo
    ws.metrics.time_offset = res.time_offset[0].item() if single else res.time_offset
    return (res.symbols[0], res.sync[0]) if single else (res.symbols, res.sync)


def lora_modulate(symbols, sf: int, osr: int = 1, bw: int = 125000, amplitude: float = 1.0,
                  sync: int = 0x12, device=None) -> torch.Tensor:
    """LoRaMod.cpp:8-43."""
    s = symbols if isinstance(symbols, torch.Tensor) else torch.as_tensor(np.asarray(symbols, np.int32))
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return _modulate(s.to(dev), sf, osr, bw, amplitude, sync)


def lora_encode(payload: bytes, sf: int = 7) -> np.ndarray:
    """LoRaEncoder.cpp:8-19 (sf unused by the reference's encoder)."""
    return codes.lora_encode(payload)


def lora_decode(symbols) -> bytes:
    """LoRaDecoder.cpp:8-19."""
    if isinstance(symbols, torch.Tensor):
        symbols = symbols.cpu().numpy()
    return codes.lora_decode(np.asarray(symbols)).tobytes()
