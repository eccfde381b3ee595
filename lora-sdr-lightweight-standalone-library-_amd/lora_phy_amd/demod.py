"""GPU demodulation: plan wrapper over lora_demod_batch and the LoRaDemod block.

The plan mirrors ``lora_demod_workspace`` (include/lora_phy/phy.hpp:170-185): it is
created once per (sf, osr, bw, window, dechirp, mode, device) and holds only constant
tables on the device.  IQ buffers are torch.complex64 CUDA tensors owned by the
caller; outputs are allocated with torch's caching allocator (no hipMalloc per call).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import threading
from dataclasses import dataclass
from typing import Optional

import torch

from . import _capi

_WINDOWS = {"none": _capi.LORA_WINDOW_NONE, "hann": _capi.LORA_WINDOW_HANN,
            None: _capi.LORA_WINDOW_NONE, 0: _capi.LORA_WINDOW_NONE, 1: _capi.LORA_WINDOW_HANN}
_MODES = {"legacy": _capi.LORA_MODE_LEGACY, "api": _capi.LORA_MODE_API, "raw": _capi.LORA_MODE_RAW}
# include/lora_mi355x.h LORA_PRECISION_*: "exact" = bit-identical to the reference
# (default); "fast" = hardware sin/cos for the per-sample CFO rotation (stated tolerance).
_PRECISIONS = {"exact": 0, "fast": 1}


@dataclass
class DemodResult:
    """Per-frame results of one batched call (all tensors on the plan's device)."""

    symbols: torch.Tensor      # [F, S] uint16   (LoRaDemod.cpp:165-174)
    sync: torch.Tensor         # [F] uint8       (LoRaDemod.cpp:177-192)
    cfo: torch.Tensor          # [F] float32     (lora_metrics.cfo)
    time_offset: torch.Tensor  # [F] float32     (lora_metrics.time_offset)
    max_amp: torch.Tensor      # [F] float32     (LoRaDemod.cpp:59-67; 0 in API mode)


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_cuda(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor; the product path has no "
                        "CPU fallback")


def _check_buf(t: torch.Tensor, name: str, dtype: torch.dtype, device: torch.device, numel: int) -> None:
    """Everything the C library cannot check about a raw pointer: a wrong device, dtype,
    stride or length would be a GPU memory fault or silent corruption, not an error."""
    _require_cuda(t, name)
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, the plan is on {device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if numel > 0 and (not t.is_contiguous() or t.numel() < numel):
        raise ValueError(f"{name} must be contiguous with >= {numel} elements "
                         f"(got {t.numel()}, contiguous={t.is_contiguous()})")


def _check_iq(iq: torch.Tensor, device: torch.device) -> torch.Tensor:
    _require_cuda(iq, "iq")
    if iq.device != device:
        raise ValueError(f"iq is on {iq.device}, the plan is on {device}")
    if iq.dtype != torch.complex64:
        raise TypeError("iq must be complex64 (interleaved fp32 I/Q)")
    if iq.dim() == 1:
        iq = iq.unsqueeze(0)
    if iq.dim() != 2 or (iq.shape[1] > 1 and iq.stride(1) != 1) or (iq.shape[0] > 1 and iq.stride(0) < iq.shape[1]):
        raise ValueError("iq must be [frames, samples] with unit sample stride and non-overlapping rows")
    return iq


class DemodPlan:
    """A device plan for one demodulator configuration (lora_demod_init equivalent)."""

    def __init__(self, sf: int, osr: int = 1, bw: int = 125000, window="none",
                 dechirp: bool = False, mode: str = "legacy", device=None, precision: str = "exact",
                 pipeline: Optional[str] = None):
        """``pipeline``: "spec" = the speculative single-read pipeline wherever it covers the
        configuration, "split" = always the three-launch exact path; None = the enclosing
        ``spec_pipeline`` block's choice on this thread, else the library default (spec,
        unless LORA_MI355X_SPEC=0 was set when the plan was created)."""
        if not torch.cuda.is_available():
            raise RuntimeError("lora_phy_amd needs a HIP GPU (torch.cuda.is_available() is False)")
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                           torch.device(device).index or 0)
        self.device = dev
        self.sf, self.osr, self.bw = int(sf), int(osr) if osr else 1, int(bw)
        self.N = 1 << self.sf
        self.step = self.N * self.osr
        self.window = window
        self.dechirp = bool(dechirp)
        self.mode = mode
        if precision not in _PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}")
        self.precision = precision
        self._lib = _capi.lib()
        prm = _capi.DemodParams(self.sf, self.osr, self.bw, _WINDOWS[window], int(self.dechirp),
                                _MODES[mode], dev.index, _PRECISIONS[precision])
        h = C.c_void_p()
        _capi.check(self._lib.lora_demod_plan_create(C.byref(prm), C.byref(h)))
        self._h = h
        if pipeline is None:
            pipeline = getattr(_PIPELINE, "choice", None)
        if pipeline is not None:
            if pipeline not in ("spec", "split"):
                raise ValueError('pipeline must be "spec", "split" or None')
            _capi.check(self._lib.lora_demod_plan_set_pipeline(h, int(pipeline == "spec")))
        self.pipeline = pipeline
        # Workspaces per stream (two streams never share frame maxima / FrameParams);
        # ones used while a HIP graph was being captured are kept for the plan's lifetime,
        # since the graph replays with their addresses.
        self._ws: dict = {}
        self._ws_captured: list = []

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.lora_demod_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def symbols_per_frame(self, frame_len: int) -> int:
        return _capi.check(self._lib.lora_demod_symbols_per_frame(self._h, int(frame_len)))

    def last_kernels(self) -> set:
        """Kernels the last run() launched: {"spec", "estimate", "demod"} for the speculative
        single-read pipeline, {"frame_max", "estimate", "demod"} for the three-launch path
        (+"generic", "frame_max_wave")."""
        m = self._lib.lora_demod_last_kernels(self._h)
        return {k for k, b in _capi.KERNEL_BITS.items() if m & b}

    def spec_recomputed(self) -> int:
        """Data symbols the speculative pipeline has recomputed exactly on this plan (their
        certification margin was too small); synchronises the device."""
        return _capi.check(self._lib.lora_demod_spec_recomputed(self._h))

    def _workspace(self, frames: int, frame_len: int) -> torch.Tensor:
        need = self._lib.lora_demod_workspace_bytes(self._h, int(frames), int(frame_len))
        key = _stream_handle(self.device)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need:
            # allocated on (and stream-ordered with) the current stream, so dropping the
            # smaller one is safe for work already queued on it
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
            if torch.cuda.is_current_stream_capturing():
                self._ws_captured.append(ws)
        return ws

    def run(self, iq: torch.Tensor, out: Optional[DemodResult] = None) -> DemodResult:
        """Demodulate a [F, L] (or [L]) complex64 CUDA tensor; one frame per row."""
        iq = _check_iq(iq, self.device)
        F, L = iq.shape
        S = self.symbols_per_frame(L)
        dev = self.device
        if out is None:
            out = DemodResult(
                symbols=torch.empty((F, max(S, 0)), dtype=torch.uint16, device=dev),
                sync=torch.empty(F, dtype=torch.uint8, device=dev),
                cfo=torch.empty(F, dtype=torch.float32, device=dev),
                time_offset=torch.empty(F, dtype=torch.float32, device=dev),
                max_amp=torch.zeros(F, dtype=torch.float32, device=dev))
        else:
            if S > 0:
                _require_cuda(out.symbols, "out.symbols")
                if (out.symbols.dtype != torch.uint16 or out.symbols.device != dev or out.symbols.dim() != 2
                        or out.symbols.shape[0] < F or out.symbols.shape[1] < S or out.symbols.stride(1) != 1):
                    raise ValueError(f"out.symbols must be a uint16 [>={F}, >={S}] tensor on {dev}")
            for name, dt in (("sync", torch.uint8), ("cfo", torch.float32), ("time_offset", torch.float32),
                             ("max_amp", torch.float32)):
                _check_buf(getattr(out, name), "out." + name, dt, dev, F)
        ws = self._workspace(F, L)
        o = _capi.DemodOutputs(out.symbols.data_ptr() if S > 0 else None,
                               out.symbols.stride(0) if S > 0 else 0,
                               out.sync.data_ptr(), out.cfo.data_ptr(), out.time_offset.data_ptr(),
                               out.max_amp.data_ptr())
        stride = iq.stride(0) if F > 1 else L
        _capi.check(self._lib.lora_demod_batch(self._h, iq.data_ptr(), F, L, stride, C.byref(o),
                                               ws.data_ptr(), ws.numel(), _stream_handle(dev)))
        return out

    def estimate_offsets(self, iq: torch.Tensor, cfo: torch.Tensor, time_offset: torch.Tensor) -> int:
        """phy.cpp:78-145 over every whole symbol of each frame (raw samples)."""
        iq = _check_iq(iq, self.device)
        F, L = iq.shape
        _check_buf(cfo, "cfo", torch.float32, self.device, F)
        _check_buf(time_offset, "time_offset", torch.float32, self.device, F)
        stride = iq.stride(0) if F > 1 else L
        return _capi.check(self._lib.lora_estimate_offsets_batch(
            self._h, iq.data_ptr(), F, L, stride, cfo.data_ptr(), time_offset.data_ptr(),
            _stream_handle(self.device)))


def compensate_offsets(iq: torch.Tensor, sf: int, osr: int, cfo: torch.Tensor,
                       time_offset: torch.Tensor) -> torch.Tensor:
    """phy.cpp:147-176 for a [F, L] batch; returns a new tensor (out of place)."""
    _require_cuda(iq, "iq")
    squeeze = iq.dim() == 1
    x = _check_iq((iq.unsqueeze(0) if squeeze else iq).contiguous(), iq.device)
    F, L = x.shape
    _check_buf(cfo, "cfo", torch.float32, x.device, F)
    _check_buf(time_offset, "time_offset", torch.float32, x.device, F)
    out = torch.empty_like(x)
    lib = _capi.lib()
    _capi.check(lib.lora_compensate_offsets_batch(
        int(sf), int(osr), x.data_ptr(), F, L, L, cfo.contiguous().data_ptr(),
        time_offset.contiguous().data_ptr(), x.device.index, _stream_handle(x.device),
        out.data_ptr()))
    return out[0] if squeeze else out


class LoRaDemod:
    """Block-style demodulator mirroring the Pothos ``/lora/lora_demod`` surface
    (examples/lora_simulation.pth:427-445: sf, sync, thresh, mtu) plus the library
    parameters bw / cr / osr / window (phy.hpp:51-58).

    ``work(iq)`` consumes one frame (or a [F, L] batch) of raw IQ and returns the
    symbol stream; per-frame metrics of the last call are in ``last``.

    The Pothos-only parameters (the upstream block is an empty submodule in the
    reference, so their semantics are not pinned by any reference code):
      * ``mtu`` - the most data symbols one frame (packet) yields: ``work`` returns at
        most ``mtu`` symbols per frame (the first ones); ``last`` keeps them all.
      * ``thresh`` - a detection threshold in dB.  The reference library path
        (LoRaDemod.cpp:49-195) has no detection gate, so no gate is applied; only the
        graph's value -30.0 (examples/lora_simulation.pth:440) is accepted, and any
        other value raises instead of being silently ignored.
    """

    THRESH_DEFAULT = -30.0

    def __init__(self, sf: int, sync: int = 0x12, thresh: float = -30.0, mtu: int = 256,
                 bw: int = 125000, cr: int = 1, osr: int = 1, window="none",
                 dechirp: bool = True, mode: str = "legacy", device=None, precision: str = "exact"):
        if float(thresh) != self.THRESH_DEFAULT:
            raise ValueError(f"thresh={thresh}: no detection gate is defined by the reference path; "
                             f"only the default {self.THRESH_DEFAULT} is accepted")
        if int(mtu) < 1:
            raise ValueError("mtu must be >= 1 symbol")
        self.sf, self.sync, self.thresh, self.mtu = int(sf), int(sync) & 0xFF, float(thresh), int(mtu)
        self.bw, self.cr, self.osr = int(bw), int(cr), int(osr) if osr else 1
        self.plan = DemodPlan(sf, self.osr, bw, window, dechirp, mode, device, precision)
        self.last: Optional[DemodResult] = None

    def work(self, iq: torch.Tensor) -> torch.Tensor:
        res = self.plan.run(iq)
        self.last = res
        syms = res.symbols[:, :self.mtu]
        return syms[0] if iq.dim() == 1 else syms

    def work_frames(self, iq: torch.Tensor) -> DemodResult:
        self.last = self.plan.run(iq)
        return self.last

    def sync_ok(self) -> torch.Tensor:
        """Per-frame flag: recovered sync word equals the configured one."""
        if self.last is None:
            raise RuntimeError("work() has not run")
        return self.last.sync == self.sync


_PIPELINE = threading.local()


@contextlib.contextmanager
def spec_pipeline(enabled: bool = True):
    """Plans created inside this block ON THIS THREAD use the speculative single-read pipeline
    (``enabled=True``, whatever LORA_MI355X_SPEC says) or the three-launch exact path (frame
    max, estimate, demod: ``enabled=False``) - ``DemodPlan(pipeline=...)`` with the choice
    filled in.  Nothing process-wide changes (no environment variable is touched), so other
    threads creating plans meanwhile are unaffected; blocks nest."""
    prev = getattr(_PIPELINE, "choice", None)
    _PIPELINE.choice = "spec" if enabled else "split"
    try:
        yield
    finally:
        _PIPELINE.choice = prev
