"""AWGN sweeps with the demodulation on the GPU (BASELINE.json configs[3]).

Two harnesses, both host-driven with one batched GPU call per SNR point:

``simulate(sf, cr, snr_db, packets, payload_len, up, down)``
    Drop-in for the reference's ``tests/awgn_sweep.py:simulate`` (same signature, same
    ``np.random`` draw order: per packet ``randint(0, 256, L)`` then per symbol
    ``normal(N)`` for I and ``normal(N)`` for Q, awgn_sweep.py:251-267).  The channel
    and the dechirp ``r * down`` are computed in float64 exactly as the script does;
    the per-symbol FFT + argmax runs on the GPU in LORA_MODE_RAW (fp32 kissfft order)
    instead of numpy's float64 FFT.  FEC (CR 4/5 parity, 4/8 Hamming) and the bit <->
    symbol packing restate the script's host code.  Decisions can differ from the
    script's only where two bins' magnitudes tie to within fp32 rounding.

``sweep_chain(sf, snr_dbs, frames, payload_len, seed, cfo_bins=0.0)``
    The library's own chain: ``lora_encode`` (Hamming 8/4 per nibble) -> GPU
    ``lora_modulate`` (2 sync up-chirps + payload) -> complex AWGN with
    sigma = 10^(-SNR/20) (awgn_sweep_gtest.cpp:76-80) and an optional CFO phase ramp
    ``2*pi*cfo_bins*(n mod N)/N`` (lora_phy_vector_generate.cpp:102-108) -> GPU LEGACY
    ``lora_demodulate`` with the caller-side dechirp, i.e. normalisation + the 2-sync-
    symbol CFO/timing estimate + per-symbol CFO rotation (the reference's "preamble
    detect + CFO correct", LoRaDemod.cpp:79-157) -> ``lora_decode``.  Reports SER, BER,
    PER and returns the noisy IQ so callers can check the GPU against the oracle.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import codes
from .demod import DemodPlan
from .mod import modulate

# --------------------------------------------------------------------------------------
# tests/awgn_sweep.py host pieces (restated; pinned by tests/golden/awgn_sweep.json)
# --------------------------------------------------------------------------------------

_WIDTH = {"4/5": 5, "4/8": 8}


def encode_payload(payload: bytes, cr: str) -> np.ndarray:
    """Bits (uint8, LSB-first per codeword) of the high/low nibbles of every byte,
    CR 4/5 = parity54, CR 4/8 = Hamming 8/4 (awgn_sweep.py:139-158)."""
    if cr not in _WIDTH:
        raise ValueError(f"Unsupported coding rate: {cr}")
    b = np.frombuffer(bytes(payload), np.uint8).astype(np.int64)
    nib = np.stack([b >> 4, b & 0xF], 1).reshape(-1)
    cw = (codes.ENC_P54 if cr == "4/5" else codes.ENC_H84)[nib].astype(np.int64)
    w = _WIDTH[cr]
    return ((cw[:, None] >> np.arange(w)) & 1).astype(np.uint8).reshape(-1)


def decode_payload(bits: np.ndarray, cr: str, num_bytes: int) -> np.ndarray:
    """Inverse of encode_payload (CR 4/5: data nibble as received; CR 4/8: Hamming 8/4
    correction of single-bit errors), awgn_sweep.py:161-189."""
    w = _WIDTH[cr]
    b = np.asarray(bits, np.int64)[: num_bytes * 2 * w].reshape(num_bytes * 2, w)
    cw = (b << np.arange(w)).sum(1)
    nib = (cw & 0xF) if cr == "4/5" else codes.decode_hamming84(cw)[0].astype(np.int64)
    return ((nib[0::2] << 4) | nib[1::2]).astype(np.uint8)


def bits_to_symbols(bits: np.ndarray, sf: int) -> np.ndarray:
    """Pack bits LSB-first into sf-bit symbols, zero padded (awgn_sweep.py:197-207)."""
    b = np.asarray(bits, np.int64)
    pad = (-len(b)) % sf
    b = np.concatenate([b, np.zeros(pad, np.int64)]).reshape(-1, sf)
    return (b << np.arange(sf)).sum(1)


def symbols_to_bits(symbols, sf: int, bit_len: int) -> np.ndarray:
    """awgn_sweep.py:210-217."""
    s = np.asarray(symbols, np.int64)
    return ((s[:, None] >> np.arange(sf)) & 1).reshape(-1)[:bit_len].astype(np.uint8)


def make_chirps(sf: int):
    """awgn_sweep.py:225-234: float64 up/down chirps of the Python model."""
    N = 1 << sf
    n = np.arange(N, dtype=float)
    accum = np.cumsum(-math.pi + (2 * math.pi * n) / N)
    up = np.exp(1j * accum)
    return up, np.conj(up)


def simulate(sf: int, cr: str, snr_db: float, packets: int, payload_len: int, up: np.ndarray,
             down: np.ndarray, device=None, return_symbols: bool = False):
    """GPU-demodulated twin of awgn_sweep.py:simulate -> (ber, per)."""
    N = len(up)
    n = np.arange(N)
    sigma = 10 ** (-snr_db / 20.0)
    rows, meta = [], []
    for _ in range(packets):
        payload = np.random.randint(0, 256, payload_len, dtype=np.uint8)
        tx_bits = encode_payload(payload.tobytes(), cr)
        syms = bits_to_symbols(tx_bits, sf)
        for sym in syms:
            shift = np.exp(1j * 2 * math.pi * int(sym) * n / N)
            tx = up * shift
            noise = np.random.normal(size=N) + 1j * np.random.normal(size=N)
            noise *= sigma / math.sqrt(2.0)
            rows.append((tx + noise) * down)
        meta.append((payload, tx_bits, len(syms)))
    iq = torch.from_numpy(np.asarray(rows).astype(np.complex64))
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    plan = DemodPlan(sf, 1, 125000, "none", dechirp=False, mode="raw", device=dev)
    rx = plan.run(iq.to(dev)).symbols[:, 0].to(torch.int64).cpu().numpy()
    bit_errors = packet_errors = total_bits = 0
    off = 0
    for payload, tx_bits, ns in meta:
        rx_bits = symbols_to_bits(rx[off:off + ns], sf, len(tx_bits))
        off += ns
        rx_payload = decode_payload(rx_bits, cr, payload_len)
        diff = np.bitwise_xor(payload, rx_payload)
        bit_errors += int(np.unpackbits(diff).sum())
        total_bits += payload_len * 8
        packet_errors += int(diff.any())
    ber = bit_errors / total_bits if total_bits else 0.0
    per = packet_errors / packets if packets else 0.0
    if return_symbols:
        return ber, per, rx, np.asarray(rows)
    return ber, per


# --------------------------------------------------------------------------------------
# The library chain under AWGN (+ optional CFO)
# --------------------------------------------------------------------------------------

def sweep_chain(sf: int, snr_dbs: Sequence[float], frames: int = 1000, payload_len: int = 16,
                seed: int = 1234, cfo_bins: float = 0.0, osr: int = 1, device=None,
                keep_iq: bool = False, exact_check: bool = False) -> List[Dict]:
    """SER / BER / PER of encode -> modulate -> AWGN (+CFO) -> LEGACY demod -> decode.

    exact_check: also run every point through the three-launch exact path (the oracle-pinned
    kernels, LORA_MI355X_SPEC=0) and count the frames whose symbols, sync word or cfo /
    time_offset bits differ from the default (speculative, certified) pipeline's."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    N = 1 << sf
    rng = np.random.default_rng(seed)
    payloads = rng.integers(0, 256, (frames, payload_len)).astype(np.uint8)
    tx = np.stack([codes.lora_encode(p.tobytes()) for p in payloads]).astype(np.int32)
    clean = modulate(torch.from_numpy(tx).to(dev), sf, osr)
    L = clean.shape[1]
    if cfo_bins:
        nn = torch.arange(L, device=dev, dtype=torch.float64) % (N * osr)
        ph = 2.0 * math.pi * cfo_bins * nn / (N * osr)
        clean = (clean.to(torch.complex128) * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
    plan = DemodPlan(sf, osr, 125000, "none", dechirp=True, mode="legacy", device=dev)
    xplan = None
    if exact_check:
        from .demod import spec_pipeline

        with spec_pipeline(False):
            xplan = DemodPlan(sf, osr, 125000, "none", dechirp=True, mode="legacy", device=dev)
    gen = torch.Generator(device=dev).manual_seed(seed + 1)
    out = []
    for snr in snr_dbs:
        sigma = 10.0 ** (-snr / 20.0) / math.sqrt(2.0)
        noise = torch.randn((frames, L, 2), generator=gen, device=dev) * sigma
        iq = clean + torch.view_as_complex(noise)
        fixed0 = plan.spec_recomputed()
        res = plan.run(iq)
        rx = res.symbols.to(torch.int64).cpu().numpy()
        dec = codes.lora_decode(rx)
        # the modulator sends each 8-bit Hamming codeword modulo N (SF7 drops bit 7,
        # which the decoder then corrects), so symbol errors count against tx mod N
        ser = float((rx != (tx % N)).mean())
        diff = np.bitwise_xor(dec, payloads)
        rec = {"sf": sf, "snr_db": float(snr), "frames": frames, "ser": ser,
               "ber": float(np.unpackbits(diff).mean()), "per": float(diff.any(1).mean()),
               "sync_ok": float((res.sync == 0x12).float().mean()), "cfo_bins": cfo_bins,
               "recomputed_symbols": int(plan.spec_recomputed() - fixed0)}
        if xplan is not None:
            rx_ = xplan.run(iq)
            bad = ((res.symbols != rx_.symbols).any(1) | (res.sync != rx_.sync)
                   | (res.cfo.view(torch.int32) != rx_.cfo.view(torch.int32))
                   | (res.time_offset.view(torch.int32) != rx_.time_offset.view(torch.int32)))
            rec["exact_path_frames_compared"] = frames
            rec["exact_path_frame_mismatches"] = int(bad.sum())
        if keep_iq:
            rec["iq"] = iq
            rec["result"] = res
        out.append(rec)
    return out
