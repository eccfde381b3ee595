"""Shared, reference-free helpers for the golden fixtures (tests/golden/).

tests/golden/make_golden.py uses these with the reference build (oracle/_ref) as the
modulator; the tests use them with the restatement (oracle/liblora_oracle.so, pinned
bit-exact to the reference) to regenerate the same seeded inputs, checked by sha256.
`M` is any object with gen_chirp() and lora_modulate() (oracle.pyoracle._Common).
"""
from __future__ import annotations

import hashlib

import numpy as np


def sha(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def f32bits(v) -> int:
    return int(np.float32(v).view(np.uint32))


def down_table(M, sf: int, osr: int, bw_scale: float = 1.0) -> np.ndarray:
    """genChirp(N, osr, N*osr, 0, down) as e2e_chain_test.cpp:85-87 builds it."""
    N = 1 << sf
    tab, _ = M.gen_chirp(N, osr, N * osr, 0.0, True, 1.0, 0.0, bw_scale)
    return tab


def cmul_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """std::complex<float> product, each fp32 op rounded separately (no FMA)."""
    ar, ai = a.real.astype(np.float32), a.imag.astype(np.float32)
    br, bi = b.real.astype(np.float32), b.imag.astype(np.float32)
    out = np.empty(a.shape, np.complex64)
    out.real = ar * br - ai * bi
    out.imag = ar * bi + ai * br
    return out


def dechirp(M, x: np.ndarray, sf: int, osr: int = 1, bw_scale: float = 1.0) -> np.ndarray:
    """The caller-side dechirp loop (e2e_chain_test.cpp:88-93) over a whole frame."""
    tab = down_table(M, sf, osr, bw_scale)
    reps = -(-len(x) // len(tab))
    return cmul_f32(x, np.tile(tab, reps)[: len(x)])


# Seeded synthetic frames exercising every branch of lora_demodulate (LoRaDemod.cpp:
# 49-195): normalisation on/off, osr phase search, both windows, t_off shifts of both
# signs, odd lengths, one-symbol and zero-symbol frames, every SF.
STRESS = [  # (sf, osr, hann, dechirp, F, symbols per frame, extra samples, kind)
    (2, 1, False, False, 6, 9, 1, "noise"),
    (3, 4, True, False, 4, 5, 3, "mod"),
    (4, 2, False, True, 4, 12, 0, "mod"),
    (5, 1, False, True, 4, 30, 0, "mod"),
    (6, 2, False, False, 4, 3, 0, "noise"),
    (7, 1, False, True, 8, 66, 0, "mod"),
    (7, 2, True, True, 3, 11, 7, "mod"),
    (7, 1, False, False, 3, 1, 20, "noise"),
    (7, 1, False, False, 2, 0, 50, "noise"),
    (8, 1, True, False, 3, 20, 0, "mod"),
    (9, 3, True, True, 2, 9, 5, "mod"),
    (10, 1, False, False, 2, 12, 0, "noise"),
    (11, 2, False, True, 2, 7, 100, "mod"),
    (12, 1, False, True, 2, 10, 0, "mod"),
    (12, 1, True, False, 1, 6, 17, "noise"),
]


def stress_input(M, case, seed: int) -> np.ndarray:
    """Deterministic inputs (numpy PCG64); the 'mod' kind is the reference modulator
    plus scaled AWGN."""
    sf, osr, hann, dech, F, nsym, extra, kind = case
    rng = np.random.default_rng(seed)
    N = 1 << sf
    L = nsym * N * osr + extra
    rows = []
    for _ in range(F):
        if kind == "noise":
            amp = np.float32(rng.uniform(0.05, 3.0))
            x = ((rng.standard_normal(L) + 1j * rng.standard_normal(L)) * amp).astype(np.complex64)
        else:
            k = L // (N * osr) + 1
            syms = rng.integers(0, N, max(k - 2, 0)).astype(np.uint16)
            x = M.lora_modulate(syms, sf, osr, 125000, 1.0, int(rng.integers(0, 256)))
            x = np.concatenate([x, np.zeros(max(L - len(x), 0), np.complex64)])[:L]
            sig = float(rng.choice([0.0, 0.05, 0.3, 1.0, 3.0]))
            if sig > 0:
                x = (x + sig * (rng.standard_normal(L) + 1j * rng.standard_normal(L))).astype(np.complex64)
        rows.append(x)
    return np.stack(rows) if rows else np.zeros((0, L), np.complex64)


