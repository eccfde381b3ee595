"""Host-side LoRa coding chain (numpy), bit-exact with include/lora_phy/LoRaCodes.hpp.

Per the north star these stay on the host: they are byte/bit work on a few bytes per
packet, far off the demod hot path.  Table-driven and vectorised over arrays so a
batch of demodulated frames [F, S] decodes in one call.  Parity with the reference's
own functions is checked in tests/test_codes.py (compiled reference in the build
container) and against the committed golden vectors.
"""
from __future__ import annotations

import numpy as np

# ---------------------------------------------------------------------------
# Hamming 8/4 and 7/4, parity 5/4 and 6/4 (LoRaCodes.hpp:229-371)
# ---------------------------------------------------------------------------


def _bits(x, n):
    return [(x >> i) & 1 for i in range(n)]


def _enc_h84_scalar(x: int) -> int:  # LoRaCodes.hpp:229-242
    d0, d1, d2, d3 = _bits(x, 4)
    b = x & 0xF
    b |= (d0 ^ d1 ^ d2) << 4
    b |= (d1 ^ d2 ^ d3) << 5
    b |= (d0 ^ d1 ^ d3) << 6
    b |= (d0 ^ d2 ^ d3) << 7
    return b


def _dec_h84_scalar(b: int):  # LoRaCodes.hpp:250-281 -> (nibble, error, bad)
    b0, b1, b2, b3, b4, b5, b6, b7 = _bits(b, 8)
    p = (b0 ^ b1 ^ b2 ^ b4) | ((b1 ^ b2 ^ b3 ^ b5) << 1) | ((b0 ^ b1 ^ b3 ^ b6) << 2) | \
        ((b0 ^ b2 ^ b3 ^ b7) << 3)
    fix = {0xD: 1, 0x7: 2, 0xB: 4, 0xE: 8}
    if p in fix:
        return (b ^ fix[p]) & 0xF, p != 0, False
    if p in (0x0, 0x1, 0x2, 0x4, 0x8):
        return b & 0xF, p != 0, False
    return b & 0xF, True, True


def _enc_h74_scalar(x: int) -> int:  # LoRaCodes.hpp:287-299
    d0, d1, d2, d3 = _bits(x, 4)
    b = x & 0xF
    b |= (d0 ^ d1 ^ d2) << 4
    b |= (d1 ^ d2 ^ d3) << 5
    b |= (d0 ^ d1 ^ d3) << 6
    return b


def _dec_h74_scalar(b: int):  # LoRaCodes.hpp:306-334 -> (nibble, error)
    b0, b1, b2, b3, b4, b5, b6, _ = _bits(b, 8)
    p = (b0 ^ b1 ^ b2 ^ b4) | ((b1 ^ b2 ^ b3 ^ b5) << 1) | ((b0 ^ b1 ^ b3 ^ b6) << 2)
    fix = {0x5: 1, 0x7: 2, 0x3: 4, 0x6: 8}
    if p in fix:
        return (b ^ fix[p]) & 0xF, p != 0
    return b & 0xF, p != 0


def _chk_p54_scalar(b: int):  # LoRaCodes.hpp:340-345
    x = b ^ (b >> 2)
    x = x ^ (x >> 1) ^ (b >> 4)
    return b & 0xF, bool(x & 1)


def _enc_p54_scalar(b: int) -> int:  # LoRaCodes.hpp:347-351
    x = b ^ (b >> 2)
    x = x ^ (x >> 1)
    return (b & 0xF) | ((x << 4) & 0x10)


def _chk_p64_scalar(b: int):  # LoRaCodes.hpp:357-365
    x = b ^ (b >> 1) ^ (b >> 2)
    y = x ^ b ^ (b >> 3)
    x ^= b >> 4
    y ^= b >> 5
    return b & 0xF, bool((x | y) & 1)


def _enc_p64_scalar(b: int) -> int:  # LoRaCodes.hpp:367-371
    x = b ^ (b >> 1) ^ (b >> 2)
    y = x ^ b ^ (b >> 3)
    return ((x & 1) << 4) | ((y & 1) << 5) | (b & 0xF)


# 256-entry tables indexed by the low byte (the reference casts symbols to uint8).
ENC_H84 = np.array([_enc_h84_scalar(x) for x in range(256)], np.uint8)
_D84 = [_dec_h84_scalar(b) for b in range(256)]
DEC_H84 = np.array([d[0] for d in _D84], np.uint8)
DEC_H84_ERR = np.array([d[1] for d in _D84], bool)
DEC_H84_BAD = np.array([d[2] for d in _D84], bool)
ENC_H74 = np.array([_enc_h74_scalar(x) for x in range(256)], np.uint8)
_D74 = [_dec_h74_scalar(b) for b in range(256)]
DEC_H74 = np.array([d[0] for d in _D74], np.uint8)
DEC_H74_ERR = np.array([d[1] for d in _D74], bool)
ENC_P54 = np.array([_enc_p54_scalar(x) for x in range(256)], np.uint8)
CHK_P54_ERR = np.array([_chk_p54_scalar(b)[1] for b in range(256)], bool)
ENC_P64 = np.array([_enc_p64_scalar(x) for x in range(256)], np.uint8)
CHK_P64_ERR = np.array([_chk_p64_scalar(b)[1] for b in range(256)], bool)


def encode_hamming84(x):
    return ENC_H84[np.asarray(x, np.int64) & 0xFF]


def decode_hamming84(b):
    """-> (nibbles, error, bad) arrays (LoRaCodes.hpp:250-281)."""
    i = np.asarray(b, np.int64) & 0xFF
    return DEC_H84[i], DEC_H84_ERR[i], DEC_H84_BAD[i]


def encode_hamming74(x):
    return ENC_H74[np.asarray(x, np.int64) & 0xFF]


def decode_hamming74(b):
    i = np.asarray(b, np.int64) & 0xFF
    return DEC_H74[i], DEC_H74_ERR[i]


def encode_parity54(x):
    return ENC_P54[np.asarray(x, np.int64) & 0xFF]


def check_parity54(b):
    i = np.asarray(b, np.int64) & 0xFF
    return (i & 0xF).astype(np.uint8), CHK_P54_ERR[i]


def encode_parity64(x):
    return ENC_P64[np.asarray(x, np.int64) & 0xFF]


def check_parity64(b):
    i = np.asarray(b, np.int64) & 0xFF
    return (i & 0xF).astype(np.uint8), CHK_P64_ERR[i]


# ---------------------------------------------------------------------------
# Gray code (LoRaCodes.hpp:201-222)
# ---------------------------------------------------------------------------


def binary_to_gray16(x):
    x = np.asarray(x).astype(np.uint16)
    return (x ^ (x >> 1)).astype(np.uint16)


def gray_to_binary16(x):
    n = np.asarray(x).astype(np.uint16)
    n = n ^ (n >> 8)
    n = n ^ (n >> 4)
    n = n ^ (n >> 2)
    n = n ^ (n >> 1)
    return n.astype(np.uint16)


# ---------------------------------------------------------------------------
# Checksums / CRC (LoRaCodes.hpp:32-105)
# ---------------------------------------------------------------------------


def checksum8(data) -> int:  # LoRaCodes.hpp:32-41
    acc = 0
    for v in bytes(data):
        acc = ((acc >> 1) + ((acc & 1) << 7)) & 0xFF
        acc = (acc + v) & 0xFF
    return acc


def header_checksum(h) -> int:  # LoRaCodes.hpp:43-67
    h0, h1 = int(h[0]), int(h[1])
    a0, a1, a2, a3 = (h0 >> 4) & 1, (h0 >> 5) & 1, (h0 >> 6) & 1, (h0 >> 7) & 1
    b0, b1, b2, b3 = h0 & 1, (h0 >> 1) & 1, (h0 >> 2) & 1, (h0 >> 3) & 1
    c0, c1, c2, c3 = h1 & 1, (h1 >> 1) & 1, (h1 >> 2) & 1, (h1 >> 3) & 1
    res = (a0 ^ a1 ^ a2 ^ a3) << 4
    res |= (a3 ^ b1 ^ b2 ^ b3 ^ c0) << 3
    res |= (a2 ^ b0 ^ b3 ^ c1 ^ c3) << 2
    res |= (a1 ^ b0 ^ b2 ^ c0 ^ c1 ^ c2) << 1
    res |= a0 ^ b1 ^ c0 ^ c1 ^ c2 ^ c3
    return res


def _crc16sx(crc: int, poly: int) -> int:  # LoRaCodes.hpp:69-79
    for _ in range(8):
        crc = ((crc << 1) ^ poly) if crc & 0x8000 else (crc << 1)
        crc &= 0xFFFF
    return crc


def _xsum8(t: int) -> int:  # LoRaCodes.hpp:81-86
    t ^= t >> 4
    t ^= t >> 2
    t ^= t >> 1
    return t & 1


def sx1272_data_checksum(data) -> int:  # LoRaCodes.hpp:92-105
    res, v, crc = 0, 0xFF, 0
    for b in bytes(data):
        crc = _crc16sx(res, 0x1021)
        v = (_xsum8(v & 0xB8) | (v << 1)) & 0xFF
        res = crc ^ b
    res ^= v
    v = (_xsum8(v & 0xB8) | (v << 1)) & 0xFF
    res ^= (v << 8) & 0xFFFF
    return res & 0xFFFF


# ---------------------------------------------------------------------------
# Whitening (LoRaCodes.hpp:111-189)
# ---------------------------------------------------------------------------


def sx1232_whitening(buf) -> bytes:  # LoRaCodes.hpp:111-137
    out = bytearray(buf)
    msb, lsb = 0x01, 0xFF
    for j in range(len(out)):
        out[j] ^= lsb
        for _ in range(8):
            prev = msb
            msb = (lsb & 1) ^ ((lsb >> 5) & 1)
            lsb = ((lsb >> 1) & 0xFF) | ((prev << 7) & 0x80)
    return bytes(out)


_WHITEN_SEQ = [0x0102291EA751AAFF, 0xD24B050A8D643A17, 0x5B279B671120B8F4, 0x032B37B9F6FB55A2,
               0x994E0F87E95E2D16, 0x7CBCFC7631984C26, 0x281C8E4F0DAEF7F9, 0x1741886EB7733B15]


def sx1272_whitening(buf, bit_ofs: int, rdd: int) -> bytes:  # LoRaCodes.hpp:147-167
    ofs = [6, 4, 2, 0, -360] if rdd == 1 else [6, 4, 2, 0, -112, -114, -302, -34]
    out = bytearray(buf)
    for j in range(len(out) & 0xFFFF):
        x = 0
        for i in range(4 + rdd):
            t = (ofs[i] + j + bit_ofs + 510) % 510
            if (_WHITEN_SEQ[t >> 6] >> (t & 0x3F)) & 1:
                x |= 1 << i
        out[j] ^= x & 0xFF
    return bytes(out)


_M64 = (1 << 64) - 1


def _lfsr_step(r: int) -> int:  # poly 0x1D on interleaved 8-bit lanes
    return ((r >> 8) | ((((r >> 32) ^ (r >> 24) ^ (r >> 16) ^ r) << 56) & _M64)) & _M64


def sx1272_whitening_lfsr(buf, bit_ofs: int, rdd: int) -> bytes:  # LoRaCodes.hpp:176-189
    m = (0xFF >> (4 - rdd)) & 0xFF
    if rdd == 1:
        r = [0x05121100F8ECFEEF, 0xF8ECFEEFEFEFEFEF]
    else:
        r = [0x6572D100E85C2EFF, 0xE85C2EFFFFFFFFFF]
    i = 0
    while i < bit_ofs:
        r[i & 1] = _lfsr_step(r[i & 1])
        i += 1
    out = bytearray(buf)
    for j in range(len(out) & 0xFFFF):
        out[j] ^= (r[i & 1] & m) & 0xFF
        r[i & 1] = _lfsr_step(r[i & 1])
        i += 1
    return bytes(out)


# ---------------------------------------------------------------------------
# Diagonal (de)interleaver (LoRaCodes.hpp:376-432)
# ---------------------------------------------------------------------------


def diagonal_interleave(codewords, ppm: int, rdd: int) -> np.ndarray:
    cw = np.asarray(codewords, np.uint8)
    nblk = len(cw) // ppm
    out = np.zeros(nblk * (4 + rdd), np.uint16)
    for blk in range(nblk):
        for bit in range(4 + rdd):
            sym = 0
            for c in range(ppm):
                src = (c + bit) % ppm
                sym |= ((int(cw[blk * ppm + src]) >> bit) & 1) << c
            out[blk * (4 + rdd) + bit] = sym
    return out


def diagonal_deinterleave(symbols, ppm: int, rdd: int) -> np.ndarray:
    s = np.asarray(symbols, np.uint16)
    nblk = len(s) // (4 + rdd)
    out = np.zeros(nblk * ppm, np.uint8)
    for blk in range(nblk):
        for bit in range(4 + rdd):
            sym = int(s[blk * (4 + rdd) + bit])
            for c in range(ppm):
                dst = (c + bit) % ppm
                out[blk * ppm + dst] |= ((sym >> c) & 1) << bit
    return out


def diagonal_deinterleave2(symbols, ppm: int, rdd: int) -> np.ndarray:
    """LoRaCodes.hpp:415-432 (indexes symbols by row m < PPM within each block)."""
    s = np.asarray(symbols, np.uint16)
    nb = rdd + 4
    nblk = len(s) // nb
    out = np.zeros(nblk * ppm + ppm, np.uint8)
    for x in range(nblk):
        for m in range(ppm):
            i = m
            sym = int(s[x * nb + m])
            for _ in range(ppm):
                out[x * ppm + i] |= ((sym & 1) << m) & 0xFF
                sym >>= 1
                i = 0 if i + 1 == ppm else i + 1
    return out[: nblk * ppm]


# ---------------------------------------------------------------------------
# Library encoder / decoder (LoRaEncoder.cpp:8-19, LoRaDecoder.cpp:8-19)
# ---------------------------------------------------------------------------


def lora_encode(payload) -> np.ndarray:
    """Each byte -> two Hamming 8/4 codewords (high nibble first) used as symbols."""
    b = np.frombuffer(bytes(payload), np.uint8).astype(np.int64)
    out = np.empty(2 * len(b), np.uint16)
    out[0::2] = ENC_H84[b >> 4]
    out[1::2] = ENC_H84[b & 0xF]
    return out


def lora_decode(symbols) -> np.ndarray:
    """Pairs of symbols -> bytes via Hamming 8/4 on the symbols' low byte.

    Works on [S] or [F, S] (row-wise); an odd trailing symbol is ignored.
    """
    s = np.asarray(symbols)
    n = (s.shape[-1] // 2) * 2
    lo8 = s[..., :n].astype(np.int64) & 0xFF
    hi = DEC_H84[lo8[..., 0::2]] & 0xF
    lo = DEC_H84[lo8[..., 1::2]] & 0xF
    return ((hi << 4) | lo).astype(np.uint8)


def decode_with_crc(symbols):
    """phy.cpp:241-256: decode, then SX1272 CRC over payload[2:n-2] vs the last 2 bytes.

    Returns (payload bytes, crc_ok)."""
    out = lora_decode(symbols)
    n = len(out)
    if n >= 4:
        provided = int(out[n - 2]) | (int(out[n - 1]) << 8)
        return out, provided == sx1272_data_checksum(out[2:n - 2].tobytes())
    return out, False


# ---------------------------------------------------------------------------
# The coding chain around the demodulator, per coding rate 4/(4+RDD): nibble codes,
# whitening, diagonal interleave, Gray mapping (LoRaCodes.hpp:176-189, 201-222,
# 229-371, 376-412), in the order of the LoRa-SDR encoder the reference ports (runners/
# lora_phy_vector_generate.cpp:189-223 uses the RDD = 4 case with Hamming 8/4).
# ---------------------------------------------------------------------------


def rdd_of(cr) -> int:
    """'4/5'..'4/8' -> RDD 1..4, '4/4' -> 0; an integer CR index 1..4 is RDD itself."""
    s = str(cr)
    if "/" in s:
        num, den = s.split("/")
        rdd = int(den) - int(num)
    else:
        rdd = int(s)
    if not 0 <= rdd <= 4:
        raise ValueError(f"coding rate {cr!r}: RDD must be 0..4")
    return rdd


def nibble_encode(nibbles, rdd: int) -> np.ndarray:
    """Nibble -> codeword: RDD 4 Hamming 8/4, 3 Hamming 7/4, 2 parity 6/4, 1 parity 5/4,
    0 the bare nibble."""
    x = np.asarray(nibbles, np.int64) & 0xF
    if rdd == 4:
        return encode_hamming84(x)
    if rdd == 3:
        return encode_hamming74(x)
    if rdd == 2:
        return encode_parity64(x)
    if rdd == 1:
        return encode_parity54(x)
    return x.astype(np.uint8)


def nibble_decode(codewords, rdd: int):
    """Codeword -> (nibble, error) with the decoder of nibble_encode's code (Hamming 8/4's
    'bad' flag is folded into error)."""
    b = np.asarray(codewords, np.int64) & 0xFF
    if rdd == 4:
        n, e, bad = decode_hamming84(b)
        return n & 0xF, e | bad
    if rdd == 3:
        n, e = decode_hamming74(b)
        return n & 0xF, e
    if rdd == 2:
        return check_parity64(b)
    if rdd == 1:
        return check_parity54(b)
    return (b & 0xF).astype(np.uint8), np.zeros(b.shape, bool)


def payload_nibbles(payload) -> np.ndarray:
    """Bytes -> nibbles, high nibble first (lora_phy_vector_generate.cpp:196-199)."""
    b = np.frombuffer(bytes(payload), np.uint8).astype(np.int64)
    out = np.empty(2 * len(b), np.int64)
    out[0::2] = b >> 4
    out[1::2] = b & 0xF
    return out


def encode_chain(payload, sf: int, rdd: int):
    """TX side: nibbles -> codewords (padded with zero codewords to a multiple of
    PPM = sf) -> whitening -> diagonal interleave -> Gray.  Returns the stages as a dict
    (codewords, whitened, interleaved, symbols)."""
    cw = nibble_encode(payload_nibbles(payload), rdd).astype(np.uint8)
    n = -(-len(cw) // sf) * sf
    cw = np.concatenate([cw, np.zeros(n - len(cw), np.uint8)])
    wh = np.frombuffer(sx1272_whitening_lfsr(cw.tobytes(), 0, rdd), np.uint8)
    il = diagonal_interleave(wh, sf, rdd)
    return {"codewords": cw, "whitened": wh, "interleaved": il, "symbols": binary_to_gray16(il)}


def decode_chain(symbols, sf: int, rdd: int, nbytes: int):
    """RX side, the inverse of encode_chain: Gray demap -> diagonal deinterleave ->
    de-whitening -> nibble decode -> bytes.  Returns the stages (binary, deinterleaved,
    dewhitened, nibbles, errors, payload)."""
    bi = gray_to_binary16(symbols)
    di = diagonal_deinterleave(bi, sf, rdd)
    dw = np.frombuffer(sx1272_whitening_lfsr(di.tobytes(), 0, rdd), np.uint8)
    nib, err = nibble_decode(dw, rdd)
    nib = nib[: 2 * nbytes].astype(np.int64)
    pay = ((nib[0::2] << 4) | nib[1::2]).astype(np.uint8)
    return {"binary": bi, "deinterleaved": di, "dewhitened": dw, "nibbles": nib.astype(np.uint8),
            "errors": err, "payload": pay}
