"""ctypes bindings for the CPU checker libraries.

*** TEST INFRASTRUCTURE ONLY. *** Importable by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product package (lora_phy_amd) never imports this.

* ``Oracle`` wraps ``oracle/liblora_oracle.so`` - the C++ restatement of the reference
  hot path (oracle/lora_oracle.cpp), available everywhere including the GPU box.
* ``Reference`` wraps ``oracle/_ref/liblora_ref.so`` - the reference library itself,
  compiled from /root/reference by oracle/Makefile in the build container (the built
  .so travels to the GPU box with the repo snapshot); ``Reference.available()`` tells.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liblora_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "liblora_ref.so")

BW_SCALE = {125000: 1.0, 250000: 2.0, 500000: 4.0}

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_c64p = np.ctypeslib.ndpointer(np.complex64, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")


def build_oracle(force: bool = False) -> None:
    """Compile the restatement (and, where /root/reference exists, the reference)."""
    if force or not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])
    if os.path.isdir("/root/reference/src/phy") and (force or not os.path.exists(REF_SO)):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def _c64(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.complex64))


class _Common:
    lib: C.CDLL
    prefix: str

    def fft(self, x):
        x = _c64(x)
        out = np.empty_like(x)
        getattr(self.lib, self.prefix + "fft")(x.view(np.float32), out.view(np.float32), len(x))
        return out

    def gen_chirp(self, N, osr, NN, f0, down, ampl, phase, bw_scale):
        out = np.empty(NN, np.complex64)
        ph = C.c_float(phase)
        getattr(self.lib, self.prefix + "gen_chirp")(out.ctypes.data_as(C.c_void_p), N, osr, NN,
                                                     C.c_float(f0),
                                                     int(down), C.c_float(ampl), C.byref(ph),
                                                     C.c_float(bw_scale))
        return out, ph.value

    def lora_encode(self, payload: bytes) -> np.ndarray:
        b = np.frombuffer(bytes(payload), np.uint8).copy()
        out = np.zeros(2 * len(b) + 1, np.uint16)
        if self.prefix == "ref_":
            n = self.lib.ref_lora_encode(b, len(b), out, 7)
        else:
            n = self.lib.orc_lora_encode(b, len(b), out)
        return out[:n]

    def lora_decode(self, syms) -> bytes:
        s = np.ascontiguousarray(np.asarray(syms, np.uint16))
        out = np.zeros(len(s) // 2 + 1, np.uint8)
        n = getattr(self.lib, self.prefix + "lora_decode")(s, len(s), out)
        return out[:n].tobytes()

    def lora_demodulate(self, iq, sf, osr=1, hann=False, scratch_len=None):
        """One legacy lora_demodulate call; returns (symbols, sync, cfo, time_offset)."""
        x = _c64(iq)
        n_sym = max(len(x) // ((1 << sf) * osr), 1)
        out = np.zeros(n_sym, np.uint16)
        sync = C.c_uint8(0)
        cfo = C.c_float(0)
        toff = C.c_float(0)
        sl = len(x) if scratch_len is None else scratch_len
        n = getattr(self.lib, self.prefix + "lora_demodulate")(
            x.view(np.float32), len(x), sf, int(hann), osr, out, C.byref(sync), C.byref(cfo),
            C.byref(toff), sl)
        return out[:n].copy(), sync.value, cfo.value, toff.value

    def lora_modulate(self, syms, sf, osr=1, bw=125000, amplitude=1.0, sync=0x12):
        s = np.ascontiguousarray(np.asarray(syms, np.uint16))
        out = np.zeros((len(s) + 2) * (1 << sf) * osr, np.complex64)
        if self.prefix == "ref_":
            n = self.lib.ref_lora_modulate(s, len(s), out.view(np.float32), sf, osr, bw,
                                           C.c_float(amplitude), sync)
        else:
            n = self.lib.orc_lora_modulate(s, len(s), out.view(np.float32), sf, osr,
                                           C.c_float(BW_SCALE[bw]), C.c_float(amplitude), sync)
        return out[:n]

    def api_demodulate(self, iq, sf, osr=1, hann=False, bw=125000, cap=None):
        x = _c64(iq)
        cap = max(len(x) // ((1 << sf) * osr), 2) if cap is None else cap
        out = np.zeros(max(cap, 1), np.uint16)
        sync = C.c_uint8(0)
        cfo = C.c_float(0)
        toff = C.c_float(0)
        if self.prefix == "ref_":
            r = self.lib.ref_api_demodulate(x.view(np.float32), len(x), sf, int(hann), osr, bw, out,
                                            cap, C.byref(sync), C.byref(cfo), C.byref(toff))
        else:
            r = self.lib.orc_api_demodulate(x.view(np.float32), len(x), sf, int(hann), osr,
                                            C.c_float(BW_SCALE[bw]), out, cap, C.byref(sync),
                                            C.byref(cfo), C.byref(toff))
        return r, out[:max(r, 0)].copy(), sync.value, cfo.value, toff.value

    def estimate_offsets(self, iq, sf, osr=1, hann=False):
        x = _c64(iq)
        cfo = C.c_float(0)
        toff = C.c_float(0)
        getattr(self.lib, self.prefix + "estimate_offsets")(x.view(np.float32), len(x), sf,
                                                            int(hann), osr, C.byref(cfo),
                                                            C.byref(toff))
        return cfo.value, toff.value

    def compensate_offsets(self, iq, sf, osr, cfo, to):
        x = _c64(iq).copy()
        getattr(self.lib, self.prefix + "compensate_offsets")(x.view(np.float32), len(x), sf, osr,
                                                              C.c_float(cfo), C.c_float(to))
        return x

    def demod_frames(self, iq2d, sf, osr=1, hann=False, dechirp=False, bw=125000, threads=1):
        """Legacy lora_demodulate over a [F, L] complex64 batch (one call per frame)."""
        x = _c64(iq2d)
        F, L = x.shape
        total = L // ((1 << sf) * osr)
        stride = max(total, 1)
        syms = np.zeros((F, stride), np.uint16)
        sync = np.zeros(F, np.uint8)
        cfo = np.zeros(F, np.float32)
        toff = np.zeros(F, np.float32)
        cnt = np.zeros(F, np.int64)
        getattr(self.lib, self.prefix + "demod_frames")(
            x.reshape(-1).view(np.float32), F, L, sf, int(hann), osr, int(dechirp), BW_SCALE[bw],
            syms, stride, sync, cfo, toff, cnt, threads)
        return syms, sync, cfo, toff, cnt


class Oracle(_Common):
    prefix = "orc_"

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        self.lib = C.CDLL(path)
        L = self.lib
        L.orc_gen_chirp.restype = C.c_int
        L.orc_fft.argtypes = [_f32p, _f32p, C.c_int]
        L.orc_fft_twiddles.argtypes = [_f32p, C.c_int]
        L.orc_lora_modulate.restype = C.c_size_t
        L.orc_lora_modulate.argtypes = [_u16p, C.c_size_t, _f32p, C.c_uint, C.c_uint, C.c_float,
                                        C.c_float, C.c_uint8]
        L.orc_dechirp.argtypes = [_f32p, _f32p, C.c_size_t, C.c_uint, C.c_uint, C.c_float]
        L.orc_lora_demodulate.restype = C.c_size_t
        L.orc_lora_demodulate.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint, _u16p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_demod_frames.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_uint, C.c_int, C.c_uint,
                                       C.c_int, C.c_float, _u16p, C.c_size_t, _u8p, _f32p, _f32p,
                                       _i64p, C.c_int]
        L.orc_api_demodulate.restype = C.c_long
        L.orc_api_demodulate.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint,
                                         C.c_float, _u16p, C.c_size_t, C.c_void_p, C.c_void_p,
                                         C.c_void_p]
        L.orc_estimate_offsets.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint,
                                           C.c_void_p, C.c_void_p]
        L.orc_compensate_offsets.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_uint, C.c_float,
                                             C.c_float]
        L.orc_raw_demod.restype = C.c_size_t
        L.orc_raw_demod.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint, C.c_int,
                                    C.c_float, _u16p]
        L.orc_lora_encode.restype = C.c_size_t
        L.orc_lora_encode.argtypes = [_u8p, C.c_size_t, _u16p]
        L.orc_lora_decode.restype = C.c_size_t
        L.orc_lora_decode.argtypes = [_u16p, C.c_size_t, _u8p]
        L.orc_awgn_gtest_frames.restype = C.c_size_t

    def raw_demod(self, iq, sf, osr=1, hann=False, dechirp=False, bw=125000):
        """LORA_MODE_RAW checker: per-symbol (dechirp) -> window -> FFT -> argmax."""
        x = _c64(iq)
        out = np.zeros(max(len(x) // ((1 << sf) * osr), 1), np.uint16)
        n = self.lib.orc_raw_demod(x.view(np.float32), len(x), sf, int(hann), osr, int(dechirp),
                                   C.c_float(BW_SCALE[bw]), out)
        return out[:n]

    def twiddles(self, N):
        out = np.empty(N, np.complex64)
        self.lib.orc_fft_twiddles(out.view(np.float32), N)
        return out

    def dechirp(self, iq, sf, osr=1, bw=125000):
        x = _c64(iq)
        y = np.empty_like(x)
        self.lib.orc_dechirp(x.view(np.float32), y.view(np.float32), len(x), sf, osr,
                             BW_SCALE[bw])
        return y

    def awgn_gtest_frames(self, profiles, packets=5, payload_size=16, snr_db=12.0):
        sfs = (C.c_uint * len(profiles))(*[p[0] for p in profiles])
        bws = (C.c_float * len(profiles))(*[BW_SCALE[p[1]] for p in profiles])
        total = sum(((2 * payload_size) + 2) * (1 << p[0]) * packets for p in profiles)
        iq = np.zeros(total, np.complex64)
        pay = np.zeros(len(profiles) * packets * payload_size, np.uint8)
        self.lib.orc_awgn_gtest_frames(sfs, bws, len(profiles), packets, payload_size,
                                       C.c_double(snr_db), iq.ctypes.data_as(C.c_void_p),
                                       pay.ctypes.data_as(C.c_void_p))
        return iq, pay


class Reference(_Common):
    prefix = "ref_"

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def __init__(self, path: str = REF_SO):
        self.lib = C.CDLL(path)
        L = self.lib
        L.ref_gen_chirp.restype = C.c_int
        L.ref_fft.argtypes = [_f32p, _f32p, C.c_int]
        L.ref_lora_modulate.restype = C.c_size_t
        L.ref_lora_modulate.argtypes = [_u16p, C.c_size_t, _f32p, C.c_uint, C.c_uint, C.c_uint,
                                        C.c_float, C.c_uint8]
        L.ref_lora_demodulate.restype = C.c_size_t
        L.ref_lora_demodulate.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint, _u16p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.ref_api_demodulate.restype = C.c_long
        L.ref_api_demodulate.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint, C.c_uint,
                                         _u16p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ref_estimate_offsets.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_int, C.c_uint,
                                           C.c_void_p, C.c_void_p]
        L.ref_compensate_offsets.argtypes = [_f32p, C.c_size_t, C.c_uint, C.c_uint, C.c_float,
                                             C.c_float]
        L.ref_lora_encode.restype = C.c_size_t
        L.ref_lora_encode.argtypes = [_u8p, C.c_size_t, _u16p, C.c_uint]
        L.ref_lora_decode.restype = C.c_size_t
        L.ref_lora_decode.argtypes = [_u16p, C.c_size_t, _u8p]
        L.ref_awgn_gtest_frames.restype = C.c_size_t
        L.ref_demod_frames.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_uint, C.c_int, C.c_uint,
                                       C.c_int, C.c_float, _u16p, C.c_size_t, _u8p, _f32p, _f32p,
                                       _i64p, C.c_int]
        for name, rt in [("ref_enc_h84", C.c_uint8), ("ref_enc_h74", C.c_uint8),
                         ("ref_enc_p54", C.c_uint8), ("ref_enc_p64", C.c_uint8)]:
            getattr(L, name).restype = rt
            getattr(L, name).argtypes = [C.c_uint8]
        L.ref_dec_h84.restype = C.c_uint8
        L.ref_dec_h84.argtypes = [C.c_uint8, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        for name in ("ref_dec_h74", "ref_chk_p54", "ref_chk_p64"):
            getattr(L, name).restype = C.c_uint8
            getattr(L, name).argtypes = [C.c_uint8, C.POINTER(C.c_int)]
        L.ref_gray2bin.restype = C.c_uint16
        L.ref_gray2bin.argtypes = [C.c_uint16]
        L.ref_bin2gray.restype = C.c_uint16
        L.ref_bin2gray.argtypes = [C.c_uint16]
        L.ref_checksum8.restype = C.c_uint8
        L.ref_checksum8.argtypes = [_u8p, C.c_size_t]
        L.ref_header_checksum.restype = C.c_uint8
        L.ref_header_checksum.argtypes = [_u8p]
        L.ref_sx1272_crc.restype = C.c_uint16
        L.ref_sx1272_crc.argtypes = [_u8p, C.c_int]
        L.ref_whiten_sx1232.argtypes = [_u8p, C.c_uint16]
        L.ref_whiten_sx1272.argtypes = [_u8p, C.c_uint16, C.c_int, C.c_int]
        L.ref_whiten_lfsr.argtypes = [_u8p, C.c_uint16, C.c_int, C.c_size_t]
        L.ref_interleave.argtypes = [_u8p, C.c_size_t, _u16p, C.c_size_t, C.c_size_t]
        L.ref_deinterleave.argtypes = [_u16p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t]
        L.ref_deinterleave2.argtypes = [_u16p, C.c_size_t, _u8p, C.c_size_t, C.c_size_t]

    def awgn_gtest_frames(self, profiles, packets=5, payload_size=16, snr_db=12.0):
        sfs = (C.c_uint * len(profiles))(*[p[0] for p in profiles])
        bws = (C.c_uint * len(profiles))(*[p[1] for p in profiles])
        total = sum(((2 * payload_size) + 2) * (1 << p[0]) * packets for p in profiles)
        iq = np.zeros(total, np.complex64)
        pay = np.zeros(len(profiles) * packets * payload_size, np.uint8)
        self.lib.ref_awgn_gtest_frames(sfs, bws, len(profiles), packets, payload_size,
                                       C.c_double(snr_db), iq.ctypes.data_as(C.c_void_p),
                                       pay.ctypes.data_as(C.c_void_p))
        return iq, pay
