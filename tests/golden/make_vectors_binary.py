"""Generate tests/golden/vectors_binary.json: the reference's vectors_binary/*.bin inputs run
through the reference's own LoRaCodes.hpp / LoRaEncoder / LoRaDecoder (compiled from
/root/reference/src and include by oracle/Makefile into oracle/_ref/liblora_ref.so).

The .bin files hold inputs only (scripts/create_binary_vectors.py:33-69: count, then per
record test_type, payload, spreading factor, coding-rate string, input codewords), no
expected outputs.  This script therefore stores, per record, the
parsed inputs (data) and the outputs the REFERENCE computes for them:
  * library path: lora_encode / lora_decode (LoRaEncoder.cpp:8-19, LoRaDecoder.cpp:8-19);
  * the coding chain at the record's SF / CR: nibble code (encodeHamming84sx /
    encodeHamming74sx / encodeParity64 / encodeParity54 / bare nibble), whitening
    (Sx1272ComputeWhiteningLfsr), diagonalInterleaveSx with PPM = SF, binaryToGray16,
    and back: grayToBinary16, diagonalDeterleaveSx, de-whitening, the nibble decoders;
  * the decoders on codewords with one flipped bit each (error paths);
  * interleaver records (codewords, no SF): interleave with PPM = len(codewords) and back.
Records with nothing to run (hamming_*, detection_*, interleaver_tests, modulation_test_
vectors: test types only) are listed with their count.

Run here (needs /root/reference and oracle/_ref): python tests/golden/make_vectors_binary.py
"""
import ctypes as C
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
VEC_DIR = "/root/reference/vectors_binary"
OUT = os.path.join(HERE, "vectors_binary.json")


def parse_bin(path):
    """create_binary_vectors.py:33-69 record layout (little-endian u32 lengths)."""
    b = open(path, "rb").read()
    o = 0

    def u32():
        nonlocal o
        v = struct.unpack_from("<I", b, o)[0]
        o += 4
        return v

    def blob(n):
        nonlocal o
        v = b[o:o + n]
        o += n
        return v

    recs = []
    for _ in range(u32()):
        t = blob(u32()).decode()
        payload = blob(u32())
        sf = u32()
        cr = blob(u32()).decode()
        cw = blob(u32())
        recs.append({"test_type": t, "payload": payload, "sf": sf, "cr": cr, "codewords": cw})
    assert o == len(b), f"{path}: {len(b) - o} trailing bytes"
    return recs


def rdd_of(cr):
    s = str(cr)
    return int(s.split("/")[1]) - int(s.split("/")[0]) if "/" in s else int(s)


class RefCodes:
    def __init__(self):
        from oracle.pyoracle import Reference as Ref

        self.r = Ref()
        self.L = self.r.lib

    def u8(self, a):
        if isinstance(a, (bytes, bytearray)):
            a = np.frombuffer(bytes(a), np.uint8)
        return np.ascontiguousarray(np.asarray(a, np.uint8))

    def enc(self, nib, rdd):
        f = {4: self.L.ref_enc_h84, 3: self.L.ref_enc_h74, 2: self.L.ref_enc_p64, 1: self.L.ref_enc_p54}.get(rdd)
        return [int(f(int(x))) if f else int(x) & 0xF for x in nib]

    def dec(self, cw, rdd):
        out, errs = [], []
        for b in cw:
            e, bad = C.c_int(0), C.c_int(0)
            if rdd == 4:
                n = self.L.ref_dec_h84(int(b), C.byref(e), C.byref(bad))
            elif rdd == 3:
                n = self.L.ref_dec_h74(int(b), C.byref(e))
            elif rdd == 2:
                n = self.L.ref_chk_p64(int(b), C.byref(e))
            elif rdd == 1:
                n = self.L.ref_chk_p54(int(b), C.byref(e))
            else:
                n = int(b) & 0xF
            out.append(int(n) & 0xF)
            errs.append(int(bool(e.value) or bool(bad.value)))
        return out, errs

    def whiten(self, cw, rdd):
        buf = self.u8(cw).copy()
        self.L.ref_whiten_lfsr(buf, len(buf), 0, rdd)
        return buf

    def interleave(self, cw, ppm, rdd):
        cw = self.u8(cw)
        syms = np.zeros(len(cw) // ppm * (4 + rdd), np.uint16)
        self.L.ref_interleave(cw, len(cw), syms, ppm, rdd)
        return syms

    def deinterleave(self, syms, ppm, rdd):
        syms = np.ascontiguousarray(np.asarray(syms, np.uint16))
        cw = np.zeros(len(syms) // (4 + rdd) * ppm, np.uint8)  # zero-initialised (LoRaCodes.hpp:400)
        self.L.ref_deinterleave(syms, len(syms), cw, ppm, rdd)
        return cw

    def gray(self, x):
        return [int(self.L.ref_bin2gray(int(v))) for v in x]

    def ungray(self, x):
        return [int(self.L.ref_gray2bin(int(v))) for v in x]

    def lib_encode(self, payload, sf):
        p = self.u8(bytearray(payload))
        out = np.zeros(2 * len(p), np.uint16)
        n = self.L.ref_lora_encode(p, len(p), out, sf)
        return out[:n]

    def lib_decode(self, syms):
        s = np.ascontiguousarray(np.asarray(syms, np.uint16))
        out = np.zeros(len(s) // 2 + 1, np.uint8)
        n = self.L.ref_lora_decode(s, len(s), out)
        return out[:n]


def chain_record(R, payload, sf, rdd):
    nib = []
    for byte in payload:
        nib += [byte >> 4, byte & 0xF]
    cw = R.enc(nib, rdd)
    cw += [0] * (-(-len(cw) // sf) * sf - len(cw))
    wh = R.whiten(cw, rdd)
    il = R.interleave(wh, sf, rdd)
    sy = R.gray(il)
    bi = R.ungray(sy)
    di = R.deinterleave(bi, sf, rdd)
    dw = R.whiten(di, rdd)
    dn, de = R.dec(dw, rdd)
    dec = bytes(((dn[2 * i] << 4) | dn[2 * i + 1]) for i in range(len(payload)))
    # error paths: codeword k with bit (k mod (4 + rdd)) flipped
    flipped = [int(c) ^ (1 << (k % (4 + rdd))) for k, c in enumerate(cw)]
    fn, fe = R.dec(flipped, rdd)
    return {
        "codewords": bytes(cw).hex(), "whitened": bytes(wh).hex(), "interleaved": [int(v) for v in il],
        "symbols": sy, "binary": bi, "deinterleaved": bytes(di).hex(), "dewhitened": bytes(dw).hex(),
        "nibbles": dn, "errors": de, "decoded": dec.hex(),
        "flipped": bytes(flipped).hex(), "flipped_nibbles": fn, "flipped_errors": fe,
    }


def main():
    R = RefCodes()
    files = {}
    for fn in sorted(os.listdir(VEC_DIR)):
        if not fn.endswith(".bin"):
            continue
        recs = parse_bin(os.path.join(VEC_DIR, fn))
        out, skipped = [], {}
        for i, r in enumerate(recs):
            rec = {"index": i, "test_type": r["test_type"], "sf": r["sf"], "cr": r["cr"],
                   "payload": r["payload"].hex(), "input_codewords": r["codewords"].hex()}
            rdd = rdd_of(r["cr"])
            if r["payload"] and 7 <= r["sf"] <= 12:
                sym = R.lib_encode(r["payload"], r["sf"])
                rec["lib_symbols"] = [int(v) for v in sym]
                rec["lib_decoded"] = bytes(R.lib_decode(sym)).hex()
                rec["rdd"] = rdd
                rec["chain"] = chain_record(R, r["payload"], r["sf"], rdd)
            elif r["codewords"]:
                ppm = len(r["codewords"])
                il = R.interleave(r["codewords"], ppm, rdd)
                rec["rdd"] = rdd
                rec["ppm"] = ppm
                rec["interleaved"] = [int(v) for v in il]
                rec["symbols"] = R.gray(il)
                rec["deinterleaved"] = bytes(R.deinterleave(il, ppm, rdd)).hex()
            else:
                skipped[r["test_type"]] = skipped.get(r["test_type"], 0) + 1
                continue
            out.append(rec)
        files[fn] = {"records": len(recs), "checked": out, "no_data": skipped}
        print(f"{fn}: {len(recs)} records, {len(out)} with data, no data: {skipped}")
    with open(OUT, "w") as fh:
        json.dump({"source": "reference vectors_binary/*.bin (inputs) + oracle/_ref LoRaCodes.hpp (outputs)",
                   "files": files}, fh, separators=(",", ":"), sort_keys=True)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
