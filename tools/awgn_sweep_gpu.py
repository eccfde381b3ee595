#!/usr/bin/env python3
"""AWGN SNR sweep on one MI355X (BASELINE.json configs[3]).

Library chain per SF: lora_encode -> GPU lora_modulate -> complex AWGN sigma=10^(-SNR/20)
-> GPU LEGACY lora_demodulate (normalisation + 2-sync-symbol CFO/timing estimate + CFO
rotation + FFT + argmax) -> lora_decode.  Reports SER/BER/PER per (SF, SNR) and the
agreement of every GPU output (symbols, sync, cfo/time_offset bits) with the CPU
oracle on the first `--check` frames of each point.  Also the reference script's own
model (awgn.simulate, RAW mode) at the same SNRs for SF7.

usage: python tools/awgn_sweep_gpu.py [--frames 1000] [--snr -20 10 1] [--cfo 0.2] [--out FILE]

Every frame of every point is also compared with the three-launch exact path (the
oracle-pinned kernels, LORA_MI355X_SPEC=0): symbols, sync word and cfo / time_offset bits.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from lora_phy_amd import awgn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--payload", type=int, default=16)
    ap.add_argument("--snr", type=float, nargs=3, default=[-20.0, 10.0, 1.0])
    ap.add_argument("--sfs", type=int, nargs="+", default=[7, 8, 9, 10, 11, 12])
    ap.add_argument("--check", type=int, default=32, help="frames per point checked vs the oracle")
    ap.add_argument("--cfo", type=float, default=0.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from oracle.pyoracle import Oracle

    O = Oracle()
    snrs = list(np.arange(args.snr[0], args.snr[1] + 1e-9, args.snr[2]))
    out = {"config": vars(args), "chain": [], "script_model": []}
    t0 = time.time()
    for sf in args.sfs:
        recs = awgn.sweep_chain(sf, snrs, frames=args.frames, payload_len=args.payload, seed=1234 + sf,
                                cfo_bins=args.cfo, keep_iq=True, exact_check=True)
        for r in recs:
            k = min(args.check, args.frames)
            x = r.pop("iq")[:k].cpu().numpy()
            res = r.pop("result")
            syms, sync, cfo, toff, _ = O.demod_frames(x, sf, 1, False, dechirp=True, threads=16)
            S = res.symbols.shape[1]
            agree = (np.array_equal(res.symbols[:k].cpu().numpy(), syms[:, :S])
                     and np.array_equal(res.sync[:k].cpu().numpy(), sync)
                     and np.array_equal(res.cfo[:k].cpu().numpy().view(np.uint32), cfo.view(np.uint32))
                     and np.array_equal(res.time_offset[:k].cpu().numpy().view(np.uint32), toff.view(np.uint32)))
            r["oracle_checked_frames"] = k
            r["oracle_bit_exact"] = bool(agree)
            out["chain"].append(r)
            print(f"SF{sf} {r['snr_db']:+5.1f} dB  SER {r['ser']:.4f}  BER {r['ber']:.5f}  PER {r['per']:.3f}"
                  f"  oracle-exact {agree}  vs exact path: {r['exact_path_frame_mismatches']} of "
                  f"{r['exact_path_frames_compared']} frames differ, {r['recomputed_symbols']} recomputed", flush=True)
    up, down = awgn.make_chirps(7)
    np.random.seed(1234)
    for snr in snrs:
        for cr in ("4/5", "4/8"):
            ber, per = awgn.simulate(7, cr, float(snr), 100, args.payload, up, down)
            out["script_model"].append({"sf": 7, "cr": cr, "snr_db": float(snr), "ber": ber, "per": per})
    out["seconds"] = time.time() - t0
    all_exact = all(r["oracle_bit_exact"] for r in out["chain"])
    mism = sum(r["exact_path_frame_mismatches"] for r in out["chain"])
    out["summary"] = {"points": len(out["chain"]), "oracle_checked_frames_per_point": min(args.check, args.frames),
                      "all_oracle_checked_frames_bit_exact": all_exact,
                      "exact_path_frames_compared": sum(r["exact_path_frames_compared"] for r in out["chain"]),
                      "exact_path_frame_mismatches": mism}
    print(f"done in {out['seconds']:.1f} s; every checked point bit-exact vs oracle: {all_exact}; "
          f"frames differing from the exact path: {mism}")
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
