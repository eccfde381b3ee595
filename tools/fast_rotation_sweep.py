#!/usr/bin/env python3
"""LORA_PRECISION_FAST vs EXACT across SF7-12 and SNR (evidence for the tolerance stated
in include/lora_mi355x.h).  Same noisy frames through both plans; reports per-symbol
agreement, SER of each against the transmitted symbols, and whether the per-frame
estimate outputs (sync, cfo, time_offset) are identical.  A CFO of `--cfo` bins is
injected (lora_phy_vector_generate.cpp:102-108 semantics) so the rotation is exercised.

usage: python tools/fast_rotation_sweep.py [--frames 200] [--out FILE]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import lora_phy_amd as amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--symbols", type=int, default=32)
    ap.add_argument("--snr", type=float, nargs=3, default=[-20.0, 10.0, 2.0])
    ap.add_argument("--sfs", type=int, nargs="+", default=[7, 8, 9, 10, 11, 12])
    ap.add_argument("--cfo", type=float, default=0.3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    snrs = list(np.arange(args.snr[0], args.snr[1] + 1e-9, args.snr[2]))
    rows = []
    for sf in args.sfs:
        N = 1 << sf
        F = max(16, args.frames // (1 << max(0, sf - 9)))
        rng = np.random.default_rng(4321 + sf)
        tx = rng.integers(0, N, (F, args.symbols)).astype(np.int32)
        clean = amd.modulate(torch.from_numpy(tx).to(dev), sf)
        L = clean.shape[1]
        nn = torch.arange(L, device=dev, dtype=torch.float64) % N
        ph = 2.0 * math.pi * args.cfo * nn / N
        clean = (clean.to(torch.complex128) * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
        exact = amd.DemodPlan(sf, dechirp=True, precision="exact")
        fast = amd.DemodPlan(sf, dechirp=True, precision="fast")
        gen = torch.Generator(device=dev).manual_seed(99 + sf)
        for snr in snrs:
            sigma = 10.0 ** (-snr / 20.0) / math.sqrt(2.0)
            iq = clean + torch.view_as_complex(torch.randn((F, L, 2), generator=gen, device=dev) * sigma)
            e, f = exact.run(iq), fast.run(iq)
            es = e.symbols.to(torch.int64).cpu().numpy()
            fs = f.symbols.to(torch.int64).cpu().numpy()
            rows.append({"sf": sf, "snr_db": float(snr), "frames": F, "symbols": int(es.size),
                         "agreement": float((es == fs).mean()),
                         "ser_exact": float((es != tx).mean()), "ser_fast": float((fs != tx).mean()),
                         "estimate_identical": bool(torch.equal(e.sync, f.sync) and torch.equal(e.cfo, f.cfo)
                                                    and torch.equal(e.time_offset, f.time_offset))})
            r = rows[-1]
            print(f"SF{sf} {snr:+5.1f} dB  agree {r['agreement']:.5f}  SER exact {r['ser_exact']:.4f} "
                  f"fast {r['ser_fast']:.4f}  estimate identical {r['estimate_identical']}", flush=True)
    worst = min(r["agreement"] for r in rows)
    dser = max(abs(r["ser_fast"] - r["ser_exact"]) for r in rows)
    summary = {"config": vars(args), "rows": rows, "min_agreement": worst, "max_abs_ser_diff": dser,
               "all_estimates_identical": all(r["estimate_identical"] for r in rows)}
    print(json.dumps({k: v for k, v in summary.items() if k != "rows"}))
    if args.out:
        json.dump(summary, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
