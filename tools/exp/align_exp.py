#!/usr/bin/env python3
"""Alignment experiment: the SF7 bench batch (noiseless) with a fractional carrier offset of
`frac` bins injected, so the estimate's t_off (about -frac N) shifts every data window; per offset the step time (HIP graph replay) and the per-kernel HIP-event
times.  usage: align_exp.py [sf] [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "lora-sdr-lightweight-standalone-library-_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lora_phy_amd as amd  # noqa: E402

sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 15625
N = 1 << sf
dev = torch.device("cuda", 0)
syms, iq0 = bench.make_input(sf, frames, 64, 20251015, dev)
n = torch.arange(iq0.shape[1], device=dev, dtype=torch.float64)
for frac in (0.0, 0.01, 0.02, 0.04, 0.06, 0.1, 0.2, 0.3):
    shift = frac
    rot = torch.exp(2j * torch.pi * frac * n / N).to(torch.complex64)
    iq = (iq0 * rot).contiguous()
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=dev)
    out = None
    for _ in range(5):
        out = plan.run(iq, out)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        out = plan.run(iq, out)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = plan.run(iq, out)
    g.replay()
    torch.cuda.synchronize()
    f0 = plan.spec_recomputed()
    steps = 100
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    fixed = (plan.spec_recomputed() - f0) / steps
    st, out = bench.stage_times(plan, iq, out, 20, dev)
    toff = out.time_offset.round().to(torch.int64)
    vals, cnt = torch.unique(toff, return_counts=True)
    ser = float((out.symbols.to(torch.int32).cpu() != syms).float().mean())
    print(f"cfo {shift:.2f} bin: step {ms:.4f} ms  est {st[1]:.4f}  demod {st[2]:.4f}  recomputed/step {fixed:.0f}  "
          f"t_off {dict(zip(vals.tolist()[:4], cnt.tolist()[:4]))}  ser_vs_tx {ser:.3f}", flush=True)
    plan.close()
