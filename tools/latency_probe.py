#!/usr/bin/env python3
"""Per-call latency of one frame (the drop-in's one-packet case) through DemodPlan.run with a
synchronize per call, for each pipeline ("spec", "split").
usage: latency_probe.py [sf ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "lora-sdr-lightweight-standalone-library-_amd"))
import torch  # noqa: E402

import lora_phy_amd as amd  # noqa: E402

sfs = [int(v) for v in sys.argv[1:]] or [7, 8, 9, 10]
dev = torch.device("cuda", 0)
res = {}
for sf in sfs:
    N = 1 << sf
    syms = torch.randint(0, N, (1, 64), dtype=torch.int32, device=dev)
    iq = amd.modulate(syms, sf)
    for pipe in ("spec", "split"):
        plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, pipeline=pipe)
        out = plan.run(iq)
        torch.cuda.synchronize()
        ok = bool((out.symbols.to(torch.int32) == syms).all())
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            plan.run(iq, out)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        res[f"sf{sf}_{pipe}"] = {"median_us": round(ts[len(ts) // 2] * 1e6, 2), "min_us": round(ts[0] * 1e6, 2),
                                 "ok": ok, "kernels": sorted(plan.last_kernels())}
        print(f"sf{sf} {pipe:8s} median {ts[len(ts)//2]*1e6:8.2f} us  min {ts[0]*1e6:8.2f} us  ok={ok}", flush=True)
print(json.dumps(res))
