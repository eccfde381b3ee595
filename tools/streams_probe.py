#!/usr/bin/env python3
"""Steps of the SF7 headline workload alternated over S HIP streams (each stream its own
workspace and outputs: consecutive batches overlap - one step's latency-bound estimate
stages beside the next one's), against one stream.  usage: streams_probe.py [sf] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "lora-sdr-lightweight-standalone-library-_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lora_phy_amd as amd  # noqa: E402

sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
frames = 15625 if sf < 12 else 4000
dev = torch.device("cuda", 0)
_, iq = bench.make_input(sf, frames, 64, 20251015, dev, None)
plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, device=dev)
ref = plan.run(iq)
torch.cuda.synchronize()
main = torch.cuda.current_stream(dev)
for rnd in range(3):
    for S in (1, 2, 3):
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        outs = [None] * S
        for s in range(S):  # warm each stream's workspace and outputs
            with torch.cuda.stream(streams[s]):
                outs[s] = plan.run(iq, outs[s])
        torch.cuda.synchronize()
        t_end = time.perf_counter() + 0.3
        k = 0
        while time.perf_counter() < t_end:  # pre-warm
            with torch.cuda.stream(streams[k % S]):
                outs[k % S] = plan.run(iq, outs[k % S])
            k += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in streams:
            s.wait_stream(main)
        for k in range(K):
            with torch.cuda.stream(streams[k % S]):
                outs[k % S] = plan.run(iq, outs[k % S])
        for s in streams:
            main.wait_stream(s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        ok = all(bool(torch.equal(o.symbols, ref.symbols)) and bool(torch.equal(o.sync, ref.sync)) for o in outs)
        print(f"round {rnd} streams {S}: {ms:.4f} ms/step  {frames * 64 / ms / 1e3:.1f} Msym/s  ok={ok}", flush=True)
