#!/usr/bin/env python3
"""One bench workload alone, for a profiler: the pipeline over `frames` frames of 2 + 64
symbols (bench.py's make_input: GPU modulation, optional AWGN at `snr` dB), `steps`
times, after an untimed pre-warm.  usage: prof_workload.py <sf> [snr_db|none] [frames] [steps]
[data_symbols] [osr] [mode]
(mode: legacy (default), api or raw - bench.py's receiver lines)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "lora-sdr-lightweight-standalone-library-_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lora_phy_amd as amd  # noqa: E402

sf = int(sys.argv[1])
snr = None if len(sys.argv) < 3 or sys.argv[2] == "none" else float(sys.argv[2])
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 15625
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
data_syms = int(sys.argv[5]) if len(sys.argv) > 5 else 64
osr = int(sys.argv[6]) if len(sys.argv) > 6 else 1
mode = sys.argv[7] if len(sys.argv) > 7 else "legacy"
dev = torch.device("cuda", 0)
_, iq = bench.make_input(sf, frames, data_syms, 20251015, dev, snr, osr=osr)
plan = amd.DemodPlan(sf, osr, 125000, "none", dechirp=True, mode=mode, device=dev)
out = None
# untimed steps for PROF_PREWARM_MS (default 300, as bench.py's --prewarm-ms): a few ms of
# launches from a cold start run below the GPU's sustained clock, and the tracer's averages
# then describe the ramp, not the kernel (round 6: 225 vs 190 us median for the SF7 pass)
import time  # noqa: E402

t_end = time.perf_counter() + float(os.environ.get("PROF_PREWARM_MS", "300")) / 1e3
while time.perf_counter() < t_end:
    for _ in range(8):
        out = plan.run(iq, out)
    torch.cuda.synchronize()
for _ in range(steps):
    out = plan.run(iq, out)
torch.cuda.synchronize()
print("recomputed", plan.spec_recomputed(), "kernels", plan.last_kernels())
