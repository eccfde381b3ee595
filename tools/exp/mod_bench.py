"""lora_mod_batch timing (per call, HIP events) for SF7 and SF12 at the bench's frame counts."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lora-sdr-lightweight-standalone-library-_amd"))
import lora_phy_amd as amd  # noqa: E402

for sf, frames in ((7, 15625), (12, 2000), (12, 15625)):
    syms = torch.randint(0, 1 << sf, (frames, 64), device="cuda", dtype=torch.int32).to(torch.uint16)
    out = amd.modulate(syms, sf)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        out = amd.modulate(syms, sf)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"SF{sf} frames {frames}: {ms:.3f} ms/call, {out.numel() * 8 / ms / 1e6:.0f} GB/s written")
    del out
    torch.cuda.empty_cache()
