"""Stage profile of k_mod_frame (a LORA_MF_PROF variant build writes per-iteration shader
cycles over the frame's first samples; results invalid): one frame of 64 symbols per SF.
Columns per iteration: chain, fill, build, recompute, emit (first worker lane), build (last
worker lane), last lane's total, iteration incl. barrier.
usage: LORA_MI355X_LIB=<variant> python tools/r05_mfprof.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "lora-sdr-lightweight-standalone-library-_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lora_phy_amd as amd  # noqa: E402

for sf in (7, 9, 12):
    syms = torch.randint(0, 1 << sf, (1, 64), dtype=torch.int32).cuda()
    for _ in range(3):
        out = amd.modulate(syms, sf)
    torch.cuda.synchronize()
    p = out.cpu().numpy().reshape(-1).view(np.uint32)[:64 * 8].reshape(64, 8)
    rows = [r for r in p.tolist() if any(r)]
    tot = np.array(rows).sum(0)
    print(f"SF{sf}: iterations {len(rows)}; cycle sums chain {tot[0]} fill {tot[1]} build {tot[2]} recompute {tot[3]} "
          f"emit {tot[4]} build(last) {tot[5]} last-lane {tot[6]} iterations {tot[7]}")
    for r in rows[:6]:
        print("   ", r)
