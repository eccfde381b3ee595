"""Phase timing of k_frame_fused (development; needs the LORA_FUSED_TIMING variant):
  tools/build_variant.sh timing -DLORA_FUSED_TIMING
  LORA_MI355X_LIB=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants/timing.so \
      python tools/exp/fused_timing.py
Stamps per workgroup/frame: 0 start, 1 loaded+max, 2 estimate FFTs, 3 params, 4 wave-0 sync
symbol, 5 wave-0 data rounds, 6 frame end (s_memrealtime ticks, 100 MHz)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lora-sdr-lightweight-standalone-library-_amd"))
import lora_phy_amd as amd  # noqa: E402
from lora_phy_amd import _capi  # noqa: E402

sf = int(os.environ.get("SF", "7"))
S = int(os.environ.get("S", "64"))
F = int(os.environ.get("FRAMES", "15625"))
lib = _capi.lib()
lib.lora_debug_fused_timing.argtypes = [C.c_void_p, C.c_size_t]
syms = torch.randint(0, 1 << sf, (F, S), device="cuda", dtype=torch.int32)
iq = amd.modulate(syms, sf)
plan = amd.DemodPlan(sf, dechirp=True)
for _ in range(3):
    plan.run(iq)
torch.cuda.synchronize()
lib.lora_debug_fused_timing_clear()
plan.run(iq)
torch.cuda.synchronize()
assert plan.last_kernels() == {"fused"}, plan.last_kernels()
buf = np.zeros(2048 * 16 * 8, np.uint64)
assert lib.lora_debug_fused_timing(buf.ctypes.data, buf.size) == 0
d = buf.reshape(2048, 16, 8).astype(np.int64)
valid = d[:, :, 6] > 0
t0 = d[valid][:, 0].min()
ph = d[valid]
dur = np.diff(ph[:, :7], axis=1)  # 6 phases
names = ["load+max", "estimate FFTs", "params", "sync(w0)", "data(w0)", "end barrier"]
tick_ns = 10.0
print(f"frames stamped: {valid.sum()}  kernel span: {(ph[:, 6].max() - t0) * tick_ns / 1000:.1f} us")
for i, n in enumerate(names):
    print(f"  {n:14s} mean {dur[:, i].mean() * tick_ns / 1000:7.2f} us   p50 {np.median(dur[:, i]) * tick_ns / 1000:7.2f}"
          f"   p90 {np.percentile(dur[:, i], 90) * tick_ns / 1000:7.2f}")
tot = ph[:, 6] - ph[:, 0]
print(f"  {'frame total':14s} mean {tot.mean() * tick_ns / 1000:7.2f} us")
gaps = (d[:, 1:, 0] - d[:, :-1, 6])[valid[:, 1:] & valid[:, :-1]]
print(f"  gap between frames mean {gaps.mean() * tick_ns / 1000:.2f} us")
# per CU: workgroups sharing a CU (hw id + xcc)
hw = d[:, 0, 7]
cu_key = (hw >> 32) * 10000 + ((hw & 0xffffffff) >> 8 & 0xf) * 100 + ((hw & 0xffffffff) >> 13 & 0x3) * 10 + ((hw & 0xffffffff) >> 16 & 0x3)
vals, cnt = np.unique(cu_key[valid[:, 0]], return_counts=True)
print(f"  workgroups per CU id: {np.bincount(cnt)}")
# overlap of two wgs on the same CU: fraction of time both in data phase
both = []
for v in vals[cnt == 2][:50]:
    ws = np.where((cu_key == v) & valid[:, 0])[0]
    a, b = ws[:2]
    def intervals(w, k0, k1):
        return [(d[w, i, k0], d[w, i, k1]) for i in range(16) if valid[w, i]]
    da, db = intervals(a, 3, 5), intervals(b, 3, 5)
    ov = sum(max(0, min(x1, y1) - max(x0, y0)) for x0, x1 in da for y0, y1 in db)
    tot_a = sum(x1 - x0 for x0, x1 in da)
    both.append(ov / max(tot_a, 1))
if both:
    print(f"  data-phase overlap of the two workgroups of a CU: {np.mean(both):.2f} of wg A's data time")
