"""Per-wave phase timing of the speculative demod kernel (diagnostic build only):

  tools/build_variant.sh stamps -DLORA_STAMPS
  LORA_MI355X_LIB=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants/stamps.so \\
      python tools/stamps.py [sf]

Runs the bench workload (noiseless, 66-symbol frames) through the pipeline a few times,
then reads the stamps of the last symbol-demod launch: per wave the shader clock after
index math + loads + dechirp + window max (phase A), the rotation (B), the FFT with its
LDS passes (C), the cross-lane reductions and stores (D), and the 100 MHz clock at wave
start / end.  Prints phase medians and the concurrency timeline.  The stamps' fences
forbid overlaps the real kernel has: read shares, not absolute lengths."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "lora-sdr-lightweight-standalone-library-_amd"))
import lora_phy_amd as amd  # noqa: E402
from lora_phy_amd import _capi  # noqa: E402

sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
frames = int(sys.argv[2]) if len(sys.argv) > 2 else (15625 if sf <= 9 else 2000)
S = 64
g = torch.Generator(device="cpu").manual_seed(1)
syms = torch.randint(0, 1 << sf, (frames, S), generator=g, dtype=torch.int32).cuda()
iq = amd.modulate(syms, sf, 1, 125000, 1.0, 0x12)
plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True)
out = None
for _ in range(5):
    out = plan.run(iq, out)
torch.cuda.synchronize()
lib = _capi.lib()
lib.lora_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
nw = 1 << 17
buf = np.zeros(nw * 8, np.uint64)
assert lib.lora_debug_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(nw, 8).astype(np.int64)
valid = (st[:, 0] > 0) & (st[:, 4] > st[:, 0])
st = st[valid]
ph = np.diff(st[:, :5], axis=1)  # cycles: A load+dechirp+max, B rotation, C FFT, D reduce+store
tot = st[:, 4] - st[:, 0]
res = {"sf": sf, "waves": int(len(st))}
for i, name in enumerate(["A_load_dechirp_max", "B_rotation", "C_fft", "D_reduce_store"]):
    res[name] = {"median": float(np.median(ph[:, i])), "p10": float(np.percentile(ph[:, i], 10)),
                 "p90": float(np.percentile(ph[:, i], 90)), "share": float(ph[:, i].sum() / tot.sum())}
res["wave_cycles_median"] = float(np.median(tot))
t0, t1 = st[:, 5], st[:, 6]
span = (t1.max() - t0.min()) * 10e-9
res["span_us"] = span * 1e6
res["wave_real_us_median"] = float(np.median(t1 - t0) * 10e-3)
res["clock_ghz"] = float(np.median(tot / np.maximum(t1 - t0, 1)) / 10.0)  # shader cycles per 10-ns tick / 10
# concurrency: waves alive per 1-us bin over the recorded span
edges = np.arange(t0.min(), t1.max() + 100, 100)
alive = np.zeros(len(edges) - 1)
for a_, b_ in zip(t0, t1):
    i0 = np.searchsorted(edges, a_, "right") - 1
    i1 = np.searchsorted(edges, b_, "right") - 1
    alive[i0:i1 + 1] += 1
res["alive_waves_median"] = float(np.median(alive[len(alive) // 4: 3 * len(alive) // 4]))
print(json.dumps(res, indent=1))

# ---- estimate kernels (stage 0 = pre-pass k_est_fast<SPEC=1>, 2 = certify <SPEC=2>) ----
lib.lora_debug_stamps_est.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
names = {0: "start", 1: "max_assembled", 2: "estimate_ffts", 3: "estimate_done", 4: "sync_or_maxloop_done",
         7: "certify_tests_done"}
for stage in (1, 2):
    b = np.zeros(nw * 8, np.uint64)
    assert lib.lora_debug_stamps_est(stage, b.ctypes.data, b.size) == 0
    e = b.reshape(nw, 8).astype(np.int64)
    e = e[(e[:, 0] > 0) & (e[:, 6] > e[:, 5])]
    out = {"stage": stage, "waves": int(len(e))}
    prev = 0
    for k in (1, 2, 3, 4, 7):
        ok = e[:, k] > 0
        if ok.sum() == 0:
            continue
        d = (e[ok, k] - e[ok, prev])
        out[f"{names[prev]}->{names[k]}_cycles_median"] = float(np.median(d))
        prev = k
    real = (e[:, 6] - e[:, 5]) * 10e-3
    out["wave_real_us_median"] = float(np.median(real))
    out["wave_real_us_p90"] = float(np.percentile(real, 90))
    out["kernel_span_us"] = float((e[:, 6].max() - e[:, 5].min()) * 10e-3)
    print(json.dumps(out, indent=1))
