"""Debug: dump the speculative pipeline's per-symbol (margin, window max) and both
estimates for one batch, and evaluate the certification bound on the host."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "lora-sdr-lightweight-standalone-library-_amd")
import lora_phy_amd as amd  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

O = Oracle()
sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
N = 1 << sf
S, F = 8, 6
rng = np.random.default_rng(100 + sf)
iq = np.zeros((F, S * N), np.complex64)
for f in range(F):
    syms = rng.integers(0, N, S - 2).astype(np.uint16)
    x = O.dechirp(O.lora_modulate(syms, sf, 1, 125000, 0.5, int(rng.integers(0, 256))), sf, 1)[: S * N]
    x = x + 0.05 * (rng.standard_normal(S * N) + 1j * rng.standard_normal(S * N))
    iq[f] = x.astype(np.complex64)
plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=False)
res = plan.run(torch.from_numpy(iq).cuda())
torch.cuda.synchronize()
print("recomputed", plan.spec_recomputed(), "kernels", plan.last_kernels())
ws = next(iter(plan._ws.values())).cpu().numpy()
def al(b):
    return (b + 255) & ~255
cnt = al(F * max(1, min(80, S * N // 4096)) * 4)  # ws_layout: frames * frame_max_blocks u32 (lora_capi.hip)
par = al(F * 32)
fp = ws[cnt:cnt + F * 32].view(np.float32).reshape(F, 8)
fps = ws[cnt + par:cnt + par + F * 32].view(np.float32).reshape(F, 8)
marg = ws[cnt + 2 * par:cnt + 2 * par + F * (S - 2) * 8].view(np.float32).reshape(F, S - 2, 2)
print("fp   (cfo toff rate scale | t_off scaled)", fp[:, :4], fp[:, 4:6].view(np.int32))
print("fp_s (cfo toff rate scale | t_off scaled)", fps[:, :4], fps[:, 4:6].view(np.int32))
print("margins", marg[..., 0])
print("window max", marg[..., 1])
