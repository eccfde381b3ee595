"""Single-frame modulator latency (k_mod_frame) per library variant: median of 30 calls of
lora_mod_batch on one frame of 64 symbols, HIP events, SF 7 / 9 / 12.
usage: python tools/r05_modprof.py name [name ...]   (default = in-tree; else lib/variants/<name>.so)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "variants")


def child():
    sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
    import torch

    import lora_phy_amd as amd

    res = {}
    for sf in (7, 9, 12):
        syms = torch.randint(0, 1 << sf, (1, 64), dtype=torch.int32).cuda()
        out = amd.modulate(syms, sf)
        ts = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            amd.modulate(syms, sf, out=out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        res[f"sf{sf}_us"] = round(sorted(ts)[len(ts) // 2], 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["--child"]:
        child()
    else:
        for name in sys.argv[1:]:
            env = dict(os.environ)
            if name != "default":
                env["LORA_MI355X_LIB"] = os.path.join(VAR, name + ".so")
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                               text=True, timeout=300)
            print(name, r.stdout.strip() or r.stderr[-800:], flush=True)
