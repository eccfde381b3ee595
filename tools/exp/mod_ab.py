"""Modulator A/B across in-tree variant libraries: for each library (a subprocess with
LORA_MI355X_LIB set), lora_mod_batch of the bench's batches (SF7 and SF12, 15,625 frames x 64
symbols) into one preallocated output, HIP events around `reps` calls, alternating libraries
over `rounds` rounds; every variant's output hashed against the first library's.
--few: k_mod_frame's shapes instead (1 and 64 frames at SF7, 1 at SF12).
usage: python tools/exp/mod_ab.py [--rounds R] [--reps K] [--few] base mph4 ..."""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "..", "lora-sdr-lightweight-standalone-library-_amd")
VAR = os.path.join(PKG, "lora_phy_amd", "lib", "variants")

CHILD = r"""
import hashlib, json, sys, torch
sys.path.insert(0, PKG)
import lora_phy_amd as amd
reps = REPS
res = {}
for sf, frames in WORKS:
    g = torch.Generator(device="cpu").manual_seed(sf)
    syms = torch.randint(0, 1 << sf, (frames, 64), generator=g, dtype=torch.int32).to(torch.uint16).cuda()
    out = amd.modulate(syms, sf)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        amd.modulate(syms, sf, out=out)
    e1.record()
    torch.cuda.synchronize()
    h = hashlib.sha256(out.reshape(-1)[::97].cpu().numpy().tobytes()).hexdigest()[:16]
    res[f"sf{sf}x{frames}"] = {"ms": e0.elapsed_time(e1) / reps, "hash": h}
    del out
    torch.cuda.empty_cache()
print(json.dumps(res))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--few", action="store_true", help="k_mod_frame's shapes: 1 and 64 frames")
    args = ap.parse_args()
    works = "((7, 1), (7, 64), (12, 1))" if args.few else "((7, 15625), (12, 15625))"
    code = CHILD.replace("PKG", repr(PKG)).replace("REPS", str(args.reps)).replace("WORKS", works)
    rows = {n: [] for n in args.libs}
    for r in range(args.rounds):
        for name in args.libs:
            env = dict(os.environ)
            if name != "base":
                env["LORA_MI355X_LIB"] = os.path.join(VAR, name + ".so")
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(name, "failed:", p.stderr[-2000:])
                sys.exit(1)
            rows[name].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(r, name, rows[name][-1], flush=True)
    ref = rows[args.libs[0]][0]
    for name, rs in rows.items():
        same = all(x[k]["hash"] == ref[k]["hash"] for x in rs for k in ref)
        print(json.dumps({"lib": name, **{k: [round(x[k]["ms"], 4) for x in rs] for k in ref}, "same_output": same}))


if __name__ == "__main__":
    main()
