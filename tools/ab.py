"""Same-box A/B of library builds on chosen workloads (any round).

usage: python tools/ab.py [--reps 3] [--steps 100] [--work sf7,awgn0,awgn10,...] name [name ...]
  name "default" = the in-tree library; any other name = lora_phy_amd/lib/variants/<name>.so
  (tools/build_variant.sh).  Each (rep, variant) runs in its own process, interleaved;
  prints one line per run: variant, then per workload ms_per_step and the symbol-pass ms.
Workloads: sf7 (headline), awgn0 / awgn10 (SF7 at 0 / -10 dB), sf12, sf12n (SF12 -10 dB),
osr2, hann; mod7 / mod12 (the modulator on 15,625 frames: ms per call, write-peak fraction).
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "variants")

WORK = {
    "sf7": dict(sf=7, frames=15625),
    "awgn0": dict(sf=7, frames=15625, snr_db=0.0),
    "awgn10": dict(sf=7, frames=15625, snr_db=-10.0),
    "osr2": dict(sf=7, frames=15625, osr=2),
    "osr4": dict(sf=7, frames=15625, osr=4),
    "api": dict(sf=7, frames=15625, mode="api"),
    "raw": dict(sf=7, frames=15625, mode="raw"),
    "api12": dict(sf=12, frames=4000, mode="api"),
    "hann": dict(sf=7, frames=15625, window="hann"),
    "sf12": dict(sf=12, frames=15625),
    "sf8": dict(sf=8, frames=15625),
    "sf9": dict(sf=9, frames=15625),
    "sf12n": dict(sf=12, frames=4000, snr_db=-10.0),
}


def child(works, steps):
    sys.path.insert(0, REPO)
    import torch

    import bench

    dev = torch.device("cuda", 0)
    out = {}
    for w in works:
        if w.startswith("mod"):  # modulator: bench.run_modulator, ms per call
            sf = int(w[3:])
            r = bench.run_modulator(sf, 15625, 64, dev, with_cpu=False)
            out[w] = [round(r["ms_per_call"], 4), round(r["roofline_frac"], 4)]
            continue
        kw = dict(WORK[w])
        sf, frames = kw.pop("sf"), kw.pop("frames")
        st = steps if sf < 12 else max(steps // 4, 4)
        r = bench.run_config(sf, frames, 64, st, 5, None, dev, **kw)
        out[w] = [round(r["ms_per_step"], 4), round(r["stage_ms"][2], 4), round(r["stage_ms"][1], 4),
                  r["symbols_ok"] if kw.get("snr_db") is None else r["spec_recomputed_per_step"]]
        del r
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--work", default="sf7,awgn0,awgn10")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    works = a.work.split(",")
    if a.child:
        child(works, a.steps)
        return
    for rep in range(a.reps):
        for name in a.names:
            env = dict(os.environ)
            if name != "default":
                env["LORA_MI355X_LIB"] = os.path.join(VAR, name + ".so")
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--work", a.work,
                                "--steps", str(a.steps)], env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(name, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(2)
            print(rep, name, r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
