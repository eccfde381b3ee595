#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/<round>/.

  kernel_stats.md   per-kernel calls / avg / total duration from the rocprofv3
                    --kernel-trace --stats database (split by grid size, so the SF7 and
                    SF12 launches of a shared kernel are separate rows)
  pmc.md            FETCH_SIZE / WRITE_SIZE per launch for our kernels
  ../pmc_summary.json  HBM bytes per launch of the dominant (demod) kernel per workload,
                    read by bench.py for roofline.traffic.  gfx950 correction
                    (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes
                    of a coalesced streaming read -> x2; WRITE_SIZE is exact.  The demod
                    kernel's 8-byte-per-lane coalesced gathers calibrate the same way: x2
                    FETCH_SIZE lands within 0.3% of the frames' IQ bytes (checked below).

usage: prof_summary.py <gpurun_out/round> <profiles/rNN>
"""
import collections
import csv
import glob
import json
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    if m:
        return m.group(1)
    return name[:60]


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, workgroup_x, duration, lds_size, vgpr_count, sgpr_count,"
                     " scratch_size from kernels").fetchall()
    agg = collections.OrderedDict()
    for name, gx, wx, dur, lds, vgpr, sgpr, scratch in rows:
        key = (short(name), gx // max(wx, 1))
        a = agg.setdefault(key, {"calls": 0, "ns": 0.0, "lds": lds, "vgpr": vgpr, "sgpr": sgpr,
                                 "scratch": scratch})
        a["calls"] += 1
        a["ns"] += float(dur)
    return agg


def pmc(dirpat):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(dirpat)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    agg = kernel_stats(os.path.join(src, "kt", "run_results.db"))
    lines = ["# rocprofv3 --kernel-trace --stats: `python bench.py --steps 10 --warmup 2 --no-cpu`",
             "", "Durations from the rocprofv3 kernel trace (ns).  Workgroups = grid/workgroup size;",
             "SF7 launches: 15,625 frames; SF12: 15,625 frames.", "",
             "| kernel | workgroups | calls | avg us | total us | LDS B | VGPR | SGPR | scratch |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for (k, wg), a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        lines.append(f"| `{k}` | {wg} | {a['calls']} | {a['ns'] / a['calls'] / 1e3:.2f} | "
                     f"{a['ns'] / 1e3:.1f} | {a['lds']} | {a['vgpr']} | {a['sgpr']} | {a['scratch']} |")
    # the bench's own HIP-event kernel times from the SAME profiled run, for comparison
    try:
        runs = [json.loads(l) for l in open(os.path.join(src, "kt.log")) if l.startswith("{")]
        for r in runs:
            st = r["config"]["stage_ms"]
            lines += ["", "bench.py HIP-event averages in the same profiled run (ms; with the speculative "
                      "pipeline `estimate` = pre-pass + certification kernels, no frame-max pass): SF7 frame max "
                      f"{st[0]:.4f}, estimate {st[1]:.4f}, demod {st[2]:.4f}"]
            if "sf12" in r.get("extra", {}):
                s12 = r["extra"]["sf12"]["stage_ms"]
                lines += [f"SF12 frame max {s12[0]:.3f}, estimate {s12[1]:.3f}, demod {s12[2]:.3f}"]
    except (OSError, ValueError, KeyError):
        pass
    # The headline SF7 run is the first bench workload: its warmup + timed + profiled
    # launches come first in the trace, before the FAST / sync-0xFF / AWGN runs that reuse
    # the same kernels (and grids).  Average those launches alone, and the per-step wall
    # time between consecutive frame-max launch starts of the timed steps.
    try:
        c = sqlite3.connect(os.path.join(src, "kt", "run_results.db"))
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
        nfirst = 2 + 10 + 10  # warmup + steps + bench.py's profiled pass (kernel-trace command)
        lines += ["", f"Headline SF7 run only (first {nfirst} launches of each kernel, in trace order):", ""]
        fm_starts = []
        names = {short(n) for n, _, _ in rows}
        # the default speculative pipeline (est pre-pass, demod, est/certify) or the
        # three-launch path (frame max, estimate, demod); the first kernel opens each step
        step_kernels = (("k_est_fast<7, 0, 1>", "k_demod_fast<7, 0, 0, false, true>", "k_est_fast<7, 0, 2>")
                        if "k_est_fast<7, 0, 1>" in names else
                        ("k_frame_max", "k_est_fast<7, 0, 0>", "k_demod_fast<7, 0, 0, false, false>"))
        for kn in step_kernels:
            d = [(b, e) for n, b, e in rows if short(n) == kn][:nfirst]
            if kn == step_kernels[0]:
                fm_starts = [b for b, _ in d]
            avg = sum(e - b for b, e in d) / max(len(d), 1) / 1e3
            lines.append(f"- `{kn}`: {len(d)} launches, average {avg:.2f} us")
        if len(fm_starts) >= 12:
            steps = [(fm_starts[i + 1] - fm_starts[i]) / 1e6 for i in range(2, 11)]
            lines.append(f"- step period from the trace (`{step_kernels[0]}` start to start, timed steps): "
                         f"{sum(steps) / len(steps):.4f} ms")
    except (sqlite3.Error, OSError):
        pass
    open(os.path.join(dst, "kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))

    summary = {}
    plines = ["# HBM counters per launch (rocprofv3 --pmc, one counter per pass)", "",
              "FETCH_SIZE / WRITE_SIZE in KB as reported; `read B (x2)` applies the gfx950",
              "correction from MI355X_MICROARCH.md (FETCH_SIZE = half the bytes of a coalesced read).", "",
              "| workload | kernel | FETCH_SIZE KB | read B (x2) | WRITE_SIZE KB | HBM B/launch |",
              "|---|---|---:|---:|---:|---:|"]
    for wl, tag in (("sf7", "nosf12"), ("sf12", "sf12only")):
        f = pmc(os.path.join(src, f"pmc_FETCH_SIZE{tag}", "run_counter_collection.csv"))
        w = pmc(os.path.join(src, f"pmc_WRITE_SIZE{tag}", "run_counter_collection.csv"))
        for k in f:
            if not k.startswith("k_"):
                continue
            fk = sum(f[k]["FETCH_SIZE"]) / len(f[k]["FETCH_SIZE"])
            wk = sum(w[k]["WRITE_SIZE"]) / len(w[k]["WRITE_SIZE"]) if k in w else 0.0
            hbm = fk * 1024 * 2 + wk * 1024
            plines.append(f"| {wl} | `{k}` | {fk:.0f} | {fk * 2048:.4g} | {wk:.0f} | {hbm:.4g} |")
            if k.startswith("k_demod"):
                summary.setdefault(wl, {}).update({"kernel": k, "fetch_size_kb": fk, "write_size_kb": wk,
                                                   "hbm_bytes_per_launch": hbm})
            if k.startswith(("k_demod", "k_frame_max", "k_est")):
                # one step = frame max + estimate + demod launches
                summary.setdefault(wl, {}).setdefault("step_kernels", {})[k] = hbm
                summary[wl]["hbm_bytes_per_step"] = sum(summary[wl]["step_kernels"].values())
    # VALU issue: dynamic instruction counts of the demod kernel (SQ_INSTS_VALU etc.) and
    # the chip's measured issue rates (tools/micro/pk_rate: scalar fp32 vs fp64 / packed)
    rates = {}
    try:
        for line in open(os.path.join(src, "valu_rates.txt")):
            m = re.match(r"mode (\d): .* ([0-9.]+) wave-instr per CU per ns", line)
            if m:
                rates[int(m.group(1))] = float(m.group(2))
    except OSError:
        pass
    for wl, tag in (("sf7", "nosf12"), ("sf12", "sf12only")):
        v = pmc(os.path.join(src, f"pmc_VALU{tag}", "run_counter_collection.csv"))
        for k, d in v.items():
            if k.startswith("k_demod") and wl in summary and "SQ_INSTS_VALU" in d:
                avg = {c: sum(x) / len(x) for c, x in d.items()}
                dp = sum(avg.get(c, 0.0) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                    "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_CVT"))
                sp = avg["SQ_INSTS_VALU"] - dp
                summary[wl]["valu_winstr_per_launch"] = avg["SQ_INSTS_VALU"]
                summary[wl]["valu_fp64_class_per_launch"] = dp
                if 0 in rates and 3 in rates:
                    # time (ns*CU) the mix needs at the measured issue rates
                    summary[wl]["valu_mix_ns_cu"] = sp / rates[0] + dp / rates[3]
                    summary[wl]["valu_rate_scalar_fp32"] = rates[0]
                    summary[wl]["valu_rate_fp64"] = rates[3]
                plines.append(f"{wl}: {avg['SQ_INSTS_VALU']:.4g} VALU wave-instructions per launch, "
                              f"{dp:.4g} of them fp64-class (fma/mul/add f64, conversions)")
    sf = {"sf7": 7, "sf12": 12}
    for wl, d in summary.items():
        algo = 15625 * 64 * (8 * (1 << sf[wl]) + 2)
        d["algorithmic_bytes_per_launch"] = algo
        d["traffic_over_algorithmic"] = d["hbm_bytes_per_launch"] / algo
        step_algo = 15625 * (66 * (8 * (1 << sf[wl]) + 2) + 9)  # SURVEY 8d, every symbol + per-frame outputs
        d["algorithmic_bytes_per_step"] = step_algo
        d["step_traffic_over_algorithmic"] = d["hbm_bytes_per_step"] / step_algo
        plines.append("")
        plines.append(f"{wl}: demod HBM {d['hbm_bytes_per_launch']:.4g} B vs algorithmic {algo:.4g} B "
                      f"-> {d['traffic_over_algorithmic']:.3f}x")
        plines.append(f"{wl}: step (frame max + estimate + demod) HBM {d['hbm_bytes_per_step']:.4g} B vs "
                      f"algorithmic {step_algo:.4g} B -> {d['step_traffic_over_algorithmic']:.3f}x")
    open(os.path.join(dst, "pmc.md"), "w").write("\n".join(plines) + "\n")
    print("\n".join(plines))
    json.dump(summary, open(os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_summary.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
