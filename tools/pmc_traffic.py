#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(PART=pmc bash tools/record.sh: <dir>/pmc_fetch<tag>, <dir>/pmc_write<tag>), with the gfx950 correction
from MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of a wide coalesced read:
doubled).  Writes <out>.md and profiles/pmc_summary.json (read by bench.py for
roofline.traffic): per workload the dominant kernel's HBM bytes per launch and the step's.

usage: [PROF_ROUND=6] pmc_traffic.py gpurun_out/rec/prof profiles/r06/pmc_traffic.md"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, dst = sys.argv[1], sys.argv[2]


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            rows[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))] += float(r["Counter_Value"])
        for (k, _), v in rows.items():
            acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


# algorithmic bytes per launch of the dominant kernel: data symbols x (8N + 2)
# workload: (tag of the pmc_* dirs, sf, frames, data symbols, osr)
WL = {"sf7": ("7", 7, 15625, 64, 1), "sf12": ("12", 12, 4000, 64, 1), "osr2_sf7": ("7o2", 7, 15625, 64, 2),
      # (round 5 on) osr 4, and bench.py's API / RAW receiver lines, whose
      # symbol pass is k_demod_fast (RAW: every symbol an output)
      "osr4_sf7": ("7o4", 7, 15625, 64, 4), "api_sf7": ("7api", 7, 15625, 64, 1), "raw_sf7": ("7raw", 7, 15625, 64, 1)}
ROUND = os.environ.get("PROF_ROUND", "6")
summary, lines = {}, [f"# HBM traffic per launch, rocprofv3 FETCH_SIZE / WRITE_SIZE (r0{ROUND})", "",
                      "FETCH_SIZE / WRITE_SIZE in KB as reported; `read B (x2)` applies the gfx950 correction "
                      "(MI355X_MICROARCH.md: FETCH_SIZE = half the bytes of a coalesced read).  Workloads: "
                      "`tools/prof_workload.py` (noiseless 2 + 64-symbol frames; SF7 15,625 frames, SF12 4,000, SF7 osr 2 15,625).", "",
                      "| workload | kernel | FETCH_SIZE KB | read B (x2) | WRITE_SIZE KB | HBM B/launch | algorithmic B | ratio |",
                      "|---|---|---:|---:|---:|---:|---:|---:|"]
for wl, (tag, sf, frames, S, osr) in WL.items():
    if not os.path.isdir(os.path.join(src, f"pmc_fetch{tag}")):
        continue
    fe = per_kernel(os.path.join(src, f"pmc_fetch{tag}"), "FETCH_SIZE")
    wr = per_kernel(os.path.join(src, f"pmc_write{tag}"), "WRITE_SIZE")
    N = 1 << sf
    # the symbol pass reads every symbol's window (the sync symbols' too) and writes one
    # u16 index per data symbol; the three-launch demod (API / RAW lines) reads and writes
    # its output symbols only (RAW: all S + 2)
    out_syms = S + 2 if wl.startswith("raw") else S
    # (round 5: the API and RAW lines run the symbol pass too - API over the data windows only,
    # RAW over every window with every symbol an output)
    spec_windows = S if wl.startswith("api") else S + 2
    algo = {"k_spec_demod": frames * (spec_windows * 8 * N * osr + 2 * out_syms),
            "k_demod_fast": frames * out_syms * (8 * N + 2)}
    step = 0.0
    d = {"step_kernels": {}}
    for k in sorted(fe):
        if not k.startswith(("k_spec", "k_est", "k_cert", "k_demod_fast", "k_frame_max")):
            continue
        hbm = fe[k] * 1024 * 2 + wr.get(k, 0.0) * 1024
        step += hbm
        d["step_kernels"][k] = hbm
        a = algo.get(k.split("<")[0])
        lines.append(f"| {wl} | `{k}` | {fe[k]:.0f} | {fe[k] * 2048:.4g} | {wr.get(k, 0.0):.0f} | {hbm:.4g} | "
                     f"{a if a else '-'} | {hbm / a if a else float('nan'):.4f} |")
        if k.startswith("k_spec_demod") or (k.startswith("k_demod_fast") and "kernel" not in d):
            d.update({"kernel": k, "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": a,
                      "traffic_over_algorithmic": hbm / a})
    step_algo = frames * ((S + 2) * (8 * N * osr + 2) + 9)
    d.update({"hbm_bytes_per_step": step, "algorithmic_bytes_per_step": step_algo,
              "step_traffic_over_algorithmic": step / step_algo, "frames": frames})
    # bench.py's workloads have 15,625 frames: the byte counts bench.py reads
    # (hbm_bytes_per_launch / _per_step) are scaled to them; the measured ones kept as raw_*
    scale = 15625 / frames
    for key in ("hbm_bytes_per_launch", "hbm_bytes_per_step", "algorithmic_bytes_per_launch",
                "algorithmic_bytes_per_step"):
        if d.get(key) is not None:
            d["raw_" + key] = d[key]
            d[key] = d[key] * scale
    summary[wl] = d
    lines.append(f"| {wl} | whole step | | | | {step:.4g} | {step_algo:.4g} | {step / step_algo:.4f} |")
# VALU issue of the symbol pass from the SQ passes (PART=pmc: pmc1/pmc2 hold
# SQ_INSTS_VALU, pmc5/pmc6 GRBM_GUI_ACTIVE for sf7/sf12): counted as 4 cycles per wave64 VALU
# instruction (a packed fp32 instruction issues at ~0.58 of the scalar rate,
# tools/micro/valu_rate.hip, so this under-counts a packed-heavy body); GRBM_GUI_ACTIVE sums
# the XCDs' busy cycles.
SIMDS, XCDS = 1024, 8
# Share of packed (v_pk_*) instructions among the VALU instructions of the symbol pass's
# steady-state loop (static counts from the disassembly of the built kernels: SF7 262 of
# 505, SF12 378 of 639) and a packed instruction's issue cost in 4-cycle slots (it issues at
# ~0.58 of the scalar rate, tools/micro/valu_rate.hip): the issue-weighted busy fraction.
PK_SHARE = {"sf7": 262 / 505, "sf12": 378 / 639}
PK_COST = 1 / 0.58
lines += ["", "## VALU issue of the symbol pass", "",
          "| workload | kernel | VALU wave-instr / launch | GPU cycles / launch (per XCD) | VALU busy (4 cycles each) | VALU busy (packed weighted) |",
          "|---|---|---:|---:|---:|---:|"]
for wl, (_, sf, frames, S, _), (pv, pg) in zip(WL, WL.values(), (("pmc1", "pmc5"), ("pmc2", "pmc6"))):
    vi = per_kernel(os.path.join(src, pv), "SQ_INSTS_VALU")
    gr = per_kernel(os.path.join(src, pg), "GRBM_GUI_ACTIVE")
    k = summary[wl].get("kernel")
    if not k or k not in vi or k not in gr:
        continue
    cyc = gr[k] / XCDS
    busy4 = vi[k] * 4 / (SIMDS * cyc)
    w = PK_SHARE[wl] * PK_COST + (1 - PK_SHARE[wl])
    busy = busy4 * w
    summary[wl].update({"valu_instr_per_launch": vi[k], "gpu_cycles_per_launch": cyc, "valu_busy_frac": busy,
                        "valu_busy_frac_4cycle": busy4, "valu_packed_share": PK_SHARE[wl],
                        "valu_instr_per_symbol": vi[k] / (frames * (S + 2))})
    lines.append(f"| {wl} | `{k}` | {vi[k]:.4g} | {cyc:.4g} | {busy4:.3f} | {busy:.3f} |")
# round 5: the API / RAW lines' symbol pass (k_spec_demod since they run the pipeline: the
# SF7 pass's packed share), one SQ_INSTS_VALU + GRBM_GUI_ACTIVE pass each (pmc_valu<tag>)
for wl in ("api_sf7", "raw_sf7"):
    tag, sf, frames, S, _ = WL[wl]
    dv = os.path.join(src, f"pmc_valu{tag}")
    k = summary.get(wl, {}).get("kernel")
    if not k or not os.path.isdir(dv):
        continue
    vi, gr = per_kernel(dv, "SQ_INSTS_VALU"), per_kernel(dv, "GRBM_GUI_ACTIVE")
    if k not in vi or k not in gr:
        continue
    cyc = gr[k] / XCDS
    busy4 = vi[k] * 4 / (SIMDS * cyc)
    out_syms = S + 2 if wl.startswith("raw") else S
    share = PK_SHARE["sf7"] if k.startswith("k_spec_demod") else 0.0
    busy = busy4 * (share * PK_COST + (1 - share))
    summary[wl].update({"valu_instr_per_launch": vi[k], "gpu_cycles_per_launch": cyc, "valu_busy_frac": busy,
                        "valu_busy_frac_4cycle": busy4, "valu_packed_share": share,
                        "valu_instr_per_symbol": vi[k] / (frames * out_syms)})
    lines.append(f"| {wl} | `{k}` | {vi[k]:.4g} | {cyc:.4g} | {busy4:.3f} | {busy:.3f} |")
os.makedirs(os.path.dirname(dst), exist_ok=True)
open(dst, "w").write("\n".join(lines) + "\n")
json.dump(summary, open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w"), indent=1)
print("\n".join(lines))
