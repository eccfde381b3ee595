#!/usr/bin/env python3
"""Summarise a round-3 profiling call (tools/r03_baseline.sh or tools/r03_diag.sh output)
into markdown: per-kernel rocprofv3 kernel-trace statistics of the SF7 headline alone
(kt7) and of the SF12 workload alone (kt12) - each run launches only that workload's
pipeline, so every kernel name maps to the headline kernel - and SQ / TA counters per
launch of the pipeline kernels (pmcN passes, one rocprofv3 --pmc run each).

usage: prof_r03.py <gpurun_out/dir> [out.md]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:50]


def stats(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), r["VGPR_Count"],
                         r["Scratch_Size"], r["LDS_Block_Size"]))
    rows.sort(key=lambda x: x[1])
    return rows


def main():
    src = sys.argv[1]
    out = []
    for tag in ("kt7", "kt7n10", "kt12"):
        rows = stats(os.path.join(src, tag))
        if not rows:
            continue
        agg = collections.OrderedDict()
        for k, b, e, wg, v, sc, lds in rows:
            a = agg.setdefault((k, wg), {"n": 0, "ns": 0, "vgpr": v, "scratch": sc, "lds": lds})
            a["n"] += 1
            a["ns"] += e - b
        out += [f"## {tag}: rocprofv3 --kernel-trace, one workload only", "",
                "| kernel | workgroups | launches | avg us | LDS B | VGPR | scratch |", "|---|---:|---:|---:|---:|---:|---:|"]
        for (k, wg), a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
            if not k.startswith("k_"):
                continue
            out.append(f"| `{k}` | {wg} | {a['n']} | {a['ns'] / a['n'] / 1e3:.2f} | {a['lds']} | {a['vgpr']} | {a['scratch']} |")
        # step structure: consecutive pipeline kernels; gaps between a kernel's end and the next start
        pipe = [r for r in rows if r[0].startswith(("k_est_fast", "k_est_split", "k_spec_fix", "k_spec_demod", "k_demod_fast", "k_frame_max"))]
        gaps = [pipe[i + 1][1] - pipe[i][2] for i in range(len(pipe) - 1)]
        if gaps:
            gaps.sort()
            out += ["", f"gap between consecutive pipeline kernels under the tracer: median {gaps[len(gaps) // 2] / 1e3:.1f} us "
                    f"(the tracer serialises dispatches; bench.py's own HIP-event stage times and ms_per_step are "
                    f"measured without it)", ""]
    # counters
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for f in glob.glob(os.path.join(src, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith("k_"):
                continue
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    if per:
        out += ["## SQ / TA counters per launch (sum over XCDs / SEs, averaged over launches)", ""]
        for k in sorted(per):
            c = {n: per[k][n] / max(cnt[k][n], 1) for n in per[k]}
            out.append(f"### `{k}`")
            out.append("")
            out.append("| counter | per launch |")
            out.append("|---|---:|")
            for n in sorted(c):
                out.append(f"| {n} | {c[n]:.4g} |")
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                          "SQ_ACTIVE_INST_LDS"):
                    if n in c:
                        out.append(f"| {n} / SQ_WAVE_CYCLES | {c[n] / wc:.3f} |")
            if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
                out.append(f"| VALU wave-instructions per wave | {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.1f} |")
            out.append("")
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
