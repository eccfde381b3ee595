#!/usr/bin/env python3
"""Summarise a profiling call (PART=trace / pmc bash tools/record.sh -> gpurun_out/rec/prof) into
markdown (profiles/rNN/kernel_stats.md): per-kernel
rocprofv3 kernel-trace statistics of each bench workload run alone (kt7: SF7 headline,
kt7n10: SF7 at -10 dB, kt12: SF12, kt7o2: SF7 osr 2 - each run launches only that
workload's pipeline), with each kernel's resources taken from the code-object metadata of
the built library (tools/kernel_resources.py: VGPRs, scratch bytes per lane, static LDS),
not from the trace; then SQ counters per launch of the pipeline kernels (pmcN passes, one
rocprofv3 --pmc run each).

usage: [PROF_ROUND=6] kernel_stats.py gpurun_out/rec/prof profiles/r06/kernel_stats.md"""
import collections
import csv
import glob
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAGS = {"kt7": "SF7 headline (15,625 frames x 66 symbols, noiseless)",
        "kt7n10": "SF7 at -10 dB AWGN (same shape)",
        "kt12": "SF12 (15,625 frames x 66 symbols, noiseless)",
        "kt7o2": "SF7 osr 2 (15,625 frames x 66 symbols, noiseless)",
        "kt7n0": "SF7 at 0 dB AWGN (same shape)",
        "kt7o4": "SF7 osr 4 (15,625 frames x 66 symbols, noiseless)",
        "kt7api": "SF7 API mode (phy::demodulate, same shape)",
        "kt7raw": "SF7 RAW mode (detector per symbol, same shape)"}
ROUND = os.environ.get("PROF_ROUND", "6")


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:50]


def trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), int(r["LDS_Block_Size"])))
    rows.sort(key=lambda x: x[1])
    return rows


def main():
    src = sys.argv[1]
    res = {}
    for r in kernel_resources.kernels(os.path.join(ROOT, kernel_resources.LIB)):
        res.setdefault(short(r.get("demangled", r["name"])), r)
    out = [f"# Round-{ROUND} kernel statistics (rocprofv3 --kernel-trace --stats)", "",
           "Each workload alone (`tools/prof_workload.py`, eager `plan.run` per step).  Resources: code-object "
           "metadata of the built `liblora_mi355x.so` (`tools/kernel_resources.py`); LDS = the metadata's static "
           "bytes + the dynamic bytes the launch requests (`kernel_resources.dynamic_lds`, the launch formulas of "
           "lora_demod_fast.hip restated; the trace's LDS_Block_Size shows only the static part).  bench.py's "
           "HIP-event stage times are measured without the tracer.", ""]
    for tag, what in TAGS.items():
        rows = trace(os.path.join(src, tag))
        if not rows:
            continue
        agg = collections.OrderedDict()
        for k, b, e, wg, lds in rows:
            a = agg.setdefault((k, wg), {"n": 0, "ns": [], "lds": lds})
            a["n"] += 1
            a["ns"].append(e - b)
        out += [f"## {tag}: {what}", "",
                "| kernel | workgroups | launches | avg us | median us | min us | max us | LDS B (static + dynamic) | VGPR | "
                "AGPR | scratch B/lane | VGPR spills |",
                "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
        for (k, wg), a in sorted(agg.items(), key=lambda kv: -sum(kv[1]["ns"])):
            if not k.startswith("k_"):
                continue
            r = res.get(k, {})
            ns = a["ns"]
            st = r.get("group_segment_fixed_size")
            dy = kernel_resources.dynamic_lds("void " + k)
            lds = f"{st} + {dy}" if st is not None and dy is not None else (f"{st} + ?" if st is not None else "?")
            med = sorted(ns)[len(ns) // 2]
            out.append(f"| `{k}` | {wg} | {a['n']} | {sum(ns) / len(ns) / 1e3:.2f} | {med / 1e3:.2f} | {min(ns) / 1e3:.2f} | "
                       f"{max(ns) / 1e3:.2f} | {lds} | {r.get('vgpr_count', '?')} | {r.get('agpr_count', '?')} | "
                       f"{r.get('private_segment_fixed_size', '?')} | {r.get('vgpr_spill_count', '?')} |")
        pipe = [r for r in rows if r[0].startswith(("k_est", "k_cert", "k_spec"))]
        gaps = sorted(pipe[i + 1][1] - pipe[i][2] for i in range(len(pipe) - 1))
        if gaps:
            out += ["", f"gap between consecutive pipeline kernels under the tracer: median "
                        f"{gaps[len(gaps) // 2] / 1e3:.1f} us", ""]
    # bench.py itself under the tracer: its HIP-event stage times beside rocprofv3's averages
    import json
    for tag, key in (("bench7", None), ("bench12", "sf12")):
        rows = trace(os.path.join(src, tag))
        jf = os.path.join(src, tag + ".json")
        if not rows or not os.path.exists(jf):
            continue
        d = json.loads(open(jf).read().strip().splitlines()[-1])
        r = d if key is None else d
        stage = r["config"]["stage_ms"] if key is None else r["stage_ms"]
        agg = collections.defaultdict(list)
        for k, b, e, wg, lds in rows:
            if k.startswith(("k_spec", "k_est", "k_cert")):
                agg[k].append(e - b)
        out += [f"## {tag}: `python bench.py {'--no-cpu --no-channels --no-fast --no-variants --no-sf12' if key is None else '--sf12-only'}` under rocprofv3 --kernel-trace --stats", "",
                f"bench.py's HIP-event stage times in the same run (ms per step): estimate stages {stage[1]:.4f}, "
                f"symbol pass {stage[2]:.4f}; ms_per_step {r['ms_per_step']:.4f} (timed steps: "
                f"{'one HIP-graph replay' if d.get('config', {}).get('launch') == 'graph' else 'plan.run'} per step, "
                f"on {d.get('config', {}).get('streams', r.get('streams', 1))} stream(s)).  The stage times "
                f"are bench.py's one-batch-at-a-time pass; the trace averages every launch of the process - "
                f"pre-warm, warm-up and timed steps on the streams, where a launch running beside the other "
                f"batch's kernels takes longer, and the stage passes - so its median is the comparable figure.", "",
                "| kernel | launches | avg us (rocprofv3) | median us |", "|---|---:|---:|---:|"]
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            vs = sorted(v)
            out.append(f"| `{k}` | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {vs[len(vs) // 2] / 1e3:.2f} |")
        out.append("")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for f in sorted(glob.glob(os.path.join(src, "pmc[0-9]*", "**", "*counter_collection.csv"), recursive=True)):
        seen = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k.startswith("k_"):
                seen[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, n, _), v in seen.items():
            per[k][n] += v
            cnt[k][n] += 1
    if per:
        out += ["## SQ counters per launch (summed over XCDs / SEs, averaged over launches)", "",
                f"SF7 workloads: 15,625 frames; SF12: 4,000 frames (tools/r0{ROUND}_prof.sh).", ""]
        for k in sorted(per):
            if not k.startswith(("k_spec_demod", "k_est", "k_cert")):
                continue
            c = {n: per[k][n] / max(cnt[k][n], 1) for n in per[k]}
            out += [f"### `{k}`", "", "| counter | per launch |", "|---|---:|"]
            out += [f"| {n} | {c[n]:.4g} |" for n in sorted(c)]
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                          "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                    if n in c:
                        out.append(f"| {n} / SQ_WAVE_CYCLES | {c[n] / wc:.3f} |")
            if c.get("SQ_INSTS_LDS"):
                out.append(f"| SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS | {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_INSTS_LDS']:.3f} |")
            if c.get("SQ_WAVES"):
                for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VALU_TRANS_F32"):
                    if n in c:
                        out.append(f"| {n} per wave | {c[n] / c['SQ_WAVES']:.1f} |")
            out.append("")
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
