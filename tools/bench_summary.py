#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (usage: bench_summary.py <bench.json>)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"SF7 {d['value']:.1f} Msym/s  {d['ms_per_step']:.4f} ms/step  stages {[round(x, 4) for x in d['config']['stage_ms']]}  "
      f"frac {r['frac']:.4f}  pipeline {r['pipeline']['pipeline_frac']:.4f}  probe {r['hbm_probe']['d2d_copy_gbs']:.0f}")
for k, v in d["extra"].items():
    if not isinstance(v, dict):
        continue
    keys = ("ms_per_step", "stage_ms", "pipeline_frac", "symbol_pass_frac", "spec_recomputed_frac", "ms_per_call",
            "roofline_frac", "value_all_ranks_msym_s", "symbol_pass_counter_over_algorithmic")
    out = {kk: (round(v[kk], 4) if isinstance(v[kk], float) else v[kk]) for kk in keys if kk in v and v[kk] is not None}
    if "stage_ms" in out:
        out["stage_ms"] = [round(x, 4) for x in out["stage_ms"]]
    if "roofline" in v:
        out["frac"] = round(v["roofline"]["frac"], 4)
        out["pipeline_frac"] = round(v["roofline"]["pipeline"]["pipeline_frac"], 4)
    par = v.get("parity") or (v.get("cpu_baseline") or {}).get("parity_ok")
    if isinstance(par, dict):
        out["parity_ok"] = par.get("parity_ok", par.get("symbol_agreement_with_exact"))
    elif par is not None:
        out["parity_ok"] = par
    if "three_launch" in v:
        out["three_launch_ms"] = round(v["three_launch"]["ms_per_step"], 4)
    print(k, out)
c = d.get("cpu_baseline") or {}
print("cpu", c.get("value"), c.get("cores"), c.get("kind"), "reference_parity", (c.get("reference_parity") or {}).get("parity_ok"))
print("headline parity", d["config"].get("parity"))
