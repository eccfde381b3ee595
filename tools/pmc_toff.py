"""Summary of tools/r05_pmc_toff.sh: per counter, the k_spec_demod launches' mean value for
the noiseless (t_off = 0) and the 0 dB (t_off != 0) SF7 batch, and their ratio."""
import csv
import glob
import os
import sys

out = sys.argv[1]
vals = {}
for d in sorted(glob.glob(os.path.join(out, "p*"))):
    if not os.path.isdir(d):
        continue
    tag = d[-1]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = {}
        for row in csv.DictReader(open(f)):
            if "k_spec_demod" not in row.get("Kernel_Name", ""):
                continue
            key = (row["Counter_Name"])
            acc.setdefault(key, {})
            did = row.get("Dispatch_Id", row.get("Correlation_Id", "0"))
            acc[key][did] = acc[key].get(did, 0.0) + float(row["Counter_Value"])
        for k, per in acc.items():
            v = sum(per.values()) / max(len(per), 1)
            vals.setdefault(k, {})[tag] = v
for k in sorted(vals):
    n, a = vals[k].get("n"), vals[k].get("a")
    r = (a / n) if n and a is not None else float("nan")
    print(f"{k:32s} t_off=0 {n:14.4g}  0dB {a if a is not None else float('nan'):14.4g}  ratio {r:.4f}")
