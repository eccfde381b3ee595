"""Summarise rocprofv3 counter CSVs (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel."""
import collections
import csv
import re
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc/p*/run_counter_collection.csv"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(pat)):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if any(x in k for x in ("demod", "frame_max", "estimate")):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}")
