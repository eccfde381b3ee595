#!/usr/bin/env python3
"""Per-kernel averages of the SQ counters collected by tools/pmc_stalls.sh."""
import collections
import csv
import glob
import os
import re
import sys


def main():
    src = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
            if not m or not m.group(1).startswith(("k_demod", "k_est", "k_frame")):
                continue
            agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in sorted(agg.items()):
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        print(k)
        for c in sorted(avg):
            print(f"  {c:24s} {avg[c]:.4g}")
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            wc = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if c in avg:
                    print(f"  {c} / WAVE_CYCLES = {avg[c] / wc:.3f}")


if __name__ == "__main__":
    main()
