#!/usr/bin/env python3
"""A pipeline step's timeline from a rocprofv3 kernel trace (PART=trace bash tools/record.sh: gpurun_out/rec/prof/bench7 /
kt7 directories): for every run of consecutive pipeline kernels that starts with the
pre-pass, each kernel's duration and the gap before it, then the medians over the steps.
usage: step_timeline.py <trace dir> [first kernel prefix (default k_est)]"""
import csv
import glob
import os
import re
import statistics
import sys


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    d = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_est"
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[1])
    steps, cur = [], None
    for k, b, e in rows:
        if k.startswith(first):
            cur = [(k, b, e)]
            steps.append(cur)
        elif cur is not None and k.startswith(("k_spec", "k_cert", "k_est")):
            cur.append((k, b, e))
        else:
            cur = None
    shape = max(set(tuple(x[0] for x in s) for s in steps), key=lambda t: sum(
        1 for s in steps if tuple(x[0] for x in s) == t))
    steps = [s for s in steps if tuple(x[0] for x in s) == shape]
    print(f"{len(steps)} steps of {' -> '.join(shape)}")
    for i, k in enumerate(shape):
        dur = statistics.median(s[i][2] - s[i][1] for s in steps) / 1e3
        gap = statistics.median(s[i][1] - s[i - 1][2] for s in steps) / 1e3 if i else 0.0
        print(f"  {k:16s} gap before {gap:6.2f} us  duration {dur:8.2f} us")
    span = statistics.median(s[-1][2] - s[0][1] for s in steps) / 1e3
    nxt = [steps[i + 1][0][1] - steps[i][-1][2] for i in range(len(steps) - 1)]
    print(f"  first start -> last end {span:.2f} us; gap to the next step {statistics.median(nxt) / 1e3 if nxt else 0:.2f} us")


if __name__ == "__main__":
    main()
