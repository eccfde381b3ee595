#!/usr/bin/env python3
"""Per-kernel SQ counters of tools/r04_pmc.sh's passes (<dir>/<variant>_g<k>_sf<sf>/), averaged
over dispatches, one table row per (variant, sf, kernel); derived: VALU instructions per
wave-cycle, bank-conflict cycles per LDS instruction.  usage: pmc_table.py <dir>"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
vals = collections.defaultdict(dict)  # (variant, sf, kernel) -> counter -> mean
for sub in sorted(glob.glob(os.path.join(d, "*_g*_sf*"))):
    m = re.match(r"(.+)_g\d+_sf(\d+)$", os.path.basename(sub))
    if not m:
        continue
    var, sf = m.group(1), int(m.group(2))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            km = re.search(r"(k_\w+)(<[^>]*>)?", r["Kernel_Name"])
            k = km.group(0) if km else r["Kernel_Name"][:40]
            acc[(k, r["Counter_Name"])][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
    for (k, c), per in acc.items():
        vals[(var, sf, k)][c] = sum(per.values()) / len(per)
for (var, sf, k), c in sorted(vals.items()):
    if "spec_demod" not in k and "cert" not in k and "est_" not in k and "spec_fix" not in k:
        continue
    line = "%-8s sf%-2d %-36s" % (var, sf, k[:36])
    for name in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
                 "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE", "SQ_INSTS_SALU",
                 "SQ_INSTS_VALU_TRANS_F32", "SQ_IFETCH"):
        if name in c:
            line += " %s=%.4g" % (name.replace("SQ_", ""), c[name])
    if "SQ_INSTS_LDS" in c and "SQ_LDS_BANK_CONFLICT" in c and c["SQ_INSTS_LDS"]:
        line += " conflict/lds=%.2f" % (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"])
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        line += " waitinst/wave=%.2f" % (c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"])
    print(line)
