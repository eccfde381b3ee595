#!/bin/bash
# Effective shader clock of the SF12 symbol pass per library variant: GRBM_GUI_ACTIVE
# (cycles, summed over XCDs) with the kernel trace's durations, one rocprofv3 --pmc pass each.
# usage: tools/clk_probe.sh name [name...]   (default = the tree's library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/clk; mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
for v in default "$@"; do
  if [ $v = default ]; then lib=""; else lib=$V/$v.so; fi
  LORA_MI355X_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv \
    -d $OUT/$v -o run -- python3 tools/prof_workload.py ${SF:-12} none ${FRAMES:-4000} 4 > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 2; }
done
python3 - $OUT "$@" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in ["default"] + sys.argv[2:]:
    dur = {}
    for f in glob.glob(os.path.join(out, v, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(out, v, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, c in sorted(acc.items(), key=lambda kv: int(kv[0])):
        k, ns = dur.get(d, ("?", 0))
        if "k_spec_demod" in k and ns:
            print(v, k[k.find("k_spec"):k.find("k_spec") + 34], "us %.1f" % (ns / 1e3),
                  "GUI_ACTIVE/XCD/ns %.3f" % (c["GRBM_GUI_ACTIVE"] / 8 / ns), "GRBM_COUNT/XCD/ns %.3f" % (c["GRBM_COUNT"] / 8 / ns))
PY
