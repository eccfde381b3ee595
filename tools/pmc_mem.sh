#!/bin/bash
# Memory-pipeline counters of the SF7 demod kernel: TA busy (address/fragment processing)
# and L2 hit/miss, for the default kernel and the no-IQ-load ablation (LORA_MI355X_ABLATE=4).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmcmem
mkdir -p $OUT
for ab in 0 4; do
  i=0
  for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    LORA_MI355X_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/a${ab}_p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast --no-sf12 > $OUT/a${ab}_p$i.log 2>&1 || { echo "pass a${ab}_p$i failed"; tail -5 $OUT/a${ab}_p$i.log; }
  done
done
python - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcmem/*/run_counter_collection.csv"):
    ab = re.search(r"/a(\d)_p", f).group(1)
    for r in csv.DictReader(open(f)):
        if "k_demod_fast" in r["Kernel_Name"]:
            agg[ab][r["Counter_Name"]].append(float(r["Counter_Value"]))
for ab, d in sorted(agg.items()):
    print("ablate", ab, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
