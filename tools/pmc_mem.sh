#!/bin/bash
# Memory-pipeline counters of the demod kernel (SF7 default; SF=12 bash tools/pmc_mem.sh
# for SF12): TA busy, L2 hit/miss, TCP stalls, for the default kernel and the no-IQ-load
# ablation (LORA_MI355X_ABLATE=4).  A pass whose counters this GPU lacks is reported and
# skipped.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
SF=${SF:-7}
OUT=gpurun_out/pmcmem$SF
mkdir -p $OUT
if [ "$SF" = 12 ]; then CFG="--sf12-only --sf12-frames 4000"; else CFG="--no-sf12"; fi
for ab in 0 4; do
  i=0
  for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" \
             "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
             "TD_BUSY_avr TCP_TCC_READ_REQ_sum" \
             "SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
    i=$((i+1))
    LORA_MI355X_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/a${ab}_p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast $CFG > $OUT/a${ab}_p$i.log 2>&1 || { echo "pass a${ab}_p$i ($grp) failed"; tail -2 $OUT/a${ab}_p$i.log; }
  done
done
python - "$OUT" <<'PY'
import csv, glob, collections, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    ab = re.search(r"/a(\d)_p", f).group(1)
    for r in csv.DictReader(open(f)):
        if "k_demod_fast" in r["Kernel_Name"]:
            agg[ab][r["Counter_Name"]].append(float(r["Counter_Value"]))
for ab, d in sorted(agg.items()):
    print("ablate", ab, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
