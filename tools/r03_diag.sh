#!/bin/bash
# Per-wave stamps of the speculative demod (diagnostic build) and SQ counters of the
# current demod kernels.  Every GPU step has its own time limit.
set -o pipefail
# status 2 on any step that failed hard (time limit, crash), 0 otherwise
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/diag
mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
for sf in 7 12; do
  echo "== stamps sf$sf $(date +%T)"
  LORA_MI355X_LIB=$V/stamps.so timeout -k 10 180 python tools/stamps.py $sf > $OUT/stamps_sf$sf.json 2> $OUT/stamps_sf$sf.err || { tail -5 $OUT/stamps_sf$sf.err; exit 2; }
  cat $OUT/stamps_sf$sf.json
done
echo "== ab nosplit $(date +%T)"
LORA_MI355X_LIB=$V/nosplit.so timeout -k 10 300 python bench.py --no-cpu --no-channels --no-fast --no-variants > $OUT/ab_nosplit.json 2> $OUT/ab_nosplit.err || { tail -5 $OUT/ab_nosplit.err; exit 2; }
echo "== kt7 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt7 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/kt7.log 2>&1 || { tail -20 $OUT/kt7.log; exit 2; }
echo "== kt12 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt12 -o run -- python bench.py --steps 6 --warmup 2 --sf12-only > $OUT/kt12.log 2>&1 || { tail -20 $OUT/kt12.log; exit 2; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
           "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"; do
  for cfg in "--no-sf12" "--sf12-only"; do
    i=$((i+1))
    echo "== pmc $i $cfg $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast --no-variants $cfg > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 2; }
  done
done
echo "== done $(date +%T)"
