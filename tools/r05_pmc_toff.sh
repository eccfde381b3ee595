#!/bin/bash
# Round 5: where the symbol pass's t_off != 0 penalty goes - counter passes (one rocprofv3
# --pmc run each) of the SF7 headline (noiseless, t_off = 0) and the SF7 0 dB batch (t_off
# != 0), tools/prof_workload.py.  Summarised by tools/pmc_toff.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/pmc5
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  for cfg in "n:7 none 15625 2" "a:7 0 15625 2"; do
    tag=${cfg%%:*}; args=${cfg#*:}
    echo "== pass $i $tag $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/p${i}$tag -o run -- python3 tools/prof_workload.py $args > $OUT/p${i}$tag.log 2>&1 || { echo "pass $i $tag failed"; tail -3 $OUT/p${i}$tag.log; exit 2; }
  done
done
python3 tools/pmc_toff.py $OUT | tee $OUT/summary.txt
