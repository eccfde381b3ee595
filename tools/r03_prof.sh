#!/bin/bash
# Round-3 profiles of the current tree: rocprofv3 kernel traces of the SF7 headline, the
# SF7 -10 dB worst case and the SF12 workload, each alone (tools/prof_workload.py), then SQ
# counter passes for SF7 and SF12.  Hard failures stop the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/prof
mkdir -p $OUT
for cfg in "kt7 7 none 15625 20" "kt7n10 7 -10 15625 20" "kt12 12 none 15625 6"; do
  set -- $cfg
  echo "== $1 $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o run -- python3 tools/prof_workload.py $2 $3 $4 $5 > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 2; }
  tail -1 $OUT/$1.log
done
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
           "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"; do
  for cfg in "7 none 15625 2" "12 none 4000 2"; do
    i=$((i+1))
    echo "== pmc $i sf${cfg%% *} $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 tools/prof_workload.py $cfg > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 2; }
  done
done
# HBM traffic: FETCH_SIZE and WRITE_SIZE in passes of their own (TCC slots), per workload
for cfg in "7 none 15625 2" "12 none 4000 2"; do
  sf=${cfg%% *}
  for c in FETCH_SIZE WRITE_SIZE; do
    tag=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    echo "== $c sf$sf $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$tag$sf -o run -- python3 tools/prof_workload.py $cfg > $OUT/pmc_$tag$sf.log 2>&1 || { echo "$c pass failed"; tail -3 $OUT/pmc_$tag$sf.log; exit 2; }
  done
done
echo "== done $(date +%T)"
