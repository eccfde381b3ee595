#!/bin/bash
# Round-3 baseline on one MI355X: default bench (CPU leg included), kernel trace of the
# SF7 headline and the SF12 workload alone, SQ stall counters of the demod kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/base
mkdir -p $OUT
step() { echo "== $1 $(date +%T)"; }
step bench
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
step kt7
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt7 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/kt7.log 2>&1 || { tail -20 $OUT/kt7.log; exit 1; }
step kt12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt12 -o run -- python bench.py --steps 6 --warmup 2 --sf12-only > $OUT/kt12.log 2>&1 || { tail -20 $OUT/kt12.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"; do
  for cfg in "--no-sf12" "--sf12-only"; do
    i=$((i+1))
    step "pmc $i $cfg"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast --no-variants $cfg > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; }
  done
done
step done
