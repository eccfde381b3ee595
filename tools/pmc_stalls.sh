#!/bin/bash
# SQ stall / instruction breakdown of the demod and estimate kernels, SF7 and SF12
# (two counter passes each; rocprofv3 --pmc, counters only).  Summary: tools/pmc_stalls.py.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/stalls
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  for cfg in "--sf12-only --sf12-frames 4000" "--no-sf12 --frames 15625"; do
    tag=p${i}_$(echo $cfg | cut -c3-6)
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/$tag -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels $cfg > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  done
done
python tools/pmc_stalls.py $OUT
