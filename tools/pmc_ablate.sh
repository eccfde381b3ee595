#!/bin/bash
# Instruction counts of the SF7 demod kernel under each profiling ablation (results invalid).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcab
for ab in 0 1 2 4 7; do
  LORA_MI355X_ABLATE=$ab timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_WAVES --output-format csv -d gpurun_out/pmcab/a$ab -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-sf12 > gpurun_out/pmcab/a$ab.log 2>&1 || { echo "ablate $ab failed"; exit 1; }
done
