#!/bin/bash
# Round measurement on one MI355X: GPU parity tests, smoke, default bench (with CPU
# baseline), rocprofv3 kernel-trace stats, and HBM counter passes for SF7 and SF12.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/round
mkdir -p $OUT
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
step bench
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
step kernel-trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-channels > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
for grp in FETCH_SIZE WRITE_SIZE; do
  for cfg in "--no-sf12" "--sf12-only"; do
    tag=$(echo "$grp$cfg" | tr -d '-')
    step "pmc $tag"
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$tag -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast $cfg > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
  done
done
for cfg in "--no-sf12" "--sf12-only"; do
  tag=$(echo "VALU$cfg" | tr -d '-')
  step "pmc $tag"
  timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $OUT/pmc_$tag -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-channels --no-fast $cfg > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
done
step "valu issue rates"
if [ -x ./tools/micro/pk_rate ]; then timeout -k 10 120 ./tools/micro/pk_rate > $OUT/valu_rates.txt 2>&1 || exit 1; fi
step done
