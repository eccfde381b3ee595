#!/bin/bash
# Counter passes for the SF7 bench workload (one rocprofv3 pass per counter group).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu --no-sf12 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok: $grp"
done
