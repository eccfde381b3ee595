#!/bin/bash
# Kernel timeline of a short SF7 bench run (for launch-gap analysis).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels > gpurun_out/gap_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-sf12 --no-channels > gpurun_out/gap.log 2>&1 || exit 1
