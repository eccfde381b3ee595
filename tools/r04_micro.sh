#!/bin/bash
# Round 4: VALU issue-rate micro-benchmark + a baseline bench of the tree (no CPU leg).
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/micro/valu_rate > gpurun_out/r04/valu_rate.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu --no-channels --no-fast --no-variants \
  > gpurun_out/r04/bench_base.json 2> gpurun_out/r04/bench_base.err || exit $?
echo done
