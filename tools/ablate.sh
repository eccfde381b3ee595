#!/bin/bash
# Profiling-only: time the SF7/SF12 demod kernel with parts removed (results invalid).
mkdir -p gpurun_out
for ab in 0 1 2 3 4 7; do
  LORA_MI355X_ABLATE=$ab timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu > gpurun_out/abl_$ab.log 2>&1 || exit 1
  echo "ablate=$ab done"
done
