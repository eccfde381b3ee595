#!/bin/bash
mkdir -p gpurun_out
for c in 4096 8448 16384 2048; do
  LORA_MI355X_MAXCHUNK=$c timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels > gpurun_out/mc_$c.log 2>&1 || exit 1
done
