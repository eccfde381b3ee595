#!/bin/bash
# Experiment: LEGACY chunk count of the fused frame-max schedule (LORA_MI355X_CHUNKS).
mkdir -p gpurun_out
for c in 1 2 4 8; do
  LORA_MI355X_CHUNKS=$c timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ch_$c.log 2>&1 || exit 1
done
