#!/bin/bash
# A/B the working library against tools/exp/lib_old.so on the same box: bench args "$@".
mkdir -p gpurun_out
L=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/liblora_mi355x.so
cp $L /tmp/new.so
for v in new old new old; do
  if [ $v = old ]; then cp tools/exp/lib_old.so $L; else cp /tmp/new.so $L; fi
  timeout -k 10 300 python bench.py --no-cpu --no-channels "$@" >> gpurun_out/ab_$v.log 2>&1 || { cp /tmp/new.so $L; exit 1; }
done
cp /tmp/new.so $L
