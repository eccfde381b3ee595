#!/bin/bash
# A/B: demod with phases past the fast sincos range (sync 0xFF) old vs new library.
mkdir -p gpurun_out
L=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/liblora_mi355x.so
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --sync 0xff > gpurun_out/sync_new.log 2>&1 || exit 1
cp $L /tmp/new.so && cp tools/exp/lib_old.so $L
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --sync 0xff > gpurun_out/sync_old.log 2>&1; rc=$?
cp /tmp/new.so $L
exit $rc
