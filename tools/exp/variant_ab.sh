#!/bin/bash
# A/B of alternative in-tree builds (lora_phy_amd/lib/<variant>/liblora_mi355x.so, selected
# with LORA_MI355X_LIB) on the default bench, no CPU leg.  Usage: variant_ab.sh v1 v2 ...
# ("default" = lora_phy_amd/lib/liblora_mi355x.so).
mkdir -p gpurun_out
L=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
for rep in 1 2; do
for v in "$@"; do
  if [ $v = default ]; then unset LORA_MI355X_LIB; else export LORA_MI355X_LIB=$L/$v/liblora_mi355x.so; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels > gpurun_out/vab_$v.log 2>&1 || { tail -3 gpurun_out/vab_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/vab_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['ms_per_step'],4), [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok'], round(d['extra']['sf12']['ms_per_step'],3), [round(x,3) for x in d['extra']['sf12']['stage_ms']])"
done
done
