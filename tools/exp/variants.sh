#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the SF7 bench workload:
# VARIANTS="main noest ..." bash tools/exp/variants.sh [extra bench args]
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/var
V=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then lib=$V/liblora_mi355x.so; else lib=$V/variants/$v.so; fi
  LORA_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels \
    --no-fast --no-variants --no-sf12 "$@" > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { echo "$v failed"; tail -3 gpurun_out/var/$v.err; exit 1; }
  python -c "
import json,sys
d=json.loads(open('gpurun_out/var/$v.json').read().strip().splitlines()[-1])
print('%-10s %8.1f Msym/s %.4f ms/step stages %s ok=%s' % ('$v', d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok']))"
done
