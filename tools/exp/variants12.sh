#!/bin/bash
# A/B of library variants on the SF12 bench workload (--sf12-only), interleaved twice.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/var12
V=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
for rep in 1 2; do
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then lib=$V/liblora_mi355x.so; else lib=$V/variants/$v.so; fi
  LORA_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${STEPS:-6} --warmup 2 --sf12-only "$@" \
    > gpurun_out/var12/$v.json 2> gpurun_out/var12/$v.err || { echo "$v failed"; tail -3 gpurun_out/var12/$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/var12/$v.json').read().strip().splitlines()[-1])
print('%-10s %7.2f Msym/s %.3f ms/step stages %s ok=%s' % ('$v', d['msym_s_data'], d['ms_per_step'], [round(x,3) for x in d['stage_ms']], d['symbols_ok']))"
done; done
