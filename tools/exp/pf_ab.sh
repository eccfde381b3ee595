#!/bin/bash
# SF7 speculative demod variants: k_demod_fast (STREAM=0), LDS-DMA stream kernel (default),
# register-prefetch kernel (PF=1), and stream-kernel ablation libraries if present.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pf
V=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants --no-sf12 \
    > gpurun_out/pf/$n.json 2> gpurun_out/pf/$n.err || { echo "$n failed"; tail -3 gpurun_out/pf/$n.err; return 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/pf/$n.json').read().strip().splitlines()[-1])
print('%-10s %8.1f Msym/s %.4f ms/step stages %s ok=%s' % ('$n', d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok']))"
}
for rep in 1 2; do
run fast LORA_MI355X_STREAM=0 || exit 1
run stream LORA_MI355X_STREAM=1 || exit 1
run pf LORA_MI355X_PF=1 || exit 1
run pf_wg3 LORA_MI355X_PF=1 LORA_MI355X_PF_WG=3 || exit 1
done
for v in ${VARIANTS:-}; do run $v LORA_MI355X_LIB=$PWD/$V/variants/$v.so || exit 1; done
