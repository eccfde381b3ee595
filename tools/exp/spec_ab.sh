#!/bin/bash
# Speculative pipeline A/B: SF7 headline and SF12 workloads with LORA_MI355X_SPEC=1 / 0.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/spec
for rep in 1 2; do
for sp in 1 0; do
  LORA_MI355X_SPEC=$sp timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast \
    --no-variants --no-sf12 > gpurun_out/spec/sf7_$sp.json 2> gpurun_out/spec/sf7_$sp.err || { echo "sf7 $sp failed"; tail -3 gpurun_out/spec/sf7_$sp.err; exit 1; }
  LORA_MI355X_SPEC=$sp timeout -k 10 200 python bench.py --steps 6 --warmup 2 --sf12-only \
    > gpurun_out/spec/sf12_$sp.json 2> gpurun_out/spec/sf12_$sp.err || { echo "sf12 $sp failed"; tail -3 gpurun_out/spec/sf12_$sp.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/spec/sf7_$sp.json').read().strip().splitlines()[-1])
print('SF7  SPEC=$sp %8.1f Msym/s %.4f ms/step stages %s ok=%s' % (d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok']))
d=json.loads(open('gpurun_out/spec/sf12_$sp.json').read().strip().splitlines()[-1])
print('SF12 SPEC=$sp %8.2f Msym/s %.3f ms/step stages %s ok=%s' % (d['msym_s_data'], d['ms_per_step'], [round(x,3) for x in d['stage_ms']], d['symbols_ok']))"
done; done
