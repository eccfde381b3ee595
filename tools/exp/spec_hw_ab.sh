#!/bin/bash
# Speculative pipeline: hardware-rotation demod + certification (LORA_MI355X_SPEC_HW=1,
# default) vs glibc-sincosf demod (0), SF7 headline / sync 0xFF / AWGN 0 dB and SF12.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/spec
for rep in 1 2; do
for hw in 1 0; do
  LORA_MI355X_SPEC_HW=$hw timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast \
    --no-sf12 > gpurun_out/spec/hw7_$hw.json 2> gpurun_out/spec/hw7_$hw.err || { echo "sf7 $hw failed"; tail -3 gpurun_out/spec/hw7_$hw.err; exit 1; }
  LORA_MI355X_SPEC_HW=$hw timeout -k 10 200 python bench.py --steps 6 --warmup 2 --sf12-only \
    > gpurun_out/spec/hw12_$hw.json 2> gpurun_out/spec/hw12_$hw.err || { echo "sf12 $hw failed"; tail -3 gpurun_out/spec/hw12_$hw.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/spec/hw7_$hw.json').read().strip().splitlines()[-1])
c=d['config']; e=d['extra']
print('SF7  HW=$hw %8.1f Msym/s %.4f ms/step stages %s ok=%s fix=%s | ff %.1f fix=%s | awgn %.1f fix=%s' % (d['value'], d['ms_per_step'], [round(x,4) for x in c['stage_ms']], c['symbols_ok'], c['spec_recomputed_per_step'], e['sync_ff_sf7']['value_all_ranks_msym_s'], e['sync_ff_sf7']['spec_recomputed_per_step'], e['awgn_0db_sf7']['value_all_ranks_msym_s'], e['awgn_0db_sf7']['spec_recomputed_per_step']))
d=json.loads(open('gpurun_out/spec/hw12_$hw.json').read().strip().splitlines()[-1])
print('SF12 HW=$hw %8.2f Msym/s %.3f ms/step stages %s ok=%s fix=%s' % (d['msym_s_data'], d['ms_per_step'], [round(x,3) for x in d['stage_ms']], d['symbols_ok'], d['spec_recomputed_per_step']))"
done; done
