#!/bin/bash
# fused vs three-launch on the SF7 bench and the configs[4] (S=16) line
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fab
for v in 1 0; do
  if [ $v = 1 ]; then e=""; else e="LORA_MI355X_FUSED=0"; fi
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-fast --no-variants --no-sf12 $BENCH_ARGS \
    > gpurun_out/fab/$v.json 2> gpurun_out/fab/$v.err || { tail -3 gpurun_out/fab/$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/fab/$v.json').read().strip().splitlines()[-1])
c=d['extra'].get('channels',{})
print('fused=$v SF7 %.1f Msym/s %.4f ms stages %s ok=%s | S16 %.1f Msym/s %.3f ms ok=%s' % (d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok'], c.get('value_all_ranks_msym_s',0), c.get('ms_per_step',0), c.get('symbols_ok_all_frames')))"
done
