#!/bin/bash
# Fused-kernel knobs A/B on the SF7 bench: runs bench once per "VAR=value ..." argument.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fenv
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants \
    --no-sf12 $BENCH_ARGS > gpurun_out/fenv/$i.json 2> gpurun_out/fenv/$i.err || { echo "[$envs] failed"; tail -3 gpurun_out/fenv/$i.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/fenv/$i.json').read().strip().splitlines()[-1])
print('%-40s %8.1f Msym/s %.4f ms/step stages %s ok=%s' % ('$envs', d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok']))"
done
