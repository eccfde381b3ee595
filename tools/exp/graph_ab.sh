#!/bin/bash
# Bench step launch A/B: plan.run per step vs one HIP-graph replay per step (SF7 + SF12).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gab
for rep in 1 2; do for m in eager graph; do
  timeout -k 10 200 python bench.py --launch $m --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants \
    > gpurun_out/gab/$m$rep.json 2> gpurun_out/gab/$m$rep.err || { echo "$m failed"; tail -5 gpurun_out/gab/$m$rep.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/gab/$m$rep.json').read().strip().splitlines()[-1])
e=d['extra']['sf12']
print('%-6s SF7 %.1f Msym/s %.4f ms/step %s ok=%s | SF12 %.2f Msym/s %.3f ms/step ok=%s' % ('$m', d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok'], e['value_all_ranks_msym_s'], e['ms_per_step'], e['symbols_ok']))"
done; done
