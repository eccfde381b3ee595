#!/bin/bash
# Default-length bench (no CPU leg) twice, summarised: step time vs kernel stage times.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/st
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/st/b$rep.json 2> gpurun_out/st/b$rep.err || { tail -5 gpurun_out/st/b$rep.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/st/b$rep.json').read().strip().splitlines()[-1])
e=d['extra']['sf12']; c=d['extra']['channels']
print('SF7 %.1f Msym/s %.4f ms/step stages %s | SF12 %.2f %.3f ms | channels %.0f | steps %d' % (d['value'], d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], e['value_all_ranks_msym_s'], e['ms_per_step'], c['value_all_ranks_msym_s'], d['steps']))"
done
