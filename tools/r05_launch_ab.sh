#!/bin/bash
# Round 5: the bench headline with the step replayed as a HIP graph (default) against
# plan.run per step (eager launches), alternated on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/r05; mkdir -p $OUT
for i in 1 2 3; do
  for l in graph eager; do
    timeout -k 10 300 python3 bench.py --launch $l --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/launch_$l$i.json 2> $OUT/launch_$l$i.err || exit 2
    python3 -c "import json,sys; d=json.loads(open('$OUT/launch_$l$i.json').read().strip().splitlines()[-1]); print('$l', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
