#!/bin/bash
# Profiling-only: time the SF7/SF12 demod kernel with parts removed (results invalid).
# ABLATE bits: 1 identity rotation (no sincos), 2 skip the pass-1 FFT stages, 4 skip the
# IQ loads.  Prints ms/step and per-stage kernel ms for SF7 and SF12.
mkdir -p gpurun_out
for ab in ${ABLS:-0 1 4 5 8 9 12 7}; do
  LORA_MI355X_ABLATE=$ab timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels --no-fast > gpurun_out/abl_$ab.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abl_$ab.log').read().strip().splitlines()[-1]);print('ablate=$ab', [round(x,4) for x in d['config']['stage_ms']], [round(x,3) for x in d['extra']['sf12']['stage_ms']])"
done
