#!/bin/bash
# A/B: SF12 LDS passes reading slot-major twiddle copies (default) vs the strided gathers
# from the natural table (LORA_MI355X_TWT=0).  GPU suite first.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for v in 1 0; do
  LORA_MI355X_TWT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels --no-fast > gpurun_out/twt_$v.log 2>&1 || { tail -5 gpurun_out/twt_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/twt_$v.log').read().strip().splitlines()[-1]);e=d['extra']['sf12'];print('twt=$v', round(d['ms_per_step'],4), [round(x,4) for x in d['config']['stage_ms']], round(e['ms_per_step'],3), [round(x,3) for x in e['stage_ms']], e['symbols_ok'])"
done
done
