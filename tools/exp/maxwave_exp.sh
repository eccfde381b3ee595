#!/bin/bash
# A/B: one wave per short frame in the frame-max pass (k_frame_max_wave, default) vs
# one block per frame (LORA_MI355X_MAXWAVE=0), on configs[4] (18-symbol SF7 frames).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for v in 1 0; do
  LORA_MI355X_MAXWAVE=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu --no-sf12 --no-fast > gpurun_out/mw_$v.log 2>&1 || { tail -5 gpurun_out/mw_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/mw_$v.log').read().strip().splitlines()[-1]);c=d['extra']['channels'];print('maxwave=$v', round(d['ms_per_step'],4), round(c['ms_per_step'],3), round(c['value_all_ranks_msym_s'],1), c['symbols_ok_first64'])"
done
done
