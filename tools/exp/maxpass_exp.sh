#!/bin/bash
# Experiment: frame-max pass (stage 0) - nontemporal loads (kept: 8 % faster than plain loads at SF7, 4 % at SF12) and the
# samples-per-block knob (LORA_MI355X_MAXCHUNK).
mkdir -p gpurun_out
L=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
run() {
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels > gpurun_out/mx_$1.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/mx_$1.log').read().strip().splitlines()[-1]);print('$1', round(d['ms_per_step'],4), [round(x,4) for x in d['config']['stage_ms']], d['config']['symbols_ok'], [round(x,3) for x in d['extra']['sf12']['stage_ms']])"
}
for rep in 1 2; do
  unset LORA_MI355X_LIB; run default
  LORA_MI355X_MAXCHUNK=6144 run mc6144
  LORA_MI355X_MAXCHUNK=8448 run mc8448
  LORA_MI355X_MAXCHUNK=2048 run mc2048
done
