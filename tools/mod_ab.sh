#!/bin/bash
# Same-box A/B of the drop-in packet timing (tests/native/dropin_timing) for a modulator change:
# the modulator tests, then three alternated runs of the libraries saved under
# lora_phy_amd/lib/variants/base (cp liblora_mi355x.so liblora_phy.so there before the change)
# and of the in-tree build.  gpurun from the repo root: bash tools/mod_ab.sh
mkdir -p gpurun_out/rec
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k modulator tests/test_gpu_dropin.py tests/test_gpu_bandwidth.py > gpurun_out/rec/pytest_mod.log 2>&1; rc=$?
tail -2 gpurun_out/rec/pytest_mod.log
[ $rc = 0 ] || exit $rc
B=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants/base
for r in 1 2 3; do
  LD_LIBRARY_PATH=$B timeout -k 10 100 tests/native/dropin_timing 300 > gpurun_out/rec/mod_base_$r.log || exit 1
  timeout -k 10 100 tests/native/dropin_timing 300 > gpurun_out/rec/mod_new_$r.log || exit 1
done
for f in gpurun_out/rec/mod_*_*.log; do echo $f; python -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'): r=json.loads(l); print(r['sf'], r['modulate_us'], r['demodulate_us'], r['pps'])"; done
