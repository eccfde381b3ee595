#!/bin/bash
# Profiling-only ablations of the speculative demod kernel (results invalid): variants
# built with tools/build_variant.sh xN "-DLORA_SPEC_ABLX=N" (bits: 1 no rotation, 4 no IQ
# loads, 8 one dechirp-table value, 16 no LDS transposes, 32 one twiddle per group) and
# xs "-DLORA_SPEC_ABL=1" (no window max / margin).  SF7 then SF12 demod stage ms.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sabl
V=lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib
for v in ${VARIANTS:-main x1 x4 x8 x12 x16 x32 x48 xs}; do
  if [ "$v" = main ]; then lib=$V/liblora_mi355x.so; else lib=$V/variants/$v.so; fi
  LORA_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels \
    --no-fast --no-variants --no-sf12 > gpurun_out/sabl/$v.json 2> gpurun_out/sabl/$v.err || { echo "$v failed"; tail -3 gpurun_out/sabl/$v.err; exit 1; }
  LORA_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 6 --warmup 2 --sf12-only \
    > gpurun_out/sabl/${v}_12.json 2> gpurun_out/sabl/${v}_12.err || { echo "$v sf12 failed"; tail -3 gpurun_out/sabl/${v}_12.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/sabl/$v.json').read().strip().splitlines()[-1])
e=json.loads(open('gpurun_out/sabl/${v}_12.json').read().strip().splitlines()[-1])
print('%-6s SF7 %.4f ms/step stages %s | SF12 %.3f ms/step stages %s' % ('$v', d['ms_per_step'], [round(x,4) for x in d['config']['stage_ms']], e['ms_per_step'], [round(x,3) for x in e['stage_ms']]))"
done
