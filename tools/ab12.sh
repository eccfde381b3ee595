#!/bin/bash
# Same-box A/B of the SF12 workload alone (bench.py --sf12-only) against variant libraries
# (ablations may give wrong symbols: the line's verification field shows it).
# usage: tools/ab12.sh name [name...]   (REPS=n)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/ab12; mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
for rep in $(seq 1 ${REPS:-2}); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=""; else lib=$V/$v.so; fi
    LORA_MI355X_LIB=$lib timeout -k 10 300 python bench.py --sf12-only --no-cpu > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail -5 $OUT/${v}_$rep.err; exit 2; }
    python - $OUT/${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 4), [round(x, 4) for x in d.get("stage_ms", [])], d.get("verified", d.get("symbols_ok")), flush=True)
PY
  done
done
