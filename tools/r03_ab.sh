#!/bin/bash
# Same-box A/B of the working tree against variant libraries (lora_phy_amd/lib/variants/
# <name>.so, tools/build_variant.sh or a build of another commit): the bench without the
# CPU leg and configs[4], interleaved, REPS times.  Hard failures stop the call.
# usage: tools/r03_ab.sh name [name...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/ab
mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
for rep in $(seq 1 ${REPS:-3}); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=""; else lib=$V/$v.so; fi
    LORA_MI355X_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-channels --no-fast ${BENCH_ARGS} > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail -5 $OUT/${v}_$rep.err; exit 2; }
    python - $OUT/${v}_$rep.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d["extra"]
r = lambda x: round(x, 4)
line = [sys.argv[2], "sf7", r(d["ms_per_step"]), [r(x) for x in d["config"]["stage_ms"][1:]]]
for k in ("awgn_m10db_sf7", "awgn_0db_sf7", "sync_ff_sf7", "hann_sf7", "long_frames_sf7", "sf12", "awgn_m10db_sf12"):
    if k in e:
        line += [k, r(e[k]["ms_per_step"]), [r(x) for x in e[k].get("stage_ms", [0, 0, 0])[1:]]]
print(*line, flush=True)
PY
  done
done
echo "== done $(date +%T)"
