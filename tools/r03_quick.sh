#!/bin/bash
# Quick GPU iteration: the alloc probe, the drop-in / spec / parity / scale tests, then the
# headline bench of the working tree and of each variant library named on the command
# line (lora_phy_amd/lib/variants/<name>.so), interleaved.  Hard failures stop the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/quick
mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
if [ -x tools/micro/pk_rate ]; then echo "== pk_rate"; timeout -k 10 60 ./tools/micro/pk_rate || exit 2; fi
echo "== probe $(date +%T)"
timeout -k 10 120 ./tests/native/alloc_probe > $OUT/probe.json 2>&1; rc=$?
cat $OUT/probe.json; [ $rc -le 1 ] || { echo "probe status $rc"; exit 2; }
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_golden.py -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head
[ $rc -le 1 ] || { echo "pytest status $rc: stopping"; exit 2; }
for rep in 1 2; do
  for v in default "$@"; do
    echo "== bench $v rep $rep $(date +%T)"
    if [ $v = default ]; then lib=""; else lib=$V/$v.so; fi
    LORA_MI355X_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-channels --no-fast --no-variants > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || { tail -5 $OUT/bench_${v}_$rep.err; exit 2; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$rep.json')); e=d['extra']['sf12']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), 'demodGBs', round(d['roofline']['achieved']), 'sf12', round(e['ms_per_step'],3), round(e['roofline']['achieved']))"
  done
done
if [ -n "$QUICK_FULL" ]; then
  echo "== full bench (no cpu) $(date +%T)"
  timeout -k 10 600 python bench.py --no-cpu > $OUT/bench_full.json 2> $OUT/bench_full.err || { tail -5 $OUT/bench_full.err; exit 2; }
  python - <<'PY'
import json
d = json.load(open("gpurun_out/quick/bench_full.json"))
print("headline", round(d["value"], 1), round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 3))
for k, v in d["extra"].items():
    if isinstance(v, dict):
        print(" ", k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in v.items()
                       if x in ("ms_per_step", "ms_per_call", "ratio_to_headline", "spec_recomputed_per_step", "value_all_ranks_msym_s")})
PY
fi
echo "== done $(date +%T)"
