#!/bin/bash
# Speculative-pipeline check of the working tree: the spec / scale / parity / golden GPU
# tests, the alignment experiment, then the full bench without the CPU leg.  Hard failures
# stop the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/spec
mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dropin.py -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; grep -E "^(FAILED|ERROR)|recomputed" $OUT/pytest.log | head -20
[ $rc -le 1 ] || { echo "pytest status $rc: stopping"; exit 2; }
echo "== align $(date +%T)"
timeout -k 10 300 python tools/exp/align_exp.py 7 > $OUT/align7.txt 2>&1 || { tail -5 $OUT/align7.txt; exit 2; }
grep cfo $OUT/align7.txt
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 2; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/spec/bench.json"))
print("headline", round(d["value"], 1), round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 3), "stages", [round(x, 4) for x in d["config"]["stage_ms"]])
for k, v in d["extra"].items():
    if isinstance(v, dict):
        print(" ", k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in v.items()
                       if x in ("ms_per_step", "ms_per_call", "ratio_to_headline", "spec_recomputed_per_step", "value_all_ranks_msym_s", "stage_ms")})
PY
echo "== done $(date +%T)"
exit $rc
