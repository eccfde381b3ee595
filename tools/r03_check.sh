#!/bin/bash
# GPU check of the working tree: the GPU test suite, then the default bench.
# Test failures (pytest exit 1) are reported and the bench still runs; anything else
# (a time limit, an abort, a crash) stops the call with status 2 so no further GPU step
# starts.  Usage: tools/r03_check.sh [pytest selection...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/check
mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head -20
[ $rc -le 1 ] || { echo "pytest status $rc: stopping"; exit 2; }
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo "== done $(date +%T)"
exit $rc
