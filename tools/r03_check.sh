#!/bin/bash
# GPU check of the working tree: the GPU test suite (stops at the first failure), then the
# default bench.  Usage: tools/r03_check.sh [pytest selection...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/check
mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; exit 1; }
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo "== done $(date +%T)"
