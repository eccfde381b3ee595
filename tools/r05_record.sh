#!/bin/bash
# Round-5 record on the GPU: PART=tests - the whole -m gpu suite; PART=bench - smoke() then
# the default bench line (every line, CPU legs included).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/r05rec
mkdir -p $OUT
if [ "$PART" = tests ]; then
  timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest_gpu.log 2>&1; rc=$?
  grep -E "pps|dropin_timing|passed|failed|error" $OUT/pytest_gpu.log | tail -25
  exit $rc
fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; rc=$?
tail -3 $OUT/bench_default.err
python3 tools/bench_summary.py $OUT/bench_default.json 2>/dev/null | head -40 || head -c 2000 $OUT/bench_default.json
exit $rc
