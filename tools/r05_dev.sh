#!/bin/bash
# Round 5 development check on the GPU: the chosen GPU tests, then a same-box A/B of the
# tree against variant libraries (tools/r05_ab.py).
# usage: TESTS="tests/..." AB="nodtab ..." WORK=sf7,awgn0 tools/r05_dev.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r05
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-700} python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/r05/dev_pytest.log 2>&1; rc=$?
  grep -E "pps|dropin_timing|passed|failed|Error|error" gpurun_out/r05/dev_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB" ]; then
  timeout -k 10 ${ABTIME:-600} python -u tools/r05_ab.py --reps ${REPS:-3} --work ${WORK:-sf7,awgn0,awgn10} default $AB \
    > gpurun_out/r05/ab.txt 2>&1; rc=$?
  cat gpurun_out/r05/ab.txt
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
