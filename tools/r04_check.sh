#!/bin/bash
# Round 4 development check on the GPU: micro-benchmark (optional), the pipeline's parity
# tests, then a same-box A/B of the tree against variant libraries.
# usage: tools/r04_check.sh [variant...]   (MICRO=1 runs tools/micro/valu_rate first;
#        TESTS="tests/..." overrides the test selection; REPS=n)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r04
if [ -n "$MICRO" ]; then timeout -k 10 200 tools/micro/valu_rate > gpurun_out/r04/valu_rate2.txt 2>&1 || exit $?; fi
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_spec.py tests/test_gpu_scale.py} \
    > gpurun_out/r04/pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
[ $# -gt 0 ] || exit 0
REPS=${REPS:-2} tools/r03_ab.sh "$@" > gpurun_out/r04/ab.txt 2>&1; rc=$?
cat gpurun_out/r04/ab.txt
exit $rc
