#!/bin/bash
# Round 5: the drop-in's per-packet path on the GPU - its tests (the reference's
# performance_test on the drop-in beside the reference's own build, the AQL timeline
# probe), then the kernel trace of the timing probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu ${DTESTS:-tests/test_gpu_dropin.py} \
  > gpurun_out/r05/dropin_pytest.log 2>&1; rc=$?
grep -E "pps|dropin_timing|passed|failed|Error" gpurun_out/r05/dropin_pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_dropin -o dropin -- \
    tests/native/dropin_timing 100 > gpurun_out/r05/prof_dropin.log 2>&1; rc=$?
  tail -5 gpurun_out/r05/prof_dropin.log
fi
exit $rc
