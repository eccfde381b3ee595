#!/bin/bash
# GPU parity suite, then A/B of the default library against variants (VARS) on SF7 + SF12.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tw
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tw/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/tw/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="main $1 main $1" bash tools/exp/spec_ablate.sh
