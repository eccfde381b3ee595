#!/bin/bash
# Rotation-recurrence A/B: GPU parity suite on the default library, then speculative
# demod ablations (spec_ablate.sh) with the r0 (per-point sin/cos) variant beside them,
# then the SF7 persistent-variant A/B (pf_ab.sh).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rr
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rr/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/rr/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-main r0 x1 x4 x8 x16 x32}" bash tools/exp/spec_ablate.sh || exit 1
bash tools/exp/pf_ab.sh
