#!/bin/bash
# A/B: estimate transforms of symbols 0 and 1 in lockstep (default) vs one after the
# other (lib variant built with -DLORA_EST_PAIR=0).  GPU suite first.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/exp/variant_ab.sh default nopair
