#!/bin/bash
# Fast-rotation mode: its GPU tests (with the measured agreement printed), then the full
# GPU suite.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast_rotation.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/fr_pytest.log 2>&1; rc=$?
grep -E 'SNR|PASS|FAIL|Error|assert' gpurun_out/fr_pytest.log | head -40; tail -3 gpurun_out/fr_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
