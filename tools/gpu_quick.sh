#!/bin/bash
# Quick GPU check used during development: parity tests + short bench (SF7 + SF12).
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu "$@" > gpurun_out/bench.log 2>&1
echo "bench rc=$?"
