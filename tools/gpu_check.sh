#!/bin/bash
# Development check: full GPU test suite, then a short bench (SF7 + SF12, no CPU leg).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("SF7", d["value"], d["ms_per_step"], d["config"]["stage_ms"], d["config"]["symbols_ok"], d["roofline"]["frac"])
for k, v in d["extra"].items():
    print(k, v.get("ms_per_step"), v.get("value_all_ranks_msym_s"), v.get("stage_ms"), v.get("symbols_ok", v.get("symbols_ok_first64")))
PY
