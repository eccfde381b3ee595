#!/bin/bash
# Development GPU check: the named test files (default: fused + parity), then a short SF7
# bench with the frame-resident kernel and with it disabled (LORA_MI355X_FUSED=0).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dev
tests=${TESTS:-"tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_capi.py"}
timeout -k 10 400 python -u -m pytest $tests -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/dev/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/dev/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants $BENCH_ARGS \
  > gpurun_out/dev/b_fused.json 2> gpurun_out/dev/b_fused.err || { tail -5 gpurun_out/dev/b_fused.err; exit 1; }
LORA_MI355X_FUSED=0 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast \
  --no-variants $BENCH_ARGS > gpurun_out/dev/b_split.json 2> gpurun_out/dev/b_split.err || exit 1
python - <<'PY'
import json
for k in ("fused", "split"):
    d = json.loads(open(f"gpurun_out/dev/b_{k}.json").read().strip().splitlines()[-1])
    s12 = d["extra"].get("sf12", {})
    print(k, "SF7", round(d["value"], 1), round(d["ms_per_step"], 4), d["config"]["stage_ms"], d["config"]["symbols_ok"],
          "| SF12", s12.get("msym_s_data"), s12.get("ms_per_step"), s12.get("stage_ms"))
PY
