#!/bin/bash
# Development check: GPU parity suite (stops at the first failure), then a short SF7 +
# SF12 bench line (no CPU leg) summarised.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dev
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/dev/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/dev/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-channels "$@" > gpurun_out/dev/bench.json 2> gpurun_out/dev/bench.err || { tail -5 gpurun_out/dev/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/dev/bench.json").read().strip().splitlines()[-1])
c = d["config"]
print("SF7 %.1f Msym/s %.4f ms/step stages %s ok=%s kernels=%s" % (d["value"], d["ms_per_step"], [round(x, 4) for x in c["stage_ms"]], c["symbols_ok"], c.get("kernels")))
for k, v in d["extra"].items():
    print(" ", k, v.get("ms_per_step"), v.get("value_all_ranks_msym_s"), [round(x, 4) for x in v.get("stage_ms", [])], v.get("symbols_ok", v.get("symbols_ok_all_frames")), v.get("spec_recomputed_per_step"))
PY
