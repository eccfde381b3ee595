#!/bin/bash
# Round 4 development step on the GPU: the pipeline's parity tests, a bench without the CPU
# leg and configs[4], and one counter pass (LDS / VALU) over the SF7 and SF12 workloads.
# usage: tools/r04_dev.sh   (TESTS="tests/..." overrides the selection; NOBENCH=1, NOPMC=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/dev
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_osr.py tests/test_gpu_golden.py tests/test_gpu_scale.py} \
  > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py --no-cpu --no-channels > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 2; }
  python tools/bench_summary.py $OUT/bench.json
fi
if [ -z "$NOPMC" ]; then
  for cfg in "7 none 15625 2" "12 none 4000 2"; do
    tag=pmc_sf${cfg%% *}
    timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
      --output-format csv -d $OUT/$tag -o run -- python3 tools/prof_workload.py $cfg > $OUT/$tag.log 2>&1 || { echo "pmc failed"; tail -3 $OUT/$tag.log; exit 2; }
  done
  python3 tools/prof_r04.py $OUT > $OUT/pmc.md 2>&1; grep -E "^### |BANK_CONFLICT /|VALU per wave|WAIT_INST_ANY /" $OUT/pmc.md
fi
echo "== done $(date +%T)"
