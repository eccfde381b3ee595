#!/bin/bash
# The round's GPU record, one script for every committed profile file (run through gpurun
# from the repo root; writes under gpurun_out/rec, copied by hand into profiles/rNN/):
#   PART=tests  the whole -m gpu suite              -> pytest_gpu.log (-> pytest_gpu_summary.log)
#   PART=only   TESTS="<pytest args>" only           -> pytest_only.log
#   PART=bench  smoke() then `python bench.py`       -> smoke.log, bench_default.json
#   PART=driver the driver's bench command           -> bench_driver.json
#   PART=prof   bench.py under the kernel tracer (SF7 headline, SF12) and the two-rank
#               rehearsal on one GPU                 -> bench7/, bench12/ (kernel_stats.md)
#   PART=pmc    FETCH_SIZE / WRITE_SIZE / SQ passes (tools/pmc_summary.py)  -> pmc/
#   PART=awgn   configs[3]: the AWGN sweep           -> awgn_sweep.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/rec
mkdir -p $OUT
case "$PART" in
tests)
  timeout -k 10 1100 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest_gpu.log 2>&1; rc=$?
  grep -E "pps|dropin_timing|passed|failed|error" $OUT/pytest_gpu.log | tail -25
  exit $rc ;;
only)
  timeout -k 10 900 python -u -m pytest -v -s -x --timeout 300 --timeout-method thread -m gpu $TESTS \
    > $OUT/pytest_only.log 2>&1; rc=$?
  grep -E "pps|dropin_timing|passed|failed|error|Error" $OUT/pytest_only.log | tail -30
  exit $rc ;;
bench)
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 2; }
  tail -1 $OUT/smoke.log
  timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; rc=$?
  tail -3 $OUT/bench_default.err
  python3 tools/bench_summary.py $OUT/bench_default.json 2>/dev/null | head -40 || head -c 2000 $OUT/bench_default.json
  exit $rc ;;
driver)
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err; rc=$?
  tail -3 $OUT/bench_driver.err
  python3 tools/bench_summary.py $OUT/bench_driver.json 2>/dev/null | head -40
  exit $rc ;;
prof)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench7 -o run -- \
    python3 bench.py --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/bench7.json 2> $OUT/bench7.err || { tail -5 $OUT/bench7.err; exit 2; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench12 -o run -- \
    python3 bench.py --sf12-only > $OUT/bench12.json 2> $OUT/bench12.err || { tail -5 $OUT/bench12.err; exit 2; }
  LORA_BENCH_SHARE_DEVICES=1 timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu --no-channels --no-fast --no-variants --no-sf12 \
    > $OUT/bench_2ranks.json 2> $OUT/bench_2ranks.err || { tail -5 $OUT/bench_2ranks.err; exit 2; }
  tail -c 600 $OUT/bench_2ranks.json
  exit 0 ;;
awgn)
  timeout -k 10 900 python -u tools/awgn_sweep_gpu.py --snr -20 10 1 --cfo 0.2 --out $OUT/awgn_sweep.json > $OUT/awgn_sweep.log 2>&1 || { tail -5 $OUT/awgn_sweep.log; exit 2; }
  tail -2 $OUT/awgn_sweep.log
  exit 0 ;;
*)
  echo "PART must be tests|only|bench|driver|prof|awgn"; exit 2 ;;
esac
