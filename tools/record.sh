#!/bin/bash
# The round's GPU record, one script for every committed profile file (run through gpurun
# from the repo root; writes under gpurun_out/rec, copied by hand into profiles/rNN/):
#   PART=tests  the whole -m gpu suite              -> pytest_gpu.log (-> pytest_gpu_summary.log)
#   PART=only   TESTS="<pytest args>" only           -> pytest_only.log
#   PART=bench  smoke() then `python bench.py`       -> smoke.log, bench_default.json
#   PART=driver the driver's bench command           -> bench_driver.json
#   PART=prof   bench.py under the kernel tracer (SF7 headline, SF12) and the two-rank
#               rehearsal on one GPU                 -> bench7/, bench12/ (kernel_stats.md)
#   PART=trace  rocprofv3 --kernel-trace --stats of each workload alone (tools/prof_workload.py)
#               and of bench.py's SF7 / SF12 lines   -> prof/   then:
#               python tools/kernel_stats.py gpurun_out/rec/prof profiles/rNN/kernel_stats.md
#   PART=pmc    SQ counter passes (SF7, SF12) and FETCH_SIZE / WRITE_SIZE per workload, one
#               rocprofv3 --pmc run each              -> prof/   then:
#               python tools/pmc_traffic.py gpurun_out/rec/prof profiles/rNN/pmc_traffic.md
#               (also writes profiles/pmc_summary.json, bench.py's roofline.traffic source)
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
trace)
  P=$OUT/prof; mkdir -p $P
  for cfg in "kt7 7 none 15625 20" "kt7n0 7 0 15625 20" "kt7n10 7 -10 15625 20" "kt12 12 none 15625 6" \
             "kt7o2 7 none 15625 20 64 2" "kt7o4 7 none 15625 10 64 4" "kt7api 7 none 15625 20 64 1 api" \
             "kt7raw 7 none 15625 20 64 1 raw"; do
    set -- $cfg
    tag=$1; shift
    echo "== $tag $(date +%T)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$tag -o run -- python3 tools/prof_workload.py "$@" > $P/$tag.log 2>&1 || { tail -20 $P/$tag.log; exit 2; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bench7 -o run -- \
    python3 bench.py --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $P/bench7.json 2> $P/bench7.err || { tail -5 $P/bench7.err; exit 2; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bench12 -o run -- \
    python3 bench.py --sf12-only > $P/bench12.json 2> $P/bench12.err || { tail -5 $P/bench12.err; exit 2; }
  exit 0 ;;
pmc)
  P=$OUT/prof; mkdir -p $P
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
             "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_IFETCH"; do
    for cfg in "7 none 15625 2" "12 none 4000 2"; do
      i=$((i+1))
      echo "== pmc $i sf${cfg%% *} $(date +%T)"
      PROF_PREWARM_MS=0 timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $P/pmc$i -o run -- python3 tools/prof_workload.py $cfg > $P/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $P/pmc$i.log; exit 2; }
    done
  done
  for cfg in "7:7 none 15625 2" "12:12 none 4000 2" "7o2:7 none 15625 2 64 2" "7o4:7 none 15625 2 64 4" \
             "7api:7 none 15625 2 64 1 api" "7raw:7 none 15625 2 64 1 raw"; do
    tag=${cfg%%:*}; args=${cfg#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      t=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
      echo "== $c $tag $(date +%T)"
      PROF_PREWARM_MS=0 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $P/pmc_$t$tag -o run -- python3 tools/prof_workload.py $args > $P/pmc_$t$tag.log 2>&1 || { echo "$c pass failed"; tail -3 $P/pmc_$t$tag.log; exit 2; }
    done
  done
  exit 0 ;;
awgn)
  timeout -k 10 900 python -u tools/awgn_sweep_gpu.py --snr -20 10 1 --cfo 0.2 --out $OUT/awgn_sweep.json > $OUT/awgn_sweep.log 2>&1 || { tail -5 $OUT/awgn_sweep.log; exit 2; }
  tail -2 $OUT/awgn_sweep.log
  exit 0 ;;
*)
  echo "PART must be tests|only|bench|driver|prof|trace|pmc|awgn"; exit 2 ;;
esac
