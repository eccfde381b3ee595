#!/bin/bash
# Round-3 record of the working tree: the whole GPU suite, smoke(), the default bench (with
# the CPU baseline), rocprofv3 kernel traces of bench.py's SF7 headline alone and its SF12
# workload alone (the trace averages and the bench's own HIP-event stage times come from the
# same process), then SQ / TA and FETCH_SIZE / WRITE_SIZE counter passes (one rocprofv3
# --pmc run each).  Test failures are reported and the rest still runs; anything else (a
# time limit, an abort, a crash) stops the call with status 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/final
mkdir -p $OUT
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head
[ $rc -le 1 ] || { echo "pytest status $rc: stopping"; exit 2; }
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 2; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo "== kt7 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt7 -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/kt7.json 2> $OUT/kt7.err || { tail -20 $OUT/kt7.err; exit 2; }
echo "== kt12 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt12 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --sf12-only > $OUT/kt12.json 2> $OUT/kt12.err || { tail -20 $OUT/kt12.err; exit 2; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
           "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"; do
  for cfg in "7 none 15625 2" "12 none 4000 2"; do
    i=$((i+1))
    echo "== pmc $i sf${cfg%% *} $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 tools/prof_workload.py $cfg > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 2; }
  done
done
for cfg in "7 none 15625 2" "12 none 4000 2"; do
  sf=${cfg%% *}
  for c in FETCH_SIZE WRITE_SIZE; do
    tag=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    echo "== $c sf$sf $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$tag$sf -o run -- python3 tools/prof_workload.py $cfg > $OUT/pmc_$tag$sf.log 2>&1 || { echo "$c pass failed"; tail -3 $OUT/pmc_$tag$sf.log; exit 2; }
  done
done
echo "== done $(date +%T)"
exit $rc
