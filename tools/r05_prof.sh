#!/bin/bash
# Round-5 profiles of the tree (summarised by PROF_ROUND=5 tools/prof_r04.py).
# PART=trace: rocprofv3 kernel traces of each bench workload alone (tools/prof_workload.py:
#   SF7 headline, SF7 0 dB and -10 dB, SF12, SF7 osr 2 / osr 4, SF7 API and RAW modes), then
#   bench.py's headline and SF12 lines under the tracer.
# PART=pmc: counter passes (one rocprofv3 --pmc run each): SQ counters for SF7 / SF12, and
#   FETCH_SIZE / WRITE_SIZE (HBM traffic) for every bench line's workload.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/prof5
mkdir -p $OUT
if [ "${PART:-trace}" = trace ]; then
for cfg in "kt7 7 none 15625 20" "kt7n0 7 0 15625 20" "kt7n10 7 -10 15625 20" "kt12 12 none 15625 6" \
           "kt7o2 7 none 15625 20 64 2" "kt7o4 7 none 15625 10 64 4" "kt7api 7 none 15625 20 64 1 api" \
           "kt7raw 7 none 15625 20 64 1 raw"; do
  set -- $cfg
  echo "== $1 $(date +%T)"
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python3 tools/prof_workload.py "$@" > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 2; }
  tail -1 $OUT/$tag.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench7 -o run -- \
  python3 bench.py --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/bench7.json 2> $OUT/bench7.err || { tail -5 $OUT/bench7.err; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench12 -o run -- \
  python3 bench.py --sf12-only > $OUT/bench12.json 2> $OUT/bench12.err || { tail -5 $OUT/bench12.err; exit 2; }
fi
if [ "${PART:-trace}" = pmc ]; then
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_IFETCH"; do
  for cfg in "7 none 15625 2" "12 none 4000 2"; do
    i=$((i+1))
    echo "== pmc $i sf${cfg%% *} $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 tools/prof_workload.py $cfg > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 2; }
  done
done
for cfg in "7:7 none 15625 2" "12:12 none 4000 2" "7o2:7 none 15625 2 64 2" "7o4:7 none 15625 2 64 4" \
           "7api:7 none 15625 2 64 1 api" "7raw:7 none 15625 2 64 1 raw"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    t=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    echo "== $c $tag $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$t$tag -o run -- python3 tools/prof_workload.py $args > $OUT/pmc_$t$tag.log 2>&1 || { echo "$c pass failed"; tail -3 $OUT/pmc_$t$tag.log; exit 2; }
  done
done
fi
if [ "${PART:-trace}" = valu ]; then
# VALU issue of the API / RAW lines' symbol pass (k_demod_fast): SQ_INSTS_VALU with the
# GPU cycles of the same launches, one pass each
for cfg in "7api:7 none 15625 2 64 1 api" "7raw:7 none 15625 2 64 1 raw"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  echo "== valu $tag $(date +%T)"
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu$tag -o run -- python3 tools/prof_workload.py $args > $OUT/pmc_valu$tag.log 2>&1 || { echo "valu pass failed"; tail -3 $OUT/pmc_valu$tag.log; exit 2; }
done
fi
echo "== done $(date +%T)"
