#!/bin/bash
# Round-5 record on the GPU: PART=tests - the whole -m gpu suite; PART=bench - smoke() then
# the default bench line (every line, CPU legs included); PART=prof - bench.py under the
# kernel tracer (headline, SF12) and the two-rank rehearsal on one GPU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/r05rec
mkdir -p $OUT
if [ "$PART" = tests ]; then
  timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest_gpu.log 2>&1; rc=$?
  grep -E "pps|dropin_timing|passed|failed|error" $OUT/pytest_gpu.log | tail -25
  exit $rc
fi
if [ "$PART" = awgn ]; then
  # configs[3]: the AWGN sweep SF 7-12, -20 .. +10 dB in 1 dB steps, 0.2-bin CFO, every frame
  # compared with the exact path and 32 per point with the oracle
  timeout -k 10 900 python -u tools/awgn_sweep_gpu.py --snr -20 10 1 --cfo 0.2 --out $OUT/awgn_sweep.json > $OUT/awgn_sweep.log 2>&1 || { tail -5 $OUT/awgn_sweep.log; exit 2; }
  tail -2 $OUT/awgn_sweep.log
  exit 0
fi
if [ "$PART" = prof ]; then
  # bench.py's headline and SF12 lines under the kernel tracer (the same command's HIP-event
  # stage times beside rocprofv3's per-kernel averages), then the two-rank rehearsal on one GPU
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench7 -o run -- \
    python3 bench.py --no-cpu --no-channels --no-fast --no-variants --no-sf12 > $OUT/bench7.json 2> $OUT/bench7.err || { tail -5 $OUT/bench7.err; exit 2; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench12 -o run -- \
    python3 bench.py --sf12-only > $OUT/bench12.json 2> $OUT/bench12.err || { tail -5 $OUT/bench12.err; exit 2; }
  LORA_BENCH_SHARE_DEVICES=1 timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu --no-channels --no-fast --no-variants --no-sf12 \
    > $OUT/bench_2ranks.json 2> $OUT/bench_2ranks.err || { tail -5 $OUT/bench_2ranks.err; exit 2; }
  tail -c 600 $OUT/bench_2ranks.json
  exit 0
fi
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; rc=$?
tail -3 $OUT/bench_default.err
python3 tools/bench_summary.py $OUT/bench_default.json 2>/dev/null | head -40 || head -c 2000 $OUT/bench_default.json
exit $rc
