#!/bin/bash
# Round-4 record on one MI355X: every GPU test, smoke(), the default bench (with its CPU leg),
# and the configs[3] AWGN sweep (SF 7-12, -20 ... +10 dB in 1 dB steps, 0.2-bin CFO, 1,000
# frames per point, every frame compared with the three-launch exact path).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 2; }
python tools/bench_summary.py $OUT/bench_default.json
timeout -k 10 600 python -u tools/awgn_sweep_gpu.py --snr -20 10 1 --cfo 0.2 --out $OUT/awgn_sweep.json > $OUT/awgn_sweep.log 2>&1 || { tail -5 $OUT/awgn_sweep.log; exit 2; }
tail -2 $OUT/awgn_sweep.log
echo "== done $(date +%T)"
