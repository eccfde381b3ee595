#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/modprof; mkdir -p $OUT
for sf in 7 12; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$sf -o run -- python3 tools/prof_workload.py $sf none 15625 1 > $OUT/kt$sf.log 2>&1 || { tail -5 $OUT/kt$sf.log; exit 2; }
python3 -c "
import csv
for x in csv.DictReader(open('$OUT/kt$sf/run_kernel_stats.csv')): print('$sf', x['Name'][:50], x['Calls'], '%.4f' % (float(x['AverageNs'])/1e6))
"
done
