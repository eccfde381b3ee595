cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rec; mkdir -p $O
for cfg in "20 5" "100 10" "20 5" "20 5 0"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --no-channels --no-fast --no-variants --no-sf12 --steps $1 --warmup $2 --prewarm-ms ${3:-300} > $O/w.json 2>/dev/null || exit 3
  python -c "import json,sys; d=json.loads(open('$O/w.json').read().strip().splitlines()[-1]); print('steps $1 warm $2 prewarm ${3:-300}', round(d['ms_per_step'],4), round(d['value'],1), d['roofline']['frac'])"
done
