cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g1
rocprofv3 -L > gpurun_out/g1/counters.txt 2>&1 || true
nproc > gpurun_out/g1/host.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/g1/host.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels --no-fast --no-sf12 > gpurun_out/g1/b_default.json 2> gpurun_out/g1/b_default.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-channels --no-fast --no-sf12 --sync 0xff > gpurun_out/g1/b_syncff.json 2> gpurun_out/g1/b_syncff.err
