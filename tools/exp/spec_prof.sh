mkdir -p gpurun_out/spec
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -q --timeout 120 --timeout-method thread > gpurun_out/spec/pytest.log 2>&1; tail -3 gpurun_out/spec/pytest.log
VARIANTS="main specabl main specabl" timeout -k 10 300 bash tools/exp/variants.sh && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
LORA_MI355X_SPEC=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/spec/prof1 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants --no-sf12 > gpurun_out/spec/prof1.log 2>&1 && \
LORA_MI355X_SPEC=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/spec/prof0 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-channels --no-fast --no-variants --no-sf12 > gpurun_out/spec/prof0.log 2>&1; echo done
