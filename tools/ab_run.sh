# GPU: the suites named in $TESTS (default: the spec / parity / scale / golden parity tests),
# then tools/ab.py over $WORK for the variants in $AB (gpurun from the repo root)
mkdir -p gpurun_out/rec
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_golden.py tests/test_gpu_bandwidth.py} > gpurun_out/rec/pytest_ab.log 2>&1; rc=$?
tail -2 gpurun_out/rec/pytest_ab.log
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python tools/ab.py --reps ${REPS:-3} --work ${WORK:-sf7,awgn0} $AB > gpurun_out/ab.log 2>&1; rc=$?
tail -12 gpurun_out/ab.log
exit $rc
