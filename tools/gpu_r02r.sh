# Bucketed data-parallel gradient SUM: the in-process DP parity tests, the step tests, one bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_local.py tests/test_gpu_model.py tests/test_gpu_b256.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/r_bench.json 2> gpurun_out/r_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/r_bench.json; exit $rc
