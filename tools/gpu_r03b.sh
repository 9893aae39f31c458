# rowconv bring-up: model parity tests, then the full GPU suite and the bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > gpurun_out/model_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/model_$TAG.log; echo "model rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_$TAG.log | cut -c1-400
exit $rc
