# GPU suite + default bench (round 3 iteration)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_$TAG.log | cut -c1-600
exit $rc
