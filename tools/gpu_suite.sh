#!/bin/bash
# GPU tests in one process (one runner, per-test timeout), then smoke() and, with BENCH=1, the
# default bench line.  TESTS selects the test files (default: the whole suite).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r06}
TESTS=${TESTS:-tests}
timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$TAG.log
fi
exit $rc
