#!/bin/bash
# Full GPU test suite in one process (one runner, per-test timeout).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log; echo "pytest rc=$rc"
exit $rc
