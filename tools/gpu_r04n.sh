#!/bin/bash
# Round-4: the deferred split-K combine (one launch ahead of NITI_SGD) -- model parity tests, then
# VGG-11 A/B against per-layer reduces (NITI_DIAG_SGD_COMBINE=0), alternating.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04n}
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_b256.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in "comb:" "nocomb:NITI_DIAG_SGD_COMBINE=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/vgg11_${TAG}_$name.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg11_${TAG}_$name.log; exit $rc; }
    echo "$name rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_${TAG}_$name.log)"
  done
done
