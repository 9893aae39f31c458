#!/bin/bash
# Round-4: ResNet-18 with the update writing the row kernels' weight copies -- parity tests, then
# the step with 64- / 128-channel NHWC16 row inputs (NITI_SEG_NHWC_MAX_CIP), alternating.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04r}
timeout -k 10 500 python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "resnet or sgd" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "nhwc64:" "nhwc128:NITI_SEG_NHWC_MAX_CIP=128"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --arch resnet18 --steps 8 --warmup 2 --cpu-sample 0 > gpurun_out/resnet_${TAG}_$name.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/resnet_${TAG}_$name.log; exit $rc; }
    echo "$name rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_${TAG}_$name.log)"
  done
done
