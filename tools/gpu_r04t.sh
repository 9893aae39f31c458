#!/bin/bash
# Round-4: the speculative two-launch pair (modes 3 / 4) -- row-kernel, model, DP and ResNet tests,
# then VGG-11 (fused and --dp-path), VGG-16 and ResNet-18 steps, each A/B against NITI_RC_SPEC2=0.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04t}
timeout -k 10 900 python -u -m pytest tests/test_gpu_rowconv.py tests/test_gpu_model.py tests/test_gpu_resnet.py tests/test_dp_local.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" --cpu-sample 0 > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${name}_$TAG.log)"; return $rc
}
b vgg11 "NITI_RC_SPEC2=1" --steps 20 --warmup 5 &&
b vgg11dp "NITI_RC_SPEC2=1" --steps 20 --warmup 5 --dp-path &&
b vgg11dp_off "NITI_RC_SPEC2=0" --steps 20 --warmup 5 --dp-path &&
b vgg16 "NITI_RC_SPEC2=1" --arch vgg16 --steps 4 --warmup 2 &&
b vgg16_off "NITI_RC_SPEC2=0" --arch vgg16 --steps 4 --warmup 2 &&
b resnet "NITI_RC_SPEC2=1" --arch resnet18 --steps 8 --warmup 2 &&
b resnet_off "NITI_RC_SPEC2=0" --arch resnet18 --steps 8 --warmup 2
