#!/bin/bash
# Round-4: the row-segment form for deep convs now that the speculative pair makes it one GEMM pass --
# VGG-16 / ResNet-18 A/B over NITI_SEG_MAX_CIN, then whole-step 224-px parity with it at 512.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04ab}
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" --cpu-sample 0 > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${name}_$TAG.log)"; return $rc
}
b vgg16_128 "NITI_SEG_MAX_CIN=128" --arch vgg16 --steps 4 --warmup 2 &&
b vgg16_256 "NITI_SEG_MAX_CIN=256" --arch vgg16 --steps 4 --warmup 2 &&
b vgg16_512 "NITI_SEG_MAX_CIN=512" --arch vgg16 --steps 4 --warmup 2 &&
b resnet_128 "NITI_SEG_MAX_CIN=128" --arch resnet18 --steps 8 --warmup 2 &&
b resnet_256 "NITI_SEG_MAX_CIN=256" --arch resnet18 --steps 8 --warmup 2 || exit 1
NITI_SEG_MAX_CIN=512 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread -k "224 or vgg16" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; exit $rc
