#!/bin/bash
# Round-4 final records of the other networks: parity tests of the taps modes and VGG-16, then
# tools/gpu_others.sh (VGG-16 with its probe's PMC traffic, LeNet, ResNet-18).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "taps or vgg16" > gpurun_out/tests_r04q.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_r04q.txt; [ $rc -eq 0 ] || exit $rc
TAG=r04 bash tools/gpu_others.sh
