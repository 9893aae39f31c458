#!/bin/bash
# Round-4 final records: VGG-16 (224 px, batch 64) bench line with its CPU baseline.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04ac}
timeout -k 10 600 python3 bench.py --arch vgg16 --steps 6 --warmup 2 > gpurun_out/vgg16_$TAG.log 2>&1
rc=$?; echo "vgg16 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_$TAG.log)"; exit $rc
