#!/bin/bash
# Round-4: 4-row tile mode of the tap-sharing weight gradient -- its op tests, then VGG-16 steps with
# the segment / tile modes at different input-channel caps (NITI_TAPS_SEG_MAX_CIP) and tile mode off.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "taps" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for v in "tile64:" "seg64:NITI_TAPS_TILE=0" "tile128:NITI_TAPS_SEG_MAX_CIP=128" "tile512:NITI_TAPS_SEG_MAX_CIP=512"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 400 python3 bench.py --arch vgg16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/vgg16_${TAG}_$name.log 2>&1
  rc=$?; echo "vgg16 $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_${TAG}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg16_${TAG}_$name.log; exit $rc; }
done
