#!/bin/bash
# The BASELINE ImageNet networks on one GPU: ResNet-18 (batch 128, config 5's per-GPU share) and
# VGG-16 (batch 64, config 4's), each benched with autotuning (plans saved), then a rocprofv3 kernel
# trace of the same step under those plans, summarised per step (tools/prof_summary.py).
# NETS selects (default "resnet18 vgg16"); EXTRA adds bench flags to every run.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
EXTRA=${EXTRA:-}
for net in ${NETS:-resnet18 vgg16}; do
  timeout -k 10 500 python3 bench.py --arch $net --cpu-sample ${CPU_SAMPLE:-0} --save-plans gpurun_out/plans_${net}_$TAG.json $EXTRA > gpurun_out/${net}_$TAG.log 2>&1
  rc=$?; echo "$net bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${net}_$TAG.log)"
  [ $rc -eq 0 ] || exit $rc
  rm -rf gpurun_out/tr_${net}_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${net}_$TAG" -o run -- python3 bench.py --arch $net --cpu-sample 0 --steps 5 --warmup 2 --load-plans gpurun_out/plans_${net}_$TAG.json $EXTRA > gpurun_out/tr_${net}_$TAG.log 2>&1
  rc=$?; echo "$net trace rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/tr_${net}_$TAG -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${net}_${TAG}_steps.txt
  grep -m1 "busy us/step" gpurun_out/tr_${net}_${TAG}_steps.txt
done
