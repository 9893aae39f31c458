#!/bin/bash
# Round-4 row-segment A/B: seg R = 2 (two waves per SIMD) vs R = 4 per layer, and the VGG-16 /
# ResNet-18 whole steps with and without the row-segment form (NITI_SEG_MAX_CIN=0 turns it off).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04c}
NITI_SEG_R=2 timeout -k 10 400 python3 -u tools/seg_bench.py > gpurun_out/seg_bench_${TAG}_r2.txt 2>&1
rc=$?; echo "seg r2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/seg_bench_${TAG}_r2.txt; exit $rc; }
for v in "seg:" "noseg:NITI_SEG_MAX_CIN=0"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 400 python3 bench.py --arch vgg16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/vgg16_${TAG}_$name.log 2>&1
  rc=$?; echo "vgg16 $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_${TAG}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg16_${TAG}_$name.log; exit $rc; }
  env $envs timeout -k 10 400 python3 bench.py --arch resnet18 --steps 6 --warmup 2 --cpu-sample 0 > gpurun_out/resnet_${TAG}_$name.log 2>&1
  rc=$?; echo "resnet $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_${TAG}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/resnet_${TAG}_$name.log; exit $rc; }
done
tail -12 gpurun_out/seg_bench_${TAG}_r2.txt
