#!/bin/bash
# The GEMM speculative pair (plan strategy 3) under the round-6 predictor: autotuned with it as a
# candidate (NITI_TUNE_SPEC=1) against the default candidate set, VGG-16 and ResNet-18, alternating.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/tune_spec_ab.txt
: > $OUT
for net in vgg16 resnet18; do
  for ts in 1 0 1 0; do
    NITI_TUNE_SPEC=$ts timeout -k 10 400 python3 bench.py --arch $net --cpu-sample 0 --save-plans gpurun_out/plans_${net}_ts$ts.json > gpurun_out/tune_spec_${net}_$ts.log 2>&1 || exit $?
    echo "$net tune_spec $ts $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune_spec_${net}_$ts.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/tune_spec_${net}_$ts.log) strat3 $(grep -o ', 3\]' gpurun_out/plans_${net}_ts$ts.json | wc -l)" >> $OUT
  done
done
cat $OUT
