#!/bin/bash
# The data-parallel kernel path (bench.py --dp-path, one GPU) under the round-6 predictor: the scaled
# forward guesses on / off (NITI_SPEC_SCALE) x store-mode cooldown after a miss (NITI_SPEC_COOLDOWN),
# against the round's starting build (tools/ablate/base).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/dp_ab.txt
: > $OUT
for rep in 1 2; do
  (cd tools/ablate/base && timeout -k 10 300 python3 bench.py --cpu-sample 0 --dp-path) > gpurun_out/dp_ab_base.log 2>&1 || exit $?
  echo "base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_ab_base.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/dp_ab_base.log)" >> $OUT
  for sc in 1 0; do
    for cd in 8 0 2; do
      NITI_SPEC_SCALE=$sc NITI_SPEC_COOLDOWN=$cd timeout -k 10 300 python3 bench.py --cpu-sample 0 --dp-path > gpurun_out/dp_ab.log 2>&1 || exit $?
      echo "scale $sc cooldown $cd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_ab.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/dp_ab.log)" >> $OUT
    done
  done
done
cat $OUT
