#!/bin/bash
# The lane-parallel predictor update: pair / residual / model parity tests, then the data-parallel
# kernel path and ResNet-18 against the round's starting build (tools/ablate/base), alternating.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rowconv.py tests/test_gpu_residual_ops.py tests/test_gpu_resnet_cpp.py tests/test_gpu_model.py tests/test_dp_local.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/learn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/learn_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/learn_ab.txt
: > $OUT
for rep in 1 2; do
  for v in new base; do
    d=.; [ $v = base ] && d=tools/ablate/base
    (cd $d && timeout -k 10 300 python3 bench.py --cpu-sample 0 --dp-path) > gpurun_out/learn_dp_$v.log 2>&1 || exit $?
    echo "$v dp-path $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/learn_dp_$v.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/learn_dp_$v.log)" >> $OUT
  done
  (timeout -k 10 300 python3 bench.py --cpu-sample 0 --arch resnet18) > gpurun_out/learn_r18.log 2>&1 || exit $?
  echo "new resnet18 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/learn_r18.log) $(grep -o '"redone": [0-9]*' gpurun_out/learn_r18.log)" >> $OUT
done
cat $OUT
