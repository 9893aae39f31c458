#!/bin/bash
# Pair / model parity tests, then the data-parallel kernel path against the round's starting build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rowconv.py tests/test_gpu_model.py tests/test_dp_local.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dp2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dp2_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/dp_ab2.txt
: > $OUT
for rep in 1 2; do
  for v in new base; do
    d=.; [ $v = base ] && d=tools/ablate/base
    (cd $d && timeout -k 10 300 python3 bench.py --cpu-sample 0 --dp-path) > gpurun_out/dp_ab2_$v.log 2>&1 || exit $?
    echo "$v dp-path $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_ab2_$v.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/dp_ab2_$v.log)" >> $OUT
  done
done
cat $OUT
for net in resnet18 vgg16; do
  timeout -k 10 400 python3 bench.py --cpu-sample 0 --arch $net > gpurun_out/dp_ab2_$net.log 2>&1 || exit $?
  echo "new $net $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_ab2_$net.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/dp_ab2_$net.log)" >> $OUT
done
cat $OUT
