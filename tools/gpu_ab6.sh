#!/bin/bash
# Round-6 A/B: residual / ResNet parity tests on the packed residual pass, then the probed
# launch's event cost on VGG-11 (probe every step / 1 in 4 / none) and ResNet-18 with the packed
# residual pass on / off, alternating on one box.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_residual_ops.py tests/test_gpu_resnet_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab6_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ab6.txt
: > $OUT
for rep in 1 2; do
  for k in 1 4 0; do
    timeout -k 10 200 python3 bench.py --cpu-sample 0 --probe-every $k > gpurun_out/ab6_p$k.log 2>&1 || exit $?
    echo "rep $rep vgg11 probe-every $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab6_p$k.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab6_p$k.log | head -1)" >> $OUT
  done
  for pk in 1 0; do
    NITI_RES_PK=$pk timeout -k 10 300 python3 bench.py --arch resnet18 --cpu-sample 0 --load-plans tools/probes/plans_resnet18_r06.json > gpurun_out/ab6_r$pk.log 2>&1 || exit $?
    echo "rep $rep resnet18 res_pk $pk $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab6_r$pk.log) $(grep -o '"redone": [0-9]*' gpurun_out/ab6_r$pk.log)" >> $OUT
  done
done
cat $OUT
