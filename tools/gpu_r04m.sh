#!/bin/bash
# Round-4: stem im2col from NCHW and the split-K combine in the NITI_SGD launch -- op, ResNet,
# model-step and batch-256 parity tests, the ResNet trace and bench, the VGG-11 bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04m}
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py tests/test_gpu_model.py tests/test_gpu_b256.py tests/test_dp_local.py -x -q --timeout 200 --timeout-method thread -k "im2col or resnet or ResNet or vgg or b256 or local" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/tr_${TAG}_resnet18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_resnet18" -o run -- python3 bench.py --arch resnet18 --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_resnet18.log 2>&1
rc=$?; echo "resnet trace rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_${TAG}_resnet18.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr_${TAG}_resnet18.log; exit $rc; }
f=$(find gpurun_out/tr_${TAG}_resnet18 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_resnet18_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_resnet18
timeout -k 10 300 python3 bench.py --arch resnet18 --steps 8 --warmup 2 --cpu-sample 0 > gpurun_out/resnet_$TAG.log 2>&1
rc=$?; echo "resnet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_$TAG.log)"
timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/vgg11_$TAG.log 2>&1
rc=$?; echo "vgg11 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_$TAG.log)"
NITI_DIAG_SGD_COMBINE=0 timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/vgg11_${TAG}_nocomb.log 2>&1
rc=$?; echo "vgg11 no-combine rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_${TAG}_nocomb.log)"
