#!/bin/bash
# Round-4: the stem's im2col op test, ResNet-18 parity, ResNet-18 trace; then the r04i checks.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04j}
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py -x -q --timeout 200 --timeout-method thread -k "im2col or resnet" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/tr_${TAG}_resnet18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_resnet18" -o run -- python3 bench.py --arch resnet18 --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_resnet18.log 2>&1
rc=$?; echo "resnet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_${TAG}_resnet18.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr_${TAG}_resnet18.log; exit $rc; }
f=$(find gpurun_out/tr_${TAG}_resnet18 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_resnet18_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_resnet18
TAG=${TAG}i bash tools/gpu_r04i.sh
