#!/bin/bash
# Round-4: ResNet-18 forward recompute form chosen by the autotuner -- ResNet tests, bench, trace.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04y}
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --arch resnet18 --steps 8 --warmup 2 --cpu-sample 0 > gpurun_out/resnet_$TAG.log 2>&1
rc=$?; echo "resnet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --arch resnet18 --steps 8 --warmup 2 --cpu-sample 0 > gpurun_out/resnet2_$TAG.log 2>&1
rc=$?; echo "resnet2 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet2_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/tr_${TAG}_resnet18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_resnet18" -o run -- python3 bench.py --arch resnet18 --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_resnet18.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_${TAG}_resnet18 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_resnet18_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_resnet18
