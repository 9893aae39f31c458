#!/bin/bash
# Round-4: conv0 with hoisted weights / prefetched rows -- model tests, VGG-11 bench + trace,
# VGG-16 bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04o}
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "vgg or lenet or conv0" > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/vgg11_${TAG}.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg11_${TAG}.log; exit $rc; }
  echo "vgg11 rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_${TAG}.log)"
done
rm -rf gpurun_out/tr_${TAG}_vgg11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_vgg11" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 > gpurun_out/tr_${TAG}_vgg11.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_${TAG}_vgg11 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/tr_${TAG}_vgg11_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_vgg11
timeout -k 10 400 python3 bench.py --arch vgg16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/vgg16_$TAG.log 2>&1
rc=$?; echo "vgg16 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_$TAG.log)"
