#!/bin/bash
# Round-4: segment-mode tap-sharing weight gradient -- its op tests, the model step tests, then
# the VGG-16 / ResNet-18 step traces.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "taps" > gpurun_out/tests_taps_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_taps_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_resnet.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for arch in ${ARCHS:-vgg16 resnet18}; do
  rm -rf gpurun_out/tr_${TAG}_${arch}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_${arch}" -o run -- python3 bench.py --arch $arch --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_${arch}.log 2>&1
  rc=$?; echo "$arch rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_${TAG}_${arch}.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr_${TAG}_${arch}.log; exit $rc; }
  f=$(find gpurun_out/tr_${TAG}_${arch} -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 7 > gpurun_out/tr_${TAG}_${arch}_breakdown.txt
  rm -rf gpurun_out/tr_${TAG}_${arch}
done
timeout -k 10 300 python3 bench.py --arch resnet18 --steps 6 --warmup 2 --cpu-sample 0 --graph > gpurun_out/resnet_graph_$TAG.log 2>&1
rc=$?; echo "resnet graph rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_graph_$TAG.log)"
