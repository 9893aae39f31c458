#!/bin/bash
# Round-4: full GPU suite, then VGG-16 / ResNet-18 traces and the VGG-11 default + DP-path benches.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for arch in vgg16 resnet18; do
  rm -rf gpurun_out/tr_${TAG}_${arch}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_${arch}" -o run -- python3 bench.py --arch $arch --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_${arch}.log 2>&1
  rc=$?; echo "$arch rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_${TAG}_${arch}.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr_${TAG}_${arch}.log; exit $rc; }
  f=$(find gpurun_out/tr_${TAG}_${arch} -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_${arch}_breakdown.txt
  rm -rf gpurun_out/tr_${TAG}_${arch}
done
for v in "on:" "dp:--dp-path"; do
  name=${v%%:*}; opt=${v#*:}
  timeout -k 10 300 python3 bench.py --cpu-sample 0 $opt > gpurun_out/vgg11_${TAG}_$name.log 2>&1
  rc=$?; echo "vgg11 $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_${TAG}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg11_${TAG}_$name.log; exit $rc; }
done
