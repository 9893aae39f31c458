#!/bin/bash
# Round-4: LUT input quantiser (NCHW 16-byte path, 512-block standalone stats), register-offset stem
# im2col -- quantiser / op / model / ResNet / b256 tests, VGG-11, ResNet-18, VGG-16 steps, ResNet trace.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04x}
timeout -k 10 900 python -u -m pytest tests/test_quant.py tests/test_gpu_ops.py tests/test_gpu_resnet.py tests/test_gpu_model.py tests/test_gpu_b256.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --cpu-sample 0 > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${name}_$TAG.log)"; return $rc
}
b vgg11 --steps 20 --warmup 5 &&
b vgg11b --steps 20 --warmup 5 &&
b resnet --arch resnet18 --steps 8 --warmup 2 &&
b vgg16 --arch vgg16 --steps 4 --warmup 2 || exit 1
rm -rf gpurun_out/tr_${TAG}_resnet18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_resnet18" -o run -- python3 bench.py --arch resnet18 --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_resnet18.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_${TAG}_resnet18 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_resnet18_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_resnet18
