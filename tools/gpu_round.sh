#!/bin/bash
# One round's measurements in one GPU call: the default VGG-11 bench with its rocprofv3 kernel stats
# and PMC passes (gpu_full.sh), the ImageNet networks' benches with kernel traces (gpu_nets.sh),
# the data-parallel kernel path on one GPU (bench.py --dp-path) and LeNet.  Every step has its own
# time limit and the chain stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
TAG=$TAG bash tools/gpu_full.sh || exit $?
TAG=$TAG NETS="${NETS:-resnet18 vgg16}" bash tools/gpu_nets.sh || exit $?
timeout -k 10 300 python3 bench.py --dp-path --cpu-sample 0 > gpurun_out/dp_path_$TAG.log 2>&1
rc=$?; echo "dp-path rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp_path_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --arch lenet > gpurun_out/lenet_$TAG.log 2>&1
rc=$?; echo "lenet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lenet_$TAG.log)"
exit $rc
