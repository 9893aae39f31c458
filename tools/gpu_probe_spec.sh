#!/bin/bash
# VGG-16 with the speculative pair forced on some GEMM layers (tools/probes/plans_vgg16_spec.json):
# bench line with its pair statistics, then a kernel trace of the same plans.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-spec}
P=tools/probes/plans_vgg16_spec.json
timeout -k 10 300 python3 bench.py --arch vgg16 --cpu-sample 0 --load-plans $P > gpurun_out/vgg16_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/tr_vgg16_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_vgg16_$TAG" -o run -- python3 bench.py --arch vgg16 --cpu-sample 0 --steps 5 --warmup 2 --load-plans $P > gpurun_out/tr_vgg16_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_vgg16_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_vgg16_${TAG}_steps.txt
grep -m1 "busy us/step" gpurun_out/tr_vgg16_${TAG}_steps.txt
