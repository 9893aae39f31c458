#!/bin/bash
# VGG-16 under saved plans with the fully connected update pass's tile forced (NITI_DIAG_FC_SGD_TILE):
# a kernel trace summarised per step.
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-fc}
T=${TILE:-64}
rm -rf gpurun_out/tr_vgg16_${TAG}_t$T
NITI_DIAG_FC_SGD_TILE=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_vgg16_${TAG}_t$T" -o run -- python3 bench.py --arch vgg16 --cpu-sample 0 --steps 5 --warmup 2 --load-plans gpurun_out/plans_vgg16_$TAG.json > gpurun_out/tr_vgg16_${TAG}_t$T.log 2>&1
rc=$?; echo "fc tile $T trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_vgg16_${TAG}_t$T -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_vgg16_${TAG}_t${T}_steps.txt
grep -E "busy|, 4, true" gpurun_out/tr_vgg16_${TAG}_t${T}_steps.txt | head -4
