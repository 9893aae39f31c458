#!/bin/bash
# Round-4: VGG-11 default bench (as the driver runs it) + step trace breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04aa}
timeout -k 10 400 python3 bench.py > gpurun_out/vgg11_$TAG.log 2>&1
rc=$?; echo "vgg11 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/tr_${TAG}_vgg11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_vgg11" -o run -- python3 bench.py --steps 5 --warmup 3 --cpu-sample 0 > gpurun_out/tr_${TAG}_vgg11.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_${TAG}_vgg11 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_vgg11_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_vgg11
