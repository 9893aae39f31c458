#!/bin/bash
# ResNet-18's fused stem requantise + 3x3 / 2 max pool (requant_pool3_kernel): its average
# duration per (pooled rows per strip, XCD remap) setting, from rocprofv3 --stats of a short bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
PLANS=${PLANS:-tools/probes/plans_resnet18_p4.json}
for cfg in ${CFGS:-8:1 4:1 16:1 8:0}; do
  set -- ${cfg//:/ }
  rm -rf gpurun_out/rq3
  NITI_RQ3_ROWS=$1 NITI_RQ3_REMAP=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rq3" -o run -- python3 bench.py --arch resnet18 --cpu-sample 0 --steps 5 --warmup 2 --load-plans $PLANS > gpurun_out/rq3.log 2>&1 || exit 1
  f=$(find gpurun_out/rq3 -name "*kernel_stats.csv" | head -1)
  echo "rows=$1 remap=$2 $(grep -h 'requant_pool3_kernel' $f | awk -F, '{print "calls", $3, "avg_ns", $5}')"
done
rm -rf gpurun_out/rq3
