#!/bin/bash
# A/B of one environment switch on the default bench, alternating on one box: A = as is, B = with
# $ENVB set (e.g. ENVB="NITI_HEAD_CHAIN=0"); then a rocprofv3 kernel trace of A summarised per step.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
ARGS=${ARGS:-}
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --cpu-sample 0 $ARGS > gpurun_out/ab_${TAG}_A$r.log 2>&1 || exit $?
  echo "A$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_A$r.log)"
  timeout -k 10 200 env $ENVB python3 bench.py --cpu-sample 0 $ARGS > gpurun_out/ab_${TAG}_B$r.log 2>&1 || exit $?
  echo "B$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_B$r.log)"
done
rm -rf gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_$TAG" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 $ARGS > gpurun_out/tr_$TAG.log 2>&1 || exit $?
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 10 > gpurun_out/tr_${TAG}_steps.txt
head -40 gpurun_out/tr_${TAG}_steps.txt
