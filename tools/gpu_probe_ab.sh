#!/bin/bash
# A/B of the probed launch's event cost on the VGG-11 step: the probe in every timed step (1), in
# one of every 4 (4), in none (0), alternating on one box.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/probe_ab.txt
: > $OUT
for rep in 1 2; do
  for k in 1 4 0; do
    timeout -k 10 200 python3 bench.py --cpu-sample 0 --probe-every $k > gpurun_out/probe_ab_$k.log 2>&1 || exit $?
    echo "rep $rep every $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/probe_ab_$k.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/probe_ab_$k.log | head -1)" >> $OUT
  done
done
cat $OUT
