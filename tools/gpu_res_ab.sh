#!/bin/bash
# The packed residual pass: the probe's isolated timings, then ResNet-18 kernel stats with the
# packed pass off / on (same plans; per-kernel averages from rocprofv3 --stats).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 60 tools/probes/exit_probe > gpurun_out/exit_probe2.txt 2>&1 || exit $?
cat gpurun_out/exit_probe2.txt
for pk in 0 1; do
  rm -rf gpurun_out/res_pk$pk
  NITI_RES_PK=$pk timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/res_pk$pk" -o run -- python3 bench.py --arch resnet18 --cpu-sample 0 --steps 10 --warmup 3 --load-plans tools/probes/plans_resnet18_r06.json > gpurun_out/res_pk$pk.log 2>&1 || exit $?
  echo "pk $pk $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/res_pk$pk.log)"
  f=$(find gpurun_out/res_pk$pk -name '*kernel_stats.csv' | head -1)
  grep -i "residual_requant" "$f"
done
