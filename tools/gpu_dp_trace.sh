#!/bin/bash
# Kernel traces of the data-parallel kernel path (bench.py --dp-path) for this build and the
# round's starting build (tools/ablate/base), summarised per step (tools/prof_summary.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in new base; do
  d=$GRAFT_REPO_ROOT; [ $v = base ] && d=$GRAFT_REPO_ROOT/tools/ablate/base
  rm -rf gpurun_out/dptr_$v
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dptr_$v" -o run -- python3 bench.py --dp-path --cpu-sample 0 --steps 10 --warmup 3) > gpurun_out/dptr_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/dptr_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 10 > gpurun_out/dptr_${v}_steps.txt
  echo "$v $(grep -m1 'busy us/step' gpurun_out/dptr_${v}_steps.txt)"
done
