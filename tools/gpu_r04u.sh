#!/bin/bash
# Round-4: step traces of the speculative pair -- VGG-11 --dp-path and VGG-16, spec on / off.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04u}
tr() {  # name, env, args
  local name=$1 envs=$2; shift 2
  rm -rf gpurun_out/tr_${TAG}_$name
  export $envs
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_$name" -o run -- python3 bench.py "$@" --cpu-sample 0 > gpurun_out/tr_${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || return $rc
  local f=$(find gpurun_out/tr_${TAG}_$name -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 5 > gpurun_out/tr_${TAG}_${name}_breakdown.txt
  rm -rf gpurun_out/tr_${TAG}_$name
}
tr vgg11dp "NITI_RC_SPEC2=1" --steps 5 --warmup 3 --dp-path &&
tr vgg11dp_off "NITI_RC_SPEC2=0" --steps 5 --warmup 3 --dp-path &&
tr vgg16 "NITI_RC_SPEC2=1" --arch vgg16 --steps 3 --warmup 2 --no-autotune
