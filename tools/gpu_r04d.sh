#!/bin/bash
# Round-4: kernel traces of the VGG-16 / ResNet-18 steps with and without the row-segment form
# (NITI_SEG_MAX_CIN=0 turns it off), to find where the whole step loses what the per-layer bench gains.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04d}
for v in "seg:" "noseg:NITI_SEG_MAX_CIN=0"; do
  name=${v%%:*}; envs=${v#*:}
  for arch in vgg16 resnet18; do
    rm -rf gpurun_out/tr_${TAG}_${arch}_$name
    [ -n "$envs" ] && export $envs
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_${arch}_$name" -o run -- python3 bench.py --arch $arch --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/tr_${TAG}_${arch}_$name.log 2>&1
    rc=$?; echo "$arch $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_${TAG}_${arch}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tr_${TAG}_${arch}_$name.log; exit $rc; }
    f=$(find gpurun_out/tr_${TAG}_${arch}_$name -name "*kernel_trace.csv" | head -1)
    python3 tools/prof_summary.py "$f" 7 > gpurun_out/tr_${TAG}_${arch}_${name}_breakdown.txt
    rm -rf gpurun_out/tr_${TAG}_${arch}_$name
  done
  unset NITI_SEG_MAX_CIN
done
