#!/bin/bash
# Same-box A/B of this round's build against the round's starting commit (29c2e06, built in the
# worktree tools/ablate/base): VGG-11 bench, its data-parallel kernel path, ResNet-18 and VGG-16
# (each with the plan set it autotunes), alternating.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/base_ab.txt
: > $OUT
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 400 python3 bench.py --cpu-sample 0 "$@") > gpurun_out/base_ab_$tag.log 2>&1 || return $?
  echo "$tag $* $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/base_ab_$tag.log) $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/base_ab_$tag.log)" >> $OUT
}
for rep in 1 2; do
  for v in new base; do
    d=.; [ $v = base ] && d=tools/ablate/base
    run ${v}_vgg11_$rep $d || exit $?
    run ${v}_dp_$rep $d --dp-path || exit $?
    run ${v}_r18_$rep $d --arch resnet18 || exit $?
    run ${v}_v16_$rep $d --arch vgg16 || exit $?
  done
done
cat $OUT
