#!/bin/bash
# Alternating A/B runs of one bench command on one box (the round-4 one-off scripts folded into
# one): ROUNDS pairs of `ENV_A python3 bench.py ARGS` / `ENV_B python3 bench.py ARGS`, each under
# its own time limit, ms per step printed per run.  Example:
#   ENV_A="NITI_RC_SPEC2=1" ENV_B="NITI_RC_SPEC2=0" ARGS="--arch vgg16 --steps 4 --warmup 2" bash tools/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-ab}
ROUNDS=${ROUNDS:-3}
ARGS=${ARGS:---cpu-sample 0}
for r in $(seq 1 "$ROUNDS"); do
  for side in A B; do
    envs=$([ $side = A ] && echo "${ENV_A:-}" || echo "${ENV_B:-}")
    log=gpurun_out/${TAG}_${side}_$r.log
    env $envs timeout -k 10 300 python3 bench.py $ARGS > "$log" 2>&1
    rc=$?
    echo "$side $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$log")"
    [ $rc -eq 0 ] || exit $rc
  done
done
