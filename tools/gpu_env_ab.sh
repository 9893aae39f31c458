#!/bin/bash
# Alternating runs of `ENV python3 bench.py ARGS` over the environment settings ENVS (one box,
# ROUNDS passes; "-" = none), ms per step and the speculative-pair counters printed per run.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-env}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for e in ${ENVS:?}; do
    log=gpurun_out/${TAG}_${e//=/_}_$r.log
    if [ "$e" = "-" ]; then e=""; fi
    env $e timeout -k 10 300 python3 bench.py ${ARGS:?} > "$log" 2>&1
    rc=$?
    echo "${e:-default} $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$log") $(grep -o '"redone": [0-9]*, "stored_or_alternate": [0-9]*' "$log")"
    [ $rc -eq 0 ] || exit $rc
  done
done
