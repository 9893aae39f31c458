#!/bin/bash
# Alternating runs of `bench.py ARGS --load-plans F` over the plan files PLANS (one box, ROUNDS
# passes), ms per step printed per run: plan choices compared under identical conditions.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-pl}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for f in ${PLANS:?}; do
    log=gpurun_out/${TAG}_$(basename "$f" .json)_$r.log
    timeout -k 10 300 python3 bench.py ${ARGS:?} --load-plans "$f" > "$log" 2>&1
    rc=$?
    echo "$(basename "$f") $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$log")"
    [ $rc -eq 0 ] || exit $rc
  done
done
