#!/bin/bash
# Diagnostic library variants (tools/ablate/<name>/libniti_hip.so, tools/stages_build.sh) against the
# in-tree build on one box: ROUNDS passes over "base VARIANTS...", `bench.py ARGS` each (fixed plans
# in ARGS keep the launch sequence the same), ms per step printed per run.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-var}
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  for v in base ${VARIANTS:?}; do
    log=gpurun_out/${TAG}_${v}_$r.log
    if [ "$v" = base ]; then lib=""; else lib="tools/ablate/$v/libniti_hip.so"; fi
    NITI_HIP_LIB=$lib timeout -k 10 300 python3 bench.py ${ARGS:?} > "$log" 2>&1
    rc=$?
    echo "$v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$log")"
    [ $rc -eq 0 ] || exit $rc
  done
done
