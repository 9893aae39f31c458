#!/bin/bash
# Kernel traces of `bench.py ARGS` under the in-tree build and diagnostic variants
# (tools/ablate/<name>/libniti_hip.so), summarised per step; GREP selects the lines printed.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-vt}
for v in base ${VARIANTS:?}; do
  if [ "$v" = base ]; then lib=""; else lib="tools/ablate/$v/libniti_hip.so"; fi
  d=gpurun_out/tr_${TAG}_$v
  rm -rf $d
  NITI_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$d" -o run -- python3 bench.py ${ARGS:?} > $d.log 2>&1
  rc=$?; echo "$v trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$f" 5 > ${d}_steps.txt
  grep -E "${GREP:-busy}" ${d}_steps.txt | head -8
done
