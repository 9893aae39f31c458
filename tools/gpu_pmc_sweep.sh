# PMC passes (one rocprofv3 run each, kernel trace + counters only) over tools/wgrad_sweep.py.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
while read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1))
  rm -rf gpurun_out/pmcs$i
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcs$i" -o run -- python3 tools/wgrad_sweep.py ${SWEEP_ARGS:-} > gpurun_out/pmcs$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc ($P)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcs$i.log; exit $rc; }
  python3 tools/pmc_summary.py gpurun_out/pmcs$i
done <<< "${PASSES}"
