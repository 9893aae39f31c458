# rocprofv3 kernel trace of tools/wgrad_sweep.py (args in SWEEP_ARGS) -> per-grid medians
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/sweep2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sweep2" -o run -- python3 tools/wgrad_sweep.py ${SWEEP_ARGS:-} > gpurun_out/sweep2.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/sweep2.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/sweep2 -name "*kernel_trace.csv" | head -1)
python3 tools/sweep_summary.py "$f"
