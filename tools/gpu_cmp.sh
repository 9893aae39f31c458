# default vs --no-overlap bench, then a kernel trace of the default run (last-step timeline)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "" "--no-overlap"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 0 $a > gpurun_out/bench_cmp.log 2>&1
  rc=$?; echo "bench [$a] rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*\|"plan": {[^}]*}' gpurun_out/bench_cmp.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
TAG=cmp BENCH_ARGS="${TRACE_ARGS:-}" bash tools/gpu_trace.sh > gpurun_out/trace_cmp_stdout.txt 2>&1
rc=$?; echo "trace rc=$rc"; head -40 gpurun_out/trace_cmp.txt
