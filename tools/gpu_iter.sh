# One iteration of the GPU loop: parity tests, per-op GEMM timings, default bench (x2).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_iter.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_iter.log
[ $rc -eq 0 ] || exit $rc
if [ "${GEMM:-1}" = "1" ]; then
  timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_iter.log 2>&1
  rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gemm_iter.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_iter.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
