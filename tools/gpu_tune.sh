# tests + A/B of the autotuned plans against the fixed defaults (bench.py, VGG-11 b256)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_tune.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu_tune.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for flag in "" "--no-overlap" "--no-autotune" ""; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 0 $flag > gpurun_out/bench_tune.log 2>&1
  rc=$?; echo "bench [$flag] rc=$rc"; tail -2 gpurun_out/bench_tune.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
