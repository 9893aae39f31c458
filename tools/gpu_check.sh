set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== rocminfo"; rocminfo 2>/dev/null | grep -E "gfx950|Compute Unit" | head -4
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_r01a.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu_r01a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_r01a.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_r01a.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof_last
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_last" -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_last.log 2>&1
  rc=$?; echo "prof rc=$rc"
fi
exit $rc
