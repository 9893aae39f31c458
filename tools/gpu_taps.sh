# Tap-sharing wgrad iteration: its parity tests first, then the full GPU suite, GEMM timings, bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider -k "taps or wgrad" --timeout 120 --timeout-method thread > gpurun_out/pytest_taps.log 2>&1
rc=$?; echo "pytest taps rc=$rc"; tail -15 gpurun_out/pytest_taps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest all rc=$rc"; tail -4 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_taps.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_taps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/bench_taps.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_taps.log | cut -c1-1500
exit $rc
