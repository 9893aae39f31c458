# P16 weight gradient: parity tests, timing, then the stamp / ablation report.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-wg}
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_p16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/wg_tests_$TAG.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wg_bench.py > gpurun_out/wg_bench_$TAG.log 2>&1
rc=$?; cat gpurun_out/wg_bench_$TAG.log | cut -c1-250; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-st}" bash tools/wg_diag.sh
