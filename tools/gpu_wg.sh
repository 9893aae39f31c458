# P16 weight-gradient kernel: parity tests, event timing, rocprofv3 kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-wg}
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_p16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg_tests_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/wg_tests_$TAG.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wg_bench.py > gpurun_out/wg_bench_$TAG.log 2>&1
rc=$?; cat gpurun_out/wg_bench_$TAG.log; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/wgprof_$TAG" -o run -- python3 tools/wg_bench.py conv4 > gpurun_out/wg_prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; find gpurun_out/wgprof_$TAG -name "*kernel_stats.csv" -exec cut -c1-200 {} \;
exit $rc
