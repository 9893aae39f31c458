# Per-layer input P16 validity (isolated re-runs without the input conversion): step tests, two bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_dp_local.py tests/test_gpu_b256.py tests/test_gpu_wgrad_p16.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v_tests.log 2>&1
rc=$?; tail -2 gpurun_out/v_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/v_bench_$rep.json 2> gpurun_out/v_bench_$rep.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/v_bench_$rep.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/v_bench_$rep.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], r['in_kernel_span_us'], r['isolated']['frac'], r['isolated']['avg_launch_us'], r['isolated']['in_kernel_span_us'])"
done
