# Fused P16 dy (requant_act out_p16): the step parity tests, then bench A/B against the separate
# conversion (NITI_P16_SEPARATE=1), alternating.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_dp_local.py tests/test_gpu_b256.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1
rc=$?; tail -4 gpurun_out/n_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sep in 0 1; do
    NITI_P16_SEPARATE=$sep timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/n_bench_${sep}_$rep.json 2> gpurun_out/n_bench_${sep}_$rep.err
    rc=$?; echo "sep=$sep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/n_bench_${sep}_$rep.err; exit $rc; }
    python -c "import json,sys; d=json.load(open('gpurun_out/n_bench_${sep}_$rep.json')); r=d['roofline']; print('sep', $sep, d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], r['isolated']['frac'])"
  done
done
