# Fused P16 dy, plain pass at 4 rows per thread: step parity, bench A/B, then a kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_dp_local.py tests/test_gpu_b256.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/q_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sep in 0 1; do
    NITI_P16_SEPARATE=$sep timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/q_bench_${sep}_$rep.json 2> gpurun_out/q_bench_${sep}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/q_bench_${sep}_$rep.err; exit $rc; }
    python -c "import json,sys; d=json.load(open('gpurun_out/q_bench_${sep}_$rep.json')); r=d['roofline']; print('sep', $sep, d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], r['isolated']['frac'])"
  done
done
rm -rf gpurun_out/q_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/q_prof" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 > gpurun_out/q_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/q_prof -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py $f 13 > gpurun_out/q_sum.txt
