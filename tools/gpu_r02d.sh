# P16 in-step A/B: model parity tests, default bench vs forced P16 plans, kernel trace of the P16 step.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02d}
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad_p16.py tests/test_gpu_model.py tests/test_gpu_b256.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/t_$TAG.log | cut -c1-600; echo "tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_$TAG.log; exit $rc; }
for V in -1 0; do
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --wgrad-p16 $V > gpurun_out/bench_${TAG}_$V.log 2>&1
  rc=$?; echo "bench p16=$V rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'], r['plan'])" gpurun_out/bench_${TAG}_$V.log
done
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --wgrad-p16 0 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/trace_$TAG.txt
grep "step span" gpurun_out/trace_$TAG.txt
