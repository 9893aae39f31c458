# P16 kernel change: P16 parity, b256 step parity, stamps, bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad_p16.py tests/test_gpu_b256.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_l.log 2>&1
rc=$?; tail -2 gpurun_out/t_l.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_l.log | head; exit $rc; }
SPLITS=4 LAYERS=conv4 VARIANTS="st" bash tools/wg_diag.sh || exit 1
timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/bench_l.log 2>&1
rc=$?; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'], r['plan'])" gpurun_out/bench_l.log; exit $rc
