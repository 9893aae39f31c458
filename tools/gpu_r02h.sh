# conv0 + merge changes: model parity, P16 parity, stamps (merge 1 vs 0), bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad_p16.py tests/test_gpu_model.py tests/test_gpu_b256.py tests/test_quant.py tests/test_dp_local.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1
rc=$?; tail -3 gpurun_out/t_h.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_h.log | head; exit $rc; }
SPLITS=4 LAYERS=conv4 VARIANTS="st m0" bash tools/wg_diag.sh || exit 1
timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/bench_h.log 2>&1
rc=$?; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'], r['plan'])" gpurun_out/bench_h.log; exit $rc
