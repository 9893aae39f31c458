# first-layer store / fused quantiser change: parity (model steps from int8 and images, b256, DP), bench, trace.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_b256.py tests/test_quant.py tests/test_dp_local.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_k.log 2>&1
rc=$?; tail -2 gpurun_out/t_k.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_k.log | head; exit $rc; }
timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/bench_k.log 2>&1
rc=$?; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'], r['plan'])" gpurun_out/bench_k.log; [ $rc -eq 0 ] || exit $rc
TAG=r02k bash tools/gpu_trace.sh > /dev/null 2>&1; echo trace rc=$?
