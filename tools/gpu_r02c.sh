# P16 kernel tests + model parity (incl. batch-256 full parity) + default bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-r02c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad_p16.py tests/test_gpu_model.py tests/test_gpu_b256.py tests/test_quant.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error|autotuned plans" gpurun_out/t_$TAG.log | cut -c1-600; echo "tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_$TAG.log; exit $rc; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_$TAG.log | cut -c1-1500; exit $rc
