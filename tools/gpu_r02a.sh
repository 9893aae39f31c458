set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_b256.py -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/b256.log 2>&1
rc=$?; tail -40 gpurun_out/b256.log | cut -c1-400; echo "b256 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r02a.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_r02a.log; exit $rc
