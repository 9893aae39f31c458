# GPU tests, then per-op GEMM timing and a short bench (no profiler)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/gemm_bench.py --reps 20 > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench.log | cut -c1-400
exit $rc
