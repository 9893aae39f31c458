# Two-pass max-pool gradient: op tests, ResNet tests, ResNet bench + kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/w_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r02s.sh
