# ResNet-18 data-parallel parity (threaded ranks on one device), then the fused-P16 profile A/B.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/p_tests.log 2>&1
rc=$?; tail -6 gpurun_out/p_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r02o.sh
