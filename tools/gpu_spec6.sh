#!/bin/bash
# Scale-compensated speculative hints (round 6): the pair / residual / whole-step parity tests, the
# residual pass probe, then ResNet-18 and VGG-16 bench lines (launches B redid: rowconv_spec).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-s6}
timeout -k 10 900 python -u -m pytest tests/test_gpu_rowconv.py tests/test_gpu_residual_ops.py tests/test_gpu_resnet_cpp.py tests/test_gpu_cfg45.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/spec6_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/spec6_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 60 tools/probes/exit_probe > gpurun_out/exit_probe3.txt 2>&1 || exit $?
grep "grid  2048" gpurun_out/exit_probe3.txt
for net in resnet18 vgg16; do
  timeout -k 10 400 python3 bench.py --arch $net --cpu-sample 0 --load-plans tools/probes/plans_${net}_r06.json > gpurun_out/spec6_${net}_$TAG.log 2>&1 || exit $?
  echo "$net $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/spec6_${net}_$TAG.log) $(grep -o '"rowconv_spec": {[^}]*}' gpurun_out/spec6_${net}_$TAG.log)"
done
timeout -k 10 300 python3 tools/spec_trace.py --arch resnet18 --load-plans tools/probes/plans_resnet18_r06.json > gpurun_out/spec_trace_r18_$TAG.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --dp-path --cpu-sample 0 > gpurun_out/spec6_dppath_$TAG.log 2>&1 || exit $?
echo "vgg11 dp-path $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/spec6_dppath_$TAG.log) $(grep -o '"rowconv_spec": {"redone": [0-9]*, "stored_or_alternate": [0-9]*' gpurun_out/spec6_dppath_$TAG.log)"
timeout -k 10 300 python3 tools/spec_trace.py --arch vgg16 --load-plans tools/probes/plans_vgg16_r06.json > gpurun_out/spec_trace_v16_$TAG.txt 2>&1 || exit $?
