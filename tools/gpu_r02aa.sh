# SGD with the range read once per job: step / op tests, then VGG-11 and VGG-16 bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py tests/test_gpu_b256.py tests/test_dp_local.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/aa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/aa_tests.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/aa11_$rep.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --arch vgg16 --steps 10 --warmup 3 > gpurun_out/aa16_$rep.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json; a=json.load(open('gpurun_out/aa11_$rep.json')); b=json.load(open('gpurun_out/aa16_$rep.json')); print(a['value'], a['ms_per_step'], a['roofline']['frac'], b['value'], b['ms_per_step'])"
done
