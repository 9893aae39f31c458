#!/bin/bash
# Round-4: the speculative pair with store-mode hysteresis -- model / DP tests, VGG-11 --dp-path A/B.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04w}
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_dp_local.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
b() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" --cpu-sample 0 > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${name}_$TAG.log) $(grep -o '"rowconv_spec": {"redone": [0-9]*, "stored": [0-9]*' gpurun_out/${name}_$TAG.log)"; return $rc
}
b vgg11dp "NITI_RC_SPEC2=1" --steps 30 --warmup 5 --dp-path &&
b vgg11dp_off "NITI_RC_SPEC2=0" --steps 30 --warmup 5 --dp-path &&
b vgg11dp2 "NITI_RC_SPEC2=1" --steps 30 --warmup 5 --dp-path &&
b vgg11dp_off2 "NITI_RC_SPEC2=0" --steps 30 --warmup 5 --dp-path
