# Round-4 check on the GPU box: the GPU suite (one runner, per-test timeout), smoke(), then the
# default bench and A/B of the row kernels' speculative epilogue and XCD tile order.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
# A/B, alternating: all on; speculation off; side SGD off; NHWC16 dy kept
for rep in 1 2; do
  for v in "on:" "spec0:--rc-spec 0" "side0:NITI_SIDE_SGD=0" "dy16:NITI_DY16=1"; do
    name=${v%%:*}; opt=${v#*:}; envs=""; flags=""
    case "$opt" in *=*) envs=$opt;; *) flags=$opt;; esac
    env $envs timeout -k 10 300 python3 bench.py --cpu-sample 0 $flags > gpurun_out/bench_${TAG}_$name.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$name.log; exit $rc; }
    echo "$name rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}_$name.log)"
  done
done
for m in x w; do
  for d in "" "--dgrad fused"; do
    NITI_RC_MAP=$m timeout -k 10 120 python3 tools/rowconv_bench.py --modes 0 $d >> gpurun_out/rcb_${TAG}_$m.log 2>&1 || exit 1
  done
  echo "== map $m"; grep -v amdgpu.ids gpurun_out/rcb_${TAG}_$m.log
done
