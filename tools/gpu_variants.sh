# Per-variant GEMM sweeps (tools/wgrad_sweep.py under rocprofv3) and benches for the variant
# libraries named in VARIANTS (tools/ablate/<name>; "base" = the in-tree library).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = "base" ]; then unset NITI_HIP_LIB; else export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so; fi
  rm -rf gpurun_out/sw_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sw_$v" -o run -- python3 tools/wgrad_sweep.py ${SWEEP_ARGS:-} > gpurun_out/sw_$v.log 2>&1
  rc=$?; echo "== $v sweep rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/sw_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/sweep_summary.py "$f" | grep gemm_kernel
  if [ "${BENCH:-1}" = "1" ]; then
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/bench_$v.log 2>&1
    rc=$?; echo "bench rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/bench_$v.log | tr '\n' ' '; echo
    [ $rc -eq 0 ] || exit $rc
  fi
done
