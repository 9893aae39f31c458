set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="st_nt" SPLITS=8 bash tools/gpu_stamps.sh || exit 1
for v in base nt; do
  if [ $v = base ]; then unset NITI_HIP_LIB; else export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so; fi
  rm -rf gpurun_out/ts_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ts_$v" -o run -- python3 tools/wgrad_sweep.py --layer ${LAYER:-3} --splits 8 > gpurun_out/ts_$v.log 2>&1
  rc=$?; echo "== $v sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/sweep_summary.py $(find gpurun_out/ts_$v -name "*kernel_trace.csv" | head -1) | grep -v at::native
done
