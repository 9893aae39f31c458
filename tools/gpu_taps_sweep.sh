# Kernel-trace sweeps of the L3 weight gradient: tap-sharing kernel (base + ablations) and the generic GEMM.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name lib args
  local name=$1 lib=$2; shift 2
  if [ "$lib" = "base" ]; then unset NITI_HIP_LIB; else export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$lib/libniti_hip.so; fi
  rm -rf gpurun_out/ts_$name
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ts_$name" -o run -- python3 tools/wgrad_sweep.py "$@" > gpurun_out/ts_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"
  [ $rc -eq 0 ] || return $rc
  f=$(find gpurun_out/ts_$name -name "*kernel_trace.csv" | head -1)
  python3 tools/sweep_summary.py "$f"
}
L=${LAYER:-3}
run taps base --layer $L --splits ${SPLITS:-2,4,8,16} && \
run abl1 abl1 --layer $L --splits 8 && \
run abl2 abl2 --layer $L --splits 8 && \
run generic base --layer $L --splits 4,7,12 --notaps
