# Kernel-trace sweep of wgrad_taps_kernel pipeline depth (tools/stages_build.sh variants) over VGG-11 layers.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base ${VARIANTS:-s6 s8}; do
  if [ "$lib" = "base" ]; then unset NITI_HIP_LIB; else export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$lib/libniti_hip.so; fi
  for L in ${LAYERS:-1 2 3 4 5 6}; do
    rm -rf gpurun_out/st_${lib}_$L
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/st_${lib}_$L" -o run -- python3 tools/wgrad_sweep.py --layer $L --splits ${SPLITS:-4,8,16} > gpurun_out/st_${lib}_$L.log 2>&1
    rc=$?; echo "== $lib layer $L rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    f=$(find gpurun_out/st_${lib}_$L -name "*kernel_trace.csv" | head -1)
    python3 tools/sweep_summary.py "$f" | grep -v "randint\|elementwise\|fill"
  done
done
