# Stamp / ablation report of the P16 weight-gradient kernel (builds from tools/wg_diag_build.sh).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${VARIANTS:-st}; do
  export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so
  for L in ${LAYERS:-conv4 conv6}; do
    timeout -k 10 120 python3 tools/wg_diag.py $L ${SPLITS:-1,4} > gpurun_out/wgd_${v}_$L.log 2>&1
    rc=$?; echo "== $v rc=$rc"; grep splits gpurun_out/wgd_${v}_$L.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/wgd_${v}_$L.log; exit $rc; }
  done
done
