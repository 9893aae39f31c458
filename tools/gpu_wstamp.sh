# per-wave stamps of the P16 weight gradient (conv4, conv6 at split 4)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/st/libniti_hip.so
for L in conv4 conv6 conv4; do
  timeout -k 10 120 python3 tools/wg_diag.py $L 4 > gpurun_out/wgw_$L.log 2>&1
  rc=$?; cat gpurun_out/wgw_$L.log | grep -v "^$" | tail -3; [ $rc -eq 0 ] || exit $rc
done
