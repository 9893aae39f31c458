# A/B of the P16 weight-gradient prologue / K-loop variants (tools/wg_diag_build.sh builds):
# stamps per variant, then launch timing of conv3/4/5 per variant (HIP events, wg_bench.py).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${STAMPED:-z0 z1 s2 s3}; do
  export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so
  timeout -k 10 120 python3 tools/wg_diag.py conv4 4 > gpurun_out/m_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; cat gpurun_out/m_$v.log | grep -v Warn; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
for v in ${TIMED:-tz0 tz1 ts2 ts3}; do
  export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so
  timeout -k 10 120 python3 tools/wg_bench.py conv3 conv4 conv5 conv6 > gpurun_out/mt_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; cat gpurun_out/mt_$v.log | grep -v Warn; [ $rc -eq 0 ] || exit $rc
done
done
