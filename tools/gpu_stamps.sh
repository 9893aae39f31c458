# Stamp reports (diagnostic NITI_STAMPS builds) of the tap-sharing wgrad kernel.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-stamps stamps_abl1}; do
  export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so
  timeout -k 10 120 python3 tools/wgrad_sweep.py --layer ${LAYER:-3} --splits ${SPLITS:-2,8} --reps 3 > gpurun_out/st_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep "taps stamps" gpurun_out/st_$v.log | sort | uniq -c | sort -rn | head -8
  [ $rc -eq 0 ] || exit $rc
done
