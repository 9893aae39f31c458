# A/B of two weight-gradient builds on one box: stamps (old vs st) and the bench step (oldns vs main) x2.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPLITS=4 LAYERS=conv4 VARIANTS="old st old st" bash tools/wg_diag.sh || exit 1
main=$GRAFT_REPO_ROOT/mandheling-dsp-training_amd/niti_amd/_lib/libniti_hip.so
for v in oldns main oldns main; do
  if [ $v = main ]; then export NITI_HIP_LIB=$main; else export NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so; fi
  timeout -k 10 300 python3 bench.py --cpu-sample 0 > gpurun_out/bench_ab_$v.log 2>&1
  rc=$?; echo -n "$v: "; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'])" gpurun_out/bench_ab_$v.log; [ $rc -eq 0 ] || exit $rc
done
