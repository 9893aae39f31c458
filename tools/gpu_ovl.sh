# Overlap policy A/B on the default bench (autotuned): side stream default / high / low priority, no overlap.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
show() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['isolated']['avg_launch_us'], r['plan'])" $1 "$2"; }
for V in ${OVL_VARIANTS:-"def::" "noov::--no-overlap"}; do
  name=${V%%:*}; rest=${V#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python3 bench.py --cpu-sample 0 $args > gpurun_out/ovl_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/ovl_$name.log; exit $rc; }
  show gpurun_out/ovl_$name.log $name
done
