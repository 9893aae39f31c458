# A/B: weight-gradient stream priority (NITI_DIAG_SIDE_PRIORITY) on the default bench
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for p in 0 -1 1 0 -1; do
  NITI_DIAG_SIDE_PRIORITY=$p timeout -k 10 200 python3 bench.py --cpu-sample 0 > gpurun_out/prio_$p.log 2>&1 || exit 1
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/prio_$p.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('prio $p', d['ms_per_step'], d['value'], 'wgrad', r['avg_launch_us'], r['frac'], 'iso', r['isolated']['avg_launch_us'])"
done
