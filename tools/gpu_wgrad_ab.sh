# A/B of tap-sharing weight-gradient variants (tools/ablate/<v>): rocprofv3 kernel stats per
# (variant, split count) on VGG-11 conv4 at batch 256.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-base prio sc1 nt}; do
  for sp in ${SPLITS:-6 8}; do
    d=gpurun_out/ab_${v}_$sp; rm -rf $d
    NITI_HIP_LIB=$GRAFT_REPO_ROOT/tools/ablate/$v/libniti_hip.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/wgrad_sweep.py --layer ${LAYER:-3} --splits $sp --reps 30 > $d.log 2>&1 || { echo "fail $v $sp"; tail -5 $d.log; exit 1; }
    python3 - "$d" "$v" "$sp" <<'PY'
import csv, glob, sys
d, v, sp = sys.argv[1:4]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "wgrad_taps" in r["Name"] or "splitk_reduce" in r["Name"]:
        print(f"{v:6s} splits {sp}: {r['Name'][:40]:40s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:7.2f} us")
PY
  done
done
