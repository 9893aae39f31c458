# PMC counters of the tap-sharing wgrad kernel (L3, 8 splits), one pass per counter group.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" ${EXTRA_PMC:-}; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_taps_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_taps_$i" -o run -- python3 tools/wgrad_sweep.py --layer ${LAYER:-3} --splits ${SPLITS:-8} --reps 5 > gpurun_out/pmc_taps_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/pmc_taps_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'wgrad_taps' in r['Kernel_Name'] or 'gemm_kernel' in r['Kernel_Name']]
d = collections.defaultdict(list)
for r in rows:
    d[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in d.items():
    v.sort()
    print(f"  {k:28s} median {v[len(v)//2]:.4g}  (n={len(v)})")
PY
done
