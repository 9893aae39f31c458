set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for s in 2 4 7 9 14 18; do
  NITI_DIAG_SPLITS=$s timeout -k 10 120 python3 tools/gemm_bench.py --only ${ONLY:-3} --reps 20 > gpurun_out/splits_$s.log 2>&1 || exit 1
  echo "splits=$s $(grep -E '^L' gpurun_out/splits_$s.log | tr '\n' '|')"
done
