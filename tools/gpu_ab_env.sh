# A/B of an environment switch: per-op GEMM timing and the bench, with and without $ENVAB
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 0 1 0 1; do
  env $ENVAB=$v timeout -k 10 120 python3 tools/gemm_bench.py --only ${ONLY:-2,3,4,5} --reps 20 > gpurun_out/abenv_$v.log 2>&1 || exit 1
  env $ENVAB=$v timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/abenvb_$v.log 2>&1 || exit 1
  echo "$ENVAB=$v $(grep -E '^L' gpurun_out/abenv_$v.log | awk '{print $1,$2,$(NF-4)}' | tr '\n' '|') step $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abenvb_$v.log)"
done
