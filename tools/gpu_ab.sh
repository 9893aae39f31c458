set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cpu-sample 0 $ARGS_A > gpurun_out/ab_a.log 2>&1 || exit 1
echo "A($ARGS_A): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_a.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab_a.log)"
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cpu-sample 0 $ARGS_B > gpurun_out/ab_b.log 2>&1 || exit 1
echo "B($ARGS_B): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_b.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab_b.log)"
done
