# Round deliverables on the GPU box: default bench (with CPU baseline), rocprofv3 kernel stats of
# the same command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 400 python3 bench.py --save-plans gpurun_out/plans_$TAG.json > gpurun_out/bench_full_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench_full_$TAG.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_$TAG gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG
# the profiled and counted runs replay the plans the timed run autotuned to (same launch sequence)
PLAN="--load-plans gpurun_out/plans_$TAG.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --cpu-sample 0 $PLAN > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/prof_$TAG.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcF_$TAG" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 $PLAN > gpurun_out/pmcF_$TAG.log 2>&1
rc=$?; echo "pmcF rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcW_$TAG" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 $PLAN > gpurun_out/pmcW_$TAG.log 2>&1
rc=$?; echo "pmcW rc=$rc"
exit $rc
