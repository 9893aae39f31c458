set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep metric gpurun_out/prof_$TAG.log | cut -c1-300
exit $rc
