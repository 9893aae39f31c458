# rocprofv3 kernel trace of a short bench run + per-step breakdown (tools/prof_summary.py)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-trace}
ARGS=${ARGS:-}
rm -rf gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_$TAG" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 $ARGS > gpurun_out/tr_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/tr_$TAG.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/tr_${TAG}_breakdown.txt
head -45 gpurun_out/tr_${TAG}_breakdown.txt
