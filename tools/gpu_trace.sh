# Kernel trace of a short default bench run (autotuned, overlapped) -> last-step timeline.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-trace}
rm -rf gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/prof_$TAG.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/trace_$TAG.txt
tail -120 gpurun_out/trace_$TAG.txt
